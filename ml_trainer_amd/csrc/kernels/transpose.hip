// bf16 matrix transpose dst[C][R] = src[R][C] (the k-contiguous W^T copies of the input-gradient
// GEMMs, ops/transformer.py bf16_weight_t). 64x64 tiles through LDS: 16-byte row loads, a
// padded LDS image (65 shorts per row: the column reads of the transposed write hit distinct
// banks), 8-byte row stores of the transposed tile. Edges are guarded element-wise.
#include "mlt_common.h"
#include "mlt_kernels.h"

namespace mlt {

constexpr int kTT = 64;

__global__ __launch_bounds__(256) void transpose_bf16_kernel(const uint16_t* __restrict__ src,
                                                             uint16_t* __restrict__ dst, int R, int C,
                                                             int src_al16, int dst_al8) {
  __shared__ uint16_t tile[kTT][kTT + 1];
  const int tiles_c = (C + kTT - 1) / kTT;
  const int r0 = (blockIdx.x / tiles_c) * kTT, c0 = (blockIdx.x % tiles_c) * kTT;
  const int t = threadIdx.x;
  const bool vec = src_al16 && (C % 8 == 0) && c0 + kTT <= C;
  // load: 64 rows x 8 chunks of 8 elements; 256 threads -> 2 chunks each
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = t + 256 * i, r = e >> 3, ch = e & 7;
    const int gr = r0 + r;
    if (gr < R) {
      if (vec) {
        const uint4 v = *reinterpret_cast<const uint4*>(src + (int64_t)gr * C + c0 + ch * 8);
        const uint16_t* pv = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
        for (int j = 0; j < 8; ++j) tile[r][ch * 8 + j] = pv[j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int gc = c0 + ch * 8 + j;
          tile[r][ch * 8 + j] = gc < C ? src[(int64_t)gr * C + gc] : 0;
        }
      }
    }
  }
  __syncthreads();
  // store: dst row = source column c0 + c (64 rows), 16 chunks of 4 elements per row
  const bool vst = dst_al8 && (R % 4 == 0) && r0 + kTT <= R;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = t + 256 * i, c = e >> 4, q = e & 15;
    const int gc = c0 + c;
    if (gc >= C) continue;
    ushort4 o;
    o.x = tile[q * 4 + 0][c];
    o.y = tile[q * 4 + 1][c];
    o.z = tile[q * 4 + 2][c];
    o.w = tile[q * 4 + 3][c];
    uint16_t* dp = dst + (int64_t)gc * R + r0 + q * 4;
    if (vst) {
      *reinterpret_cast<ushort4*>(dp) = o;
    } else {
      const uint16_t vals[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (r0 + q * 4 + j < R) dp[j] = vals[j];
    }
  }
}

void launch_transpose_bf16(const uint16_t* src, uint16_t* dst, int R, int C, hipStream_t st) {
  if (R <= 0 || C <= 0) return;
  const int64_t tiles = (int64_t)((R + kTT - 1) / kTT) * ((C + kTT - 1) / kTT);
  // (flat-buffer weight views are only 8-byte aligned: the 16-byte row loads need an aligned base)
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3((unsigned)tiles), dim3(256), 0, st, src, dst, R, C,
                     (int)(((uintptr_t)src % 16) == 0), (int)(((uintptr_t)dst % 8) == 0));
}

}  // namespace mlt
