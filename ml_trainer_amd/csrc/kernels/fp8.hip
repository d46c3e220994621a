// FP8 (OCP e4m3 / e5m2 -- gfx950 is OCP, not the MI300 fnuz variant) quantisation kernels for
// the fp8 GEMM path (BASELINE config 5, "large fp8"):
//   * cast_fp8: bf16 / fp32 -> fp8 with a per-tensor scale read from device memory, saturating,
//     recording amax(|x|) of the input for delayed scaling (one pass, 16-byte vector loads);
//   * cast_transpose_fp8: fp32 master weight [R,C] -> fp8 W [R,C] and W^T [C,R] in one pass
//     (64x64 tiles through LDS) -- forward uses W, dgrad uses W^T so both fp8 GEMM operands are
//     k-contiguous;
//   * amax: max |x| (exact current scaling when there is no history yet);
//   * update_scale: delayed scaling for n tensors at once -- push each amax into its history
//     window, scale = fmt_max / (max(history) * 2^margin), inv_scale = 1 / scale, reset amax.
// Conversions use v_cvt_pk_fp8_f32 / v_cvt_pk_bf8_f32 after clamping to the finite range.
#include "mlt_common.h"
#include "mlt_fp8.h"
#include "mlt_kernels.h"

namespace mlt {

__device__ __forceinline__ void load8(const uint16_t* p, float (&v)[8]) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = __uint_as_float(w[j] << 16);
    v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
  }
}
__device__ __forceinline__ void load8(const float* p, float (&v)[8]) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// y[i] = fp8(x[i] * scale); amax = max(amax, |x|). n % 8 == 0, 16-byte aligned.
template <typename InT, int FMT>
__global__ __launch_bounds__(256) void cast_fp8_kernel(const InT* __restrict__ x, uint8_t* __restrict__ y, int64_t n8,
                                                       const float* __restrict__ scale, float* __restrict__ amax) {
  __shared__ float red[4];
  const float s = *scale;
  float mx = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float v[8];
    load8(x + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) mx = fmaxf(mx, fabsf(v[j]));
    uint2 o;
    o.x = pack4_fp8<FMT>(v[0] * s, v[1] * s, v[2] * s, v[3] * s);
    o.y = pack4_fp8<FMT>(v[4] * s, v[5] * s, v[6] * s, v[7] * s);
    *reinterpret_cast<uint2*>(y + i * 8) = o;
  }
  if (amax) {
    mx = wave_max(mx);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) atomic_max_pos(amax, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
  }
}

template <typename InT>
__global__ __launch_bounds__(256) void amax_kernel(const InT* __restrict__ x, int64_t n8, float* __restrict__ amax) {
  __shared__ float red[4];
  float mx = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float v[8];
    load8(x + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) mx = fmaxf(mx, fabsf(v[j]));
  }
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) atomic_max_pos(amax, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
}

// fp32 W [R][C] -> fp8 W [R][C] and W^T [C][R]; 64x64 tile per block, R % 4 == 0, C % 4 == 0
__device__ __forceinline__ float4 load4f(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 load4f(const uint16_t* p) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xffff0000u));
}

// InT = float (master weights) or uint16_t (bf16 activations / gradients: the fp8 weight
// gradient needs X^T and dY^T with the token dimension contiguous)
template <int FMT, typename InT>
__global__ __launch_bounds__(256) void cast_transpose_fp8_kernel(const InT* __restrict__ w, uint8_t* __restrict__ y,
                                                                 uint8_t* __restrict__ yt, int R, int C,
                                                                 const float* __restrict__ scale,
                                                                 float* __restrict__ amax) {
  __shared__ uint8_t tile[64][68];
  __shared__ float red[4];
  const float s = *scale;
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  float mx = 0.f;
  // 64 rows x 16 float4 = 1024 items, 4 per thread
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int e = it * 256 + threadIdx.x, r = e >> 4, c4 = (e & 15) * 4;
    const int gr = r0 + r, gc = c0 + c4;
    uint32_t packed = 0;
    if (gr < R && gc < C) {
      const float4 v = load4f(w + (int64_t)gr * C + gc);
      mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
      packed = pack4_fp8<FMT>(v.x * s, v.y * s, v.z * s, v.w * s);
      *reinterpret_cast<uint32_t*>(y + (int64_t)gr * C + gc) = packed;
    }
    *reinterpret_cast<uint32_t*>(&tile[r][c4]) = packed;
  }
  __syncthreads();
  // transposed: row c of W^T = column c of the tile; 64 rows x 16 groups of 4 bytes
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int e = it * 256 + threadIdx.x, c = e >> 4, r4 = (e & 15) * 4;
    const int gc = c0 + c, gr = r0 + r4;
    if (gc < C && gr < R) {
      const uint32_t v = (uint32_t)tile[r4][c] | ((uint32_t)tile[r4 + 1][c] << 8) | ((uint32_t)tile[r4 + 2][c] << 16) |
                         ((uint32_t)tile[r4 + 3][c] << 24);
      *reinterpret_cast<uint32_t*>(yt + (int64_t)gc * R + gr) = v;
    }
  }
  if (amax) {
    mx = wave_max(mx);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) atomic_max_pos(amax, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
  }
}

// Activation / gradient variant (bf16 [R, C], R % 128 == 0, C % 128 == 0 -- checked by the
// launcher): 128 x 128 tiles, 8 x 16-byte loads in flight per thread, 8-byte y stores, and the
// transposed side read back from LDS as dwords (8 rows x 4 columns per thread, transposed in
// registers) so each wave's yt stores form 128-byte row segments instead of 64-byte ones.
// 33-dword LDS row stride: the 16 row groups of a wave's dword reads land on 2-way banks.
template <int FMT>
__global__ __launch_bounds__(256) void cast_transpose_fp8_wide_kernel(const uint16_t* __restrict__ x,
                                                                      uint8_t* __restrict__ y,
                                                                      uint8_t* __restrict__ yt, int R, int C,
                                                                      const float* __restrict__ scale,
                                                                      float* __restrict__ amax,
                                                                      float* __restrict__ colpart) {
  constexpr int S = 132;  // LDS row stride in bytes
  __shared__ uint32_t tile32[128 * S / 4];
  __shared__ float red[4];
  const float s = *scale;
  const int r0 = blockIdx.y * 128, c0 = blockIdx.x * 128;
  const int tid = threadIdx.x;
  float mx = 0.f;
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // column sums of x over this thread's 8 rows
  uint4 raw[8];
#pragma unroll
  for (int it = 0; it < 8; ++it) {  // item: row (it * 16 + tid / 16), 8 columns at (tid % 16) * 8
    const int r = it * 16 + (tid >> 4), c8 = (tid & 15) * 8;
    raw[it] = *reinterpret_cast<const uint4*>(x + (int64_t)(r0 + r) * C + c0 + c8);
  }
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int r = it * 16 + (tid >> 4), c8 = (tid & 15) * 8;
    const uint32_t w[4] = {raw[it].x, raw[it].y, raw[it].z, raw[it].w};
    float v[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[2 * j] = __uint_as_float(w[j] << 16);
      v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mx = fmaxf(mx, fabsf(v[j]));
      cs[j] += v[j];
    }
    const uint32_t lo = pack4_fp8<FMT>(v[0] * s, v[1] * s, v[2] * s, v[3] * s);
    const uint32_t hi = pack4_fp8<FMT>(v[4] * s, v[5] * s, v[6] * s, v[7] * s);
    *reinterpret_cast<uint2*>(y + (int64_t)(r0 + r) * C + c0 + c8) = make_uint2(lo, hi);
    tile32[(r * S + c8) / 4] = lo;
    tile32[(r * S + c8) / 4 + 1] = hi;
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 2; ++it) {  // item: 4 columns at c4 = (e / 16) * 4, 8 rows at r8 = (e % 16) * 8
    const int e = it * 256 + tid, c4 = (e >> 4) * 4, r8 = (e & 15) * 8;
    uint32_t d[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = tile32[((r8 + k) * S + c4) / 4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int sh = 8 * j;
      const uint32_t lo = ((d[0] >> sh) & 0xffu) | (((d[1] >> sh) & 0xffu) << 8) | (((d[2] >> sh) & 0xffu) << 16) |
                          (((d[3] >> sh) & 0xffu) << 24);
      const uint32_t hi = ((d[4] >> sh) & 0xffu) | (((d[5] >> sh) & 0xffu) << 8) | (((d[6] >> sh) & 0xffu) << 16) |
                          (((d[7] >> sh) & 0xffu) << 24);
      *reinterpret_cast<uint2*>(yt + (int64_t)(c0 + c4 + j) * R + r0 + r8) = make_uint2(lo, hi);
    }
  }
  if (colpart) {  // bias gradient of the GEMM whose dY this is: per-tile column sums, fixed order
    __syncthreads();  // the transposed reads of the tile are done; reuse it as [16][128] floats
    float* cp = reinterpret_cast<float*>(tile32);
    const int grp = tid >> 4, c8 = (tid & 15) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) cp[grp * 128 + c8 + j] = cs[j];
    __syncthreads();
    if (tid < 128) {
      float a = 0.f;
#pragma unroll
      for (int g2 = 0; g2 < 16; ++g2) a += cp[g2 * 128 + tid];
      colpart[(int64_t)blockIdx.y * C + c0 + tid] = a;
    }
  }
  if (amax) {
    mx = wave_max(mx);
    if ((tid & 63) == 0) red[tid >> 6] = mx;
    __syncthreads();
    if (tid == 0) atomic_max_pos(amax, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
  }
}

// Batched delayed scaling over n tensors: a = max over the amax slots of tensor i;
// hist[i][step % H] = a; scale[i] = fmax[i] / (max_h hist[i][h] * 2^margin);
// inv_scale[i] = 1 / scale[i]; slots reset to 0.
__global__ void update_scale_kernel(float* __restrict__ hist, int H, int n, float* __restrict__ amax,
                                    float* __restrict__ scale, float* __restrict__ inv_scale,
                                    const float* __restrict__ fmax, float margin_pow, int64_t step) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float* h = hist + (int64_t)i * H;
  float* sl = amax + (int64_t)i * kAmaxSlots * kAmaxStride;
  float a = 0.f;
  for (int k = 0; k < kAmaxSlots; ++k) {
    a = fmaxf(a, sl[k * kAmaxStride]);
    sl[k * kAmaxStride] = 0.f;
  }
  h[step % H] = a;
  float m = 0.f;
  for (int k = 0; k < H; ++k) m = fmaxf(m, h[k]);
  if (m > 0.f && isfinite(m)) {
    const float sc = fmax[i] / (m * margin_pow);
    scale[i] = sc;
    inv_scale[i] = 1.f / sc;
  }
}

static int grid_for(int64_t n8) {
  const int64_t b = (n8 + 255) / 256;
  return (int)(b < 2048 ? (b > 0 ? b : 1) : 2048);
}

void launch_cast_fp8(const void* x, bool x_f32, uint8_t* y, int64_t n, const float* scale, float* amax, int fmt,
                     hipStream_t st) {
  const int64_t n8 = n / 8;
  if (n8 <= 0) return;
  const dim3 g(grid_for(n8)), b(256);
  if (x_f32) {
    if (fmt == 0) hipLaunchKernelGGL((cast_fp8_kernel<float, 0>), g, b, 0, st, (const float*)x, y, n8, scale, amax);
    else hipLaunchKernelGGL((cast_fp8_kernel<float, 1>), g, b, 0, st, (const float*)x, y, n8, scale, amax);
  } else {
    if (fmt == 0) hipLaunchKernelGGL((cast_fp8_kernel<uint16_t, 0>), g, b, 0, st, (const uint16_t*)x, y, n8, scale, amax);
    else hipLaunchKernelGGL((cast_fp8_kernel<uint16_t, 1>), g, b, 0, st, (const uint16_t*)x, y, n8, scale, amax);
  }
}

void launch_amax(const void* x, bool x_f32, int64_t n, float* amax, hipStream_t st) {
  const int64_t n8 = n / 8;
  if (n8 <= 0) return;
  if (x_f32) hipLaunchKernelGGL((amax_kernel<float>), dim3(grid_for(n8)), dim3(256), 0, st, (const float*)x, n8, amax);
  else hipLaunchKernelGGL((amax_kernel<uint16_t>), dim3(grid_for(n8)), dim3(256), 0, st, (const uint16_t*)x, n8, amax);
}

void launch_cast_transpose_fp8(const float* w, uint8_t* y, uint8_t* yt, int R, int C, const float* scale, float* amax,
                               int fmt, hipStream_t st) {
  if (R <= 0 || C <= 0) return;
  const dim3 g((C + 63) / 64, (R + 63) / 64), b(256);
  if (fmt == 0) hipLaunchKernelGGL((cast_transpose_fp8_kernel<0, float>), g, b, 0, st, w, y, yt, R, C, scale, amax);
  else hipLaunchKernelGGL((cast_transpose_fp8_kernel<1, float>), g, b, 0, st, w, y, yt, R, C, scale, amax);
}

bool cast_transpose_fp8_wide_ok(const void* x, const void* y, const void* yt, int R, int C) {
  // MLT_FP8_CT_WIDE=0 keeps the 64x64 kernel (A/B knob)
  static const bool enabled = [] {
    const char* e = getenv("MLT_FP8_CT_WIDE");
    return !(e && e[0] == '0');
  }();
  return enabled && R > 0 && C > 0 && R % 128 == 0 && C % 128 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
         (reinterpret_cast<uintptr_t>(y) & 7) == 0 && (reinterpret_cast<uintptr_t>(yt) & 7) == 0;
}

// colpart: optional [R / 128, C] fp32 column partial sums of x -- only with the wide kernel
// (the caller checks cast_transpose_fp8_wide_ok first)
void launch_cast_transpose_fp8_bf16(const uint16_t* x, uint8_t* y, uint8_t* yt, int R, int C, const float* scale,
                                    float* amax, int fmt, hipStream_t st, float* colpart) {
  if (R <= 0 || C <= 0) return;
  if (cast_transpose_fp8_wide_ok(x, y, yt, R, C)) {
    const dim3 g(C / 128, R / 128), b(256);
    if (fmt == 0)
      hipLaunchKernelGGL((cast_transpose_fp8_wide_kernel<0>), g, b, 0, st, x, y, yt, R, C, scale, amax, colpart);
    else
      hipLaunchKernelGGL((cast_transpose_fp8_wide_kernel<1>), g, b, 0, st, x, y, yt, R, C, scale, amax, colpart);
    return;
  }
  if (colpart) return;  // contract violation: the caller must have used the wide path
  const dim3 g((C + 63) / 64, (R + 63) / 64), b(256);
  if (fmt == 0)
    hipLaunchKernelGGL((cast_transpose_fp8_kernel<0, uint16_t>), g, b, 0, st, x, y, yt, R, C, scale, amax);
  else
    hipLaunchKernelGGL((cast_transpose_fp8_kernel<1, uint16_t>), g, b, 0, st, x, y, yt, R, C, scale, amax);
}

void launch_fp8_update_scale(float* hist, int H, int n, float* amax, float* scale, float* inv_scale, const float* fmax,
                             int margin, int64_t step, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(update_scale_kernel, dim3((n + 255) / 256), dim3(256), 0, st, hist, H, n, amax, scale, inv_scale,
                     fmax, ldexpf(1.f, margin), step);
}

}  // namespace mlt
