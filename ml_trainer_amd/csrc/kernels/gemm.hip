// bf16 GEMM on CDNA4 matrix cores (v_mfma_f32_16x16x32_bf16) for the transformer
// path (BERT-base / large linears: QKV, attention-out, FFN1, FFN2 and their
// backward passes).
//
//   C[M,N] = alpha * A[M,K] . B[K,N]  (+ bias[N]) (+ epilogue), fp32 accumulate
//
// Operand storage (all three training GEMMs of a Linear without transposes):
//   A_K : A[m][k] (k contiguous, lda >= K)      A_M : A stored [k][m] (m contiguous)
//   B_K : B stored [n][k] (k contiguous)        B_N : B[k][n] (n contiguous)
//   fwd   Y  = X  . W^T   -> A_K, B_K   (W is [out,in])
//   dgrad dX = dY . W     -> A_K, B_N
//   wgrad dW = dY^T . X   -> A_M, B_N
//
// Tiling: 128x128 block tile, BK = 64, 256 threads = 4 waves in a 2x2 grid, each
// wave owns a 64x64 sub-tile = 4x4 MFMA tiles (64 fp32 accumulators / lane).
// Global -> registers -> LDS staging, double-buffered, one barrier per K-step
// (issue tile k+1's global loads before the MFMAs of tile k, write them to LDS
// after -- the T14 "issue early / write late" split). LDS images:
//   * k-contiguous tile [128 rows][64 k]: 16-byte chunks XOR-swizzled by (row & 7),
//     fragments read with ds_read_b128;
//   * mn-contiguous tile [64 k][128 mn]: 16-byte chunks XOR-swizzled by (k & 15),
//     fragments read with the gfx950 transpose read ds_read_b64_tr_b16 (T10), so the
//     transposed operands of dgrad/wgrad cost no extra pass over HBM.
// Block index -> tile mapping is XCD-aware (consecutive tiles of one tile-row land
// on one XCD's L2). The epilogue stages the tile through LDS and writes 16-byte
// vectors, fusing bias, GELU (saving the pre-activation), dGELU, residual add and
// accumulate-into-output.
#include "mlt_common.h"
#include "mlt_gemm.h"
#include "mlt_kernels.h"

namespace mlt {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int GB_M = 128, GB_N = 128, GB_K = 64, G_THREADS = 256;
constexpr int TILE_BYTES = 128 * 64 * 2;  // 16 KB per operand tile

// ---- global -> register staging ------------------------------------------------
// k-contiguous tile: rows r in [0,128), 8 chunks of 8 bf16 per row; 1024 chunks, 4 per thread.
__device__ __forceinline__ void load_k_tile(uint4 (&v)[4], const uint16_t* __restrict__ base, int64_t ld,
                                            int row0, int nrows, int k0, int K) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = threadIdx.x + i * G_THREADS, r = e >> 3, c = e & 7;
    const int row = row0 + r, k = k0 + c * 8;
    v[i] = (row < nrows && k < K) ? *reinterpret_cast<const uint4*>(base + (int64_t)row * ld + k)
                                  : make_uint4(0, 0, 0, 0);
  }
}
__device__ __forceinline__ void store_k_tile(uint8_t* lds, const uint4 (&v)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = threadIdx.x + i * G_THREADS, r = e >> 3, c = e & 7;
    *reinterpret_cast<uint4*>(lds + r * 128 + ((c ^ (r & 7)) << 4)) = v[i];
  }
}
// mn-contiguous tile: rows = k in [0,64), 16 chunks of 8 bf16 along mn; 1024 chunks, 4 per thread.
__device__ __forceinline__ void load_mn_tile(uint4 (&v)[4], const uint16_t* __restrict__ base, int64_t ld,
                                             int mn0, int nmn, int k0, int K) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = threadIdx.x + i * G_THREADS, kk = e >> 4, c = e & 15;
    const int k = k0 + kk, mn = mn0 + c * 8;
    v[i] = (k < K && mn < nmn) ? *reinterpret_cast<const uint4*>(base + (int64_t)k * ld + mn)
                               : make_uint4(0, 0, 0, 0);
  }
}
__device__ __forceinline__ void store_mn_tile(uint8_t* lds, const uint4 (&v)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = threadIdx.x + i * G_THREADS, kk = e >> 4, c = e & 15;
    *reinterpret_cast<uint4*>(lds + kk * 256 + ((c ^ (kk & 15)) << 4)) = v[i];
  }
}

// ---- LDS -> MFMA fragments (16x16x32: lane l holds rows/cols (l&15), k = 8(l>>4)+j) ----
__device__ __forceinline__ bf16x8 frag_k(const uint8_t* lds, int row, int kh) {
  const int lane = threadIdx.x & 63;
  const int r = row + (lane & 15), c = kh * 4 + (lane >> 4);
  return *reinterpret_cast<const bf16x8*>(lds + r * 128 + ((c ^ (r & 7)) << 4));
}
__device__ __forceinline__ bf16x8 frag_mn(const uint8_t* lds, int mn, int kh) {
  const int lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int col = mn + 4 * p;  // 4 consecutive mn of one k-row, 8-byte aligned
  const int c = col >> 3, half = (col & 7) * 2;
  const int k0 = kh * 32 + 8 * g + q;
  const int k1 = k0 + 4;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4*)(lds + k0 * 256 + ((c ^ (k0 & 15)) << 4) + half));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4*)(lds + k1 * 256 + ((c ^ (k1 & 15)) << 4) + half));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

template <bool AM, bool BN, typename OutT>
__global__ __launch_bounds__(G_THREADS, 2) void gemm_bf16_kernel(const uint16_t* __restrict__ A,
                                                                  const uint16_t* __restrict__ B,
                                                                  OutT* __restrict__ C, int M, int N, int K,
                                                                  int64_t lda, int64_t ldb, int64_t ldc,
                                                                  GemmEpi epi) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tiles_n = (N + GB_N - 1) / GB_N;
  const int nwg = gridDim.x;
  const int id = xcd_remap(blockIdx.x, nwg);
  const int tm = id / tiles_n, tn = id - tm * tiles_n;
  const int m0 = tm * GB_M, n0 = tn * GB_N;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = (wid >> 1) * 64, wn = (wid & 1) * 64;

  // buffer b: A tile at smem + 2b*TILE_BYTES, B tile right after it
#define AS(b) (smem + (b) * 2 * TILE_BYTES)
#define BS(b) (smem + (b) * 2 * TILE_BYTES + TILE_BYTES)

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[4], rb[4];
  const int nk = (K + GB_K - 1) / GB_K;
  // prologue: tile 0
  if (AM) load_mn_tile(ra, A, lda, m0, M, 0, K); else load_k_tile(ra, A, lda, m0, M, 0, K);
  if (BN) load_mn_tile(rb, B, ldb, n0, N, 0, K); else load_k_tile(rb, B, ldb, n0, N, 0, K);
  if (AM) store_mn_tile(AS(0), ra); else store_k_tile(AS(0), ra);
  if (BN) store_mn_tile(BS(0), rb); else store_k_tile(BS(0), rb);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {  // issue the next tile's global loads; they land while the MFMAs below run
      const int k1 = (kt + 1) * GB_K;
      if (AM) load_mn_tile(ra, A, lda, m0, M, k1, K); else load_k_tile(ra, A, lda, m0, M, k1, K);
      if (BN) load_mn_tile(rb, B, ldb, n0, N, k1, K); else load_k_tile(rb, B, ldb, n0, N, k1, K);
    }
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = AM ? frag_mn(AS(cur), wm + 16 * i, kh) : frag_k(AS(cur), wm + 16 * i, kh);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = BN ? frag_mn(BS(cur), wn + 16 * j, kh) : frag_k(BS(cur), wn + 16 * j, kh);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      if (AM) store_mn_tile(AS(cur ^ 1), ra); else store_k_tile(AS(cur ^ 1), ra);
      if (BN) store_mn_tile(BS(cur ^ 1), rb); else store_k_tile(BS(cur ^ 1), rb);
    }
    __syncthreads();
  }

#undef AS
#undef BS
  // ---- epilogue: registers (alpha, bias) -> LDS tile -> 16-byte vector stores (+aux ops) ----
  float* cs = reinterpret_cast<float*>(smem);  // [128][128] fp32 staging (64 KB)
  const int g = lane >> 4, cl = lane & 15;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = wn + 16 * j + cl;
      const float bv = (epi.bias && n0 + col < N) ? epi.bias[n0 + col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm + 16 * i + 4 * g + r;
        cs[row * 128 + col] = acc[i][j][r] * epi.alpha + bv;
      }
    }
  __syncthreads();
  // each thread stores 4 consecutive columns (16 B fp32 / 8 B bf16) per iteration
#pragma unroll 4
  for (int e = threadIdx.x; e < 128 * 32; e += G_THREADS) {
    const int row = e >> 5, c4 = (e & 31) * 4;
    const int gm = m0 + row, gn = n0 + c4;
    if (gm >= M || gn >= N) continue;
    const float4 v = *reinterpret_cast<const float4*>(cs + row * 128 + c4);
    float vv[4] = {v.x, v.y, v.z, v.w};
    epilogue_store4<OutT>(C, ldc, epi, gm, gn, N, vv);
  }
}

template <bool AM, bool BN, typename OutT>
static void launch_one(const uint16_t* A, const uint16_t* B, OutT* C, int M, int N, int K, int64_t lda, int64_t ldb,
                       int64_t ldc, const GemmEpi& e, hipStream_t st) {
  const int tiles = ((M + GB_M - 1) / GB_M) * ((N + GB_N - 1) / GB_N);
  constexpr int kSmem = 4 * TILE_BYTES;  // 64 KB (also the fp32 epilogue tile)
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_bf16_kernel<AM, BN, OutT>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, kSmem);
    attr_set = true;
  }
  hipLaunchKernelGGL((gemm_bf16_kernel<AM, BN, OutT>), dim3(tiles), dim3(G_THREADS), kSmem, st, A, B, C, M, N, K, lda,
                     ldb, ldc, e);
}

void launch_gemm_bf16_128(int a_mn, int b_mn, bool out_f32, const uint16_t* A, const uint16_t* B, void* C, int M,
                          int N, int K, int64_t lda, int64_t ldb, int64_t ldc, const GemmEpi& e, hipStream_t st) {
  if (M <= 0 || N <= 0) return;
#define MLT_GEMM_CASE(AMV, BNV)                                                                          \
  if (a_mn == AMV && b_mn == BNV) {                                                                      \
    if (out_f32)                                                                                         \
      launch_one<AMV, BNV, float>(A, B, (float*)C, M, N, K, lda, ldb, ldc, e, st);                       \
    else                                                                                                 \
      launch_one<AMV, BNV, uint16_t>(A, B, (uint16_t*)C, M, N, K, lda, ldb, ldc, e, st);                 \
    return;                                                                                              \
  }
  MLT_GEMM_CASE(0, 0)
  MLT_GEMM_CASE(0, 1)
  MLT_GEMM_CASE(1, 0)
  MLT_GEMM_CASE(1, 1)
#undef MLT_GEMM_CASE
}

// ---- column sums (bias gradients): out[n] (+)= sum_m X[m, n], X bf16 [M, N] ----------
// Column sums of a bf16 [M, N] matrix (bias gradients), two deterministic stages:
// (1) grid (N/512 column strips, R row slabs): lane = 8 columns (one 16-byte load per row),
//     4 waves interleave rows, reduced through LDS -> part[R][N];
// (2) reduce_rows (layernorm.hip): wave = 4 columns, lanes stride the R partials, xor-tree.
__global__ __launch_bounds__(256) void colsum_partial_kernel(const uint16_t* __restrict__ X, int M, int N,
                                                             int64_t ldx, int rpb, float* __restrict__ part) {
  __shared__ float red[4][512];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = blockIdx.x * 512 + lane * 8;
  const int r0 = blockIdx.y * rpb, r1 = min(M, r0 + rpb);
  float a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = 0.f;
  auto acc = [&](const uint4& v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a[2 * j] += __uint_as_float(w[j] << 16);
      a[2 * j + 1] += __uint_as_float(w[j] & 0xffff0000u);
    }
  };
  if (c < N) {
    const uint16_t* p = X + c;
    int r = r0 + wid;
    for (; r + 12 < r1; r += 16) {
      const uint4 v0 = *reinterpret_cast<const uint4*>(p + (int64_t)r * ldx);
      const uint4 v1 = *reinterpret_cast<const uint4*>(p + (int64_t)(r + 4) * ldx);
      const uint4 v2 = *reinterpret_cast<const uint4*>(p + (int64_t)(r + 8) * ldx);
      const uint4 v3 = *reinterpret_cast<const uint4*>(p + (int64_t)(r + 12) * ldx);
      acc(v0);
      acc(v1);
      acc(v2);
      acc(v3);
    }
    for (; r < r1; r += 4) acc(*reinterpret_cast<const uint4*>(p + (int64_t)r * ldx));
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[wid][lane * 8 + j] = a[j];
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 256) {
    const int cc = blockIdx.x * 512 + i;
    if (cc < N) part[(int64_t)blockIdx.y * N + cc] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
  }
}

static void colsum_geometry(int M, int& R, int& rpb) {
  R = M < 32 ? 1 : (M + 31) / 32;
  if (R > 256) R = 256;
  rpb = (M + R - 1) / R;
  R = (M + rpb - 1) / rpb;
}

int64_t colsum_ws_floats(int M, int N) {
  int R, rpb;
  colsum_geometry(M, R, rpb);
  return (int64_t)R * N;
}

void launch_colsum_bf16(const uint16_t* X, int M, int N, int64_t ldx, float* out, int accumulate, float* ws,
                        hipStream_t st) {
  if (N <= 0) return;
  if (M <= 0) {
    if (!accumulate) (void)hipMemsetAsync(out, 0, sizeof(float) * N, st);
    return;
  }
  int R, rpb;
  colsum_geometry(M, R, rpb);
  hipLaunchKernelGGL(colsum_partial_kernel, dim3((N + 511) / 512, R), dim3(256), 0, st, X, M, N, ldx, rpb, ws);
  SegOut o{{out, nullptr, nullptr}};
  launch_reduce_rows(ws, R, N, N, N, o, accumulate ? 1 : 0, st);
}

}  // namespace mlt
