// Fragment / staging helpers shared by the 256-wide bf16 / fp8 GEMM kernels (gemm_tile.hip:
// one tile per workgroup; gemm_persist.hip: persistent tile loop with register epilogue).
#pragma once
#include "mlt_common.h"

namespace mlt {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int T_BK = 64, T_NT = 512;

// mn-contiguous images XOR-swizzle the 16-B chunk index of k-row kk within aligned groups of 16
// (or 8 when a k-row holds 24 chunks) so the permutation never leaves the row.
// Rows of 256 / 512 B start at the same bank, so only the chunk position decides the bank. One
// ds_read_b64_tr_b16 lane group (32 lanes) reads 8 k-rows {8g + q: g = 0..1, q = 0..3} x two
// adjacent chunks {c0, c0 + 1} (c0 even) x two 8-B halves. The former XOR by (kk & 15) gave the 8
// rows the values {0..3, 8..11}, whose pairs {x, x ^ 1} collide -> every slot read twice, a 2-way
// conflict on every transposed read (PMC: SQ_LDS_BANK_CONFLICT = 49 % of the wgrad kernel's LDS
// cycles). XOR by 2q + 8g (all even, distinct) puts the 16 (row, chunk) pairs on 16 distinct
// chunk positions: conflict-free.
template <int CPR>
struct MnSwz {
  static constexpr bool WIDE = CPR % 16 == 0;
  static __device__ __forceinline__ int x(int kk) {
    return WIDE ? (((kk & 3) << 1) | (((kk >> 3) & 1) << 3)) : (kk & 7);
  }
};

// ---- fragments --------------------------------------------------------------------------
__device__ __forceinline__ bf16x8 tfrag_k(const uint8_t* lds, int row, int kh) {
  const int lane = threadIdx.x & 63;
  const int r = row + (lane & 15), c = kh * 4 + (lane >> 4);
  return *reinterpret_cast<const bf16x8*>(lds + r * 128 + ((c ^ (r & 7)) << 4));
}
template <int RB>  // row bytes of the mn-contiguous image (2 * BM or 2 * BN)
__device__ __forceinline__ bf16x8 tfrag_mn(const uint8_t* lds, int mn, int kh) {
  const int lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int col = mn + 4 * p;
  const int c = col >> 3, half = (col & 7) * 2;
  const int k0 = kh * 32 + 8 * g + q, k1 = k0 + 4;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + k0 * RB + ((c ^ MnSwz<RB / 16>::x(k0)) << 4) + half));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + k1 * RB + ((c ^ MnSwz<RB / 16>::x(k1)) << 4) + half));
  const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

// ---- per-thread glds sources -----------------------------------------------------------
// Chunk e = i * 512 + threadIdx.x of an operand image lands at LDS byte e * 16. Byte
// addressing: ES = element size (2 bf16, 1 fp8); a k-contiguous row holds 128 bytes per K-step.
template <int ROWS, bool MN, int ES>  // ROWS = extent of the operand's M (or N) side of the tile
__device__ __forceinline__ const uint8_t* glds_src(const uint8_t* __restrict__ base, int64_t ld, int i, int mn0,
                                                   int nmn) {
  const int e = i * T_NT + threadIdx.x;
  if (!MN) {  // [ROWS][128 B]: 8 chunks per row
    const int r = e >> 3, p = e & 7, c = p ^ (r & 7);
    const int row = min(mn0 + r, nmn - 1);
    return base + ((int64_t)row * ld) * ES + c * 16;
  } else {    // [64 k][ROWS]: ROWS/8 chunks per k-row (bf16 only)
    constexpr int CPR = ROWS / 8;
    const int kk = e / CPR, p = e % CPR, c = p ^ MnSwz<CPR>::x(kk);
    const int col = min(mn0 + c * 8, nmn - 8);
    return base + ((int64_t)kk * ld + col) * ES;
  }
}

// the same source as a 32-bit byte offset from the operand base (ping-pong kernel: a uniform
// 64-bit base in SGPRs + a 32-bit per-lane offset is the glds SADDR form, half the VGPRs)
template <int ROWS, bool MN, int ES>
__device__ __forceinline__ uint32_t glds_off(int64_t ld, int i, int mn0, int nmn) {
  const int e = i * T_NT + threadIdx.x;
  if (!MN) {
    const int r = e >> 3, p = e & 7, c = p ^ (r & 7);
    const int row = min(mn0 + r, nmn - 1);
    return (uint32_t)(row * ld * ES + c * 16);
  } else {
    constexpr int CPR = ROWS / 8;
    const int kk = e / CPR, p = e % CPR, c = p ^ MnSwz<CPR>::x(kk);
    const int col = min(mn0 + c * 8, nmn - 8);
    return (uint32_t)((kk * ld + col) * ES);
  }
}

// fp8 operand fragment of v_mfma_scale_f32_16x16x128_f8f6f4: lane l holds row (l&15), k bytes
// 32(l>>4) .. +31 = chunks 2(l>>4), 2(l>>4)+1 of the 128-byte row (positional k pairing with B)
typedef int i32x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ i32x8 tfrag_f8(const uint8_t* lds, int row) {
  const int lane = threadIdx.x & 63;
  const int r = row + (lane & 15), c0 = 2 * (lane >> 4);
  const uint4 lo = *reinterpret_cast<const uint4*>(lds + r * 128 + ((c0 ^ (r & 7)) << 4));
  const uint4 hi = *reinterpret_cast<const uint4*>(lds + r * 128 + (((c0 + 1) ^ (r & 7)) << 4));
  return i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
}

struct GemmEpi;
// gemm_persist.hip (planner cfg 6): persistent 256x256 tile loop, register epilogue, splits = 1
template <bool AM, bool BNL, typename OutT, int F8A, int F8B>
void launch_gemm_persist(const uint8_t* A, const uint8_t* B, OutT* C, int M, int N, int K, int64_t lda, int64_t ldb,
                         int64_t ldc, const GemmEpi& e, int group_m, int max_blocks, hipStream_t st);

// gemm_w4.hip (planner cfg 7): 4-wave 256x256x64 tile, generated-asm main loop, k-contiguous A,
// B k-contiguous or (b_mn) n-contiguous
bool gemm_w4_supported(int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int out_bytes, const GemmEpi& e,
                       bool b_mn);
template <typename OutT>
void launch_gemm_w4(const uint8_t* A, const uint8_t* B, OutT* C, int M, int N, int K, int64_t lda, int64_t ldb,
                    int64_t ldc, const GemmEpi& e, int group_m, bool b_mn, hipStream_t st);
// ... its weight-gradient layout (A [K][M], B [K][N]) with split-K raw partials ws[z][M][N]
bool gemm_w4_wgrad_supported(int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int out_bytes,
                             const GemmEpi& e, int splits, int ksteps);
template <typename OutT>
void launch_gemm_w4_wgrad(const uint8_t* A, const uint8_t* B, OutT* C, float* ws, int M, int N, int K, int64_t lda,
                          int64_t ldb, int64_t ldc, const GemmEpi& e, int group_m, int splits, int ksteps,
                          hipStream_t st);
// ... and its fp8 form (block-scaled MFMA, unit scales; both operands k-contiguous bytes)
bool gemm_w4_f8_supported(int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int out_bytes,
                          const GemmEpi& e);
bool gemm_w4_f8_splitk_supported(int M, int N, int K, int64_t lda, int64_t ldb, int splits, int ksteps);
template <int FA, int FB>
void launch_gemm_w4_f8_splitk(const uint8_t* A, const uint8_t* B, float* ws, int M, int N, int K, int64_t lda,
                              int64_t ldb, int group_m, int splits, int ksteps, hipStream_t st);
template <typename OutT, int FA, int FB>
void launch_gemm_w4_f8(const uint8_t* A, const uint8_t* B, OutT* C, int M, int N, int K, int64_t lda, int64_t ldb,
                       int64_t ldc, const GemmEpi& e, int group_m, hipStream_t st);
bool launch_gemm_w4_f8_q(int fmt_a, const uint8_t* A, const uint8_t* B, uint8_t* Y, int M, int N, int K,
                         int64_t lda, int64_t ldb, int64_t ldy, const GemmEpi& e, int group_m, hipStream_t st);

}  // namespace mlt
