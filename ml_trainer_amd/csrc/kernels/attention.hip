// Fused multi-head attention (flash-style) forward / backward for gfx950, bf16 MFMA.
//
// Layout: the QKV projection's output qkv [B*S, 3*H*64] is read in place (q | k | v
// blocks of H heads x 64 dims per row); O [B*S, H*64]; the backward writes dQKV in the
// same packed layout. Head dim 64, key-padding mask by per-sequence valid length.
//
// Forward, one 256-thread block per (64-query block, head, batch), wave = 16 queries:
//   S^T (keys x queries) = K . Q^T   -- "swapped" product: each lane owns ONE query
//   column, so the online-softmax max / sum is lane-local plus two xor-shuffles;
//   O^T (dims x queries) += V^T . P^T -- P^T is the accumulator of S^T re-used as the
//   MFMA B operand straight from registers (k order permuted identically on both
//   operands, cdna_hip_programming.md §3), V^T comes from the V tile in LDS through the
//   transpose read ds_read_b64_tr_b16. The S x S score matrix never touches HBM; the
//   log-sum-exp per query is saved for the backward pass.
// Backward = two kernels over the same (64-block, head, batch) grid, no atomics, bitwise
// reproducible (>= B*H*S/64 workgroups, e.g. 1536 for BERT-base b16 s512); the ring variants run
// dQ first, which also produces delta = rowsum(dO * O) for dK/dV:
//   dK/dV: block = 64 keys, wave = 16 keys (keys on lanes): S = Q K^T, dP = dO V^T,
//     P = exp2(S*scale*log2e - LSE2), dS = P (dP - delta); dV^T += dO^T P, dK^T += Q^T dS with
//     accumulators in registers across the whole query loop;
//   dQ: block = 64 queries, swapped like the forward (queries on lanes): S^T = K Q^T,
//     dP^T = V dO^T, dS^T lane-local, dQ^T += K^T dS^T with dS^T fed from registers.
// Global->LDS staging of the next tile is register-staged (loads issued before the MFMA work
// of the current tile, LDS writes after it), so HBM latency overlaps the math.
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "mlt_common.h"
#include "mlt_fp8.h"
#include "mlt_kernels.h"

namespace mlt {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int AH = 64;  // head dim
constexpr int AB = 64;  // query / key block

// raw v_exp_f32 (2^x): exp2f wraps it in a denormal-range fix-up (compare, select, two
// ldexp) that the probabilities here never need; exp2(-inf) = 0 doubles as the mask
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Backward softmax-gradient math on score PAIRS (build A/B switch, -DMLT_ATTN_PKF32=1): the
// scale-and-shift and dS = P * dP' of two adjacent accumulator rows as one v_pk_fma_f32 / one
// v_pk_mul_f32 instead of two scalar ops each; the exp2 stays scalar. Off by default: measured at
// B512 (profiles/r5/gemm_gelu_tab_attn_pkf32_ab.jsonl, profiles/pmc/attn_bf16_b512_r5*.jsonl) it
// cuts VALU instructions 5 % (dK/dV) / 9 % (dQ), VALU per MFMA 4.30 -> 4.07 / 4.89 -> 4.44, but the
// backward pair is not faster (1.946-1.958 vs 1.937-1.945 ms): dQ -2.7 % busy cycles, dK/dV +1.6 %
// (packed f32 ops between MFMAs cost more issue than the two scalar ops, MI355X_MICROARCH.md).
#ifndef MLT_ATTN_PKF32
#define MLT_ATTN_PKF32 0
#endif
// p = exp2(s * sl2 - lr) and ds = p * dp for rows (r0, r0 + 1) of one f32x4 accumulator
__device__ __forceinline__ void pk_prob_ds(const f32x4& s, const f32x4& dp, float sl2, f32x2 nlr, int r0, f32x2& p,
                                           f32x2& d) {
  const f32x2 x = __builtin_elementwise_fma(f32x2{s[r0], s[r0 + 1]}, f32x2{sl2, sl2}, nlr);
  p = f32x2{fast_exp2(x.x), fast_exp2(x.y)};
  d = p * f32x2{dp[r0], dp[r0 + 1]};
}

__device__ __forceinline__ f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// [64 rows][64 bf16] LDS tile, 128-byte rows, 16-byte chunks XOR-swizzled by (row & 7)
__device__ __forceinline__ int tile_off(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

// cooperative global -> LDS copy of a 64x64 bf16 tile (rows `row0..row0+63` of a row-major
// matrix with row stride ld elements, starting at column col0); rows >= nrows are zero
__device__ __forceinline__ void stage_tile(uint8_t* lds, const uint16_t* __restrict__ g, int64_t ld, int64_t row0,
                                           int nrows_valid, int col0) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = threadIdx.x + 256 * i, r = e >> 3, c = e & 7;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r < nrows_valid) v = *reinterpret_cast<const uint4*>(g + (row0 + r) * ld + col0 + c * 8);
    *reinterpret_cast<uint4*>(lds + tile_off(r, c)) = v;
  }
}

// register-staged variant: load_tile issues the global loads, store_tile writes them to LDS
struct TileRegs {
  uint4 v[2];
};
__device__ __forceinline__ void load_tile(TileRegs& t, const uint16_t* __restrict__ g, int64_t ld, int64_t row0,
                                          int nrows_valid, int col0) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = threadIdx.x + 256 * i, r = e >> 3, c = e & 7;
    t.v[i] = r < nrows_valid ? *reinterpret_cast<const uint4*>(g + (row0 + r) * ld + col0 + c * 8)
                             : make_uint4(0, 0, 0, 0);
  }
}
__device__ __forceinline__ void store_tile(uint8_t* lds, const TileRegs& t) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = threadIdx.x + 256 * i, r = e >> 3, c = e & 7;
    *reinterpret_cast<uint4*>(lds + tile_off(r, c)) = t.v[i];
  }
}

// row fragment: 16 rows starting at `row`, k = 32*kh + 8*(lane>>4) + j (ds_read_b128)
__device__ __forceinline__ bf16x8 frag_row(const uint8_t* lds, int row, int kh) {
  const int lane = threadIdx.x & 63;
  return *reinterpret_cast<const bf16x8*>(lds + tile_off(row + (lane & 15), kh * 4 + (lane >> 4)));
}
// transposed fragment: column (col + lane&15) of rows {r0+q} and {r1+q}, q = 0..3 (ds_read_b64_tr_b16)
__device__ __forceinline__ bf16x8 frag_tr(const uint8_t* lds, int r0, int r1, int col) {
  const int lane = threadIdx.x & 63, i = lane & 15, q = i >> 2, p = i & 3;
  const int cc = col + 4 * p, chunk = cc >> 3, half = (cc & 7) * 2;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + tile_off(r0 + q, chunk) + half));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + tile_off(r1 + q, chunk) + half));
  const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

__device__ __forceinline__ short bf16_bits(float f) { return (short)f32_to_bf16(f); }

// pack an accumulator pair (tiles t0, t1 of 16 rows each) into a k-permuted B/A operand:
// element j <-> row 16*(j>>2) + 4*(lane>>4) + (j&3) of the 32-row k-step
__device__ __forceinline__ bf16x8 pack_acc(const f32x4& t0, const f32x4& t1) {
  const s16x8 r = {bf16_bits(t0[0]), bf16_bits(t0[1]), bf16_bits(t0[2]), bf16_bits(t0[3]),
                   bf16_bits(t1[0]), bf16_bits(t1[1]), bf16_bits(t1[2]), bf16_bits(t1[3])};
  return __builtin_bit_cast(bf16x8, r);
}

// 1-D grid of (row block, head, batch) with the XCD-aware remap: the row blocks of one
// (batch, head) are consecutive after the remap, so they run on one XCD and its L2 serves the
// K / V (or Q / dO) tiles they all re-read instead of every XCD fetching them from HBM.
__device__ __forceinline__ void block_coords(int S, int rows_per_block, int H, int& rb, int& h, int& b) {
  const int nrb = (S + rows_per_block - 1) / rows_per_block;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  rb = id % nrb;
  h = (id / nrb) % H;
  b = id / (nrb * H);
  MLT_DCHECK((int)gridDim.x % (nrb * H) == 0 && rb * rows_per_block < S);  // grid = B * H * row blocks
}

// Register staging with buffer loads issued as inline asm. Through the builtins, hipcc's waitcnt
// pass puts an s_waitcnt vmcnt(0) at the top of the K/V loop (in front of the first QK^T MFMA),
// i.e. it waits for the next block's loads right after issuing them and the staging hides no
// latency. As asm the loads are invisible to that pass; vmem_wait_tiles is the one wait, placed
// just before the registers are written to LDS, with the tile registers as "+v" operands so no
// use of them can move above it (cdna_hip_programming.md §5.7 item 1). The loop issues no other
// vector-memory instruction, so vmcnt(0) there retires exactly these loads.
typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4 buffer_rsrc(const void* p, int64_t bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)p;
  i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((int)((a >> 32) & 0xffff));  // stride 0
  r[2] = __builtin_amdgcn_readfirstlane((int)bytes);                 // num_records: reads past it return 0
  r[3] = 0x00020000;
  return r;
}
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4 buffer_load_x4_asm(const i32x4& rs, int voff) {
  u32x4 v;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(voff), "s"(rs) : "memory");
  return v;
}
__device__ __forceinline__ void vmem_wait_tiles(u32x4 (&a)[2], u32x4 (&b)[2]) {
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(a[0]), "+v"(a[1]), "+v"(b[0]), "+v"(b[1]) :: "memory");
}
__device__ __forceinline__ void store_tile_v(uint8_t* lds, const u32x4 (&t)[2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = threadIdx.x + 256 * i, r = e >> 3, c = e & 7;
    *reinterpret_cast<u32x4*>(lds + tile_off(r, c)) = t[i];
  }
}

// ---------------------------------------------------------------------------
// forward: NQ 16-query groups per wave (the K / V^T fragments read from LDS feed NQ MFMAs).
// The softmax side bounded the first version of this kernel (per 64-key block a wave issued 16
// MFMAs = 256 MFMA cycles against ~150 VALU instructions = ~600 issue cycles); it is cut to ~3.5
// VALU per score:
//   * the key mask runs only on the block that holds the sequence end (block-uniform branch);
//   * the max is taken over the raw scores (scale > 0 commutes with max) and the scale is folded
//     into the exponent: p = exp2(fma(s, scale*log2e, -m)), one FMA + one v_exp per score;
//   * the row sum l comes from the MFMA pipe, which has slack: an all-ones A operand against the
//     same bf16 P^T the P.V product uses (so l normalizes exactly the weights that were summed);
//   * defer-max (cdna_hip_programming.md T13): O and l are rescaled only when some lane's max
//     grew by more than kFwdDeferThr (base 2) since the last rescale; otherwise the stale max
//     stays and p <= 2^kFwdDeferThr. The decision for a block is taken after its scores and
//     before any of its p is formed, with the previous block's P.V complete -- the textbook
//     order, so everything at the old max is scaled exactly once.
// ---------------------------------------------------------------------------
constexpr float kFwdDeferThr = 8.f;

template <int NQ>
__global__ __launch_bounds__(256) void attn_fwd_lean_kernel(const uint16_t* __restrict__ qkv,
                                                            uint16_t* __restrict__ out, float* __restrict__ lse,
                                                            const int* __restrict__ lens, int S, int H,
                                                            float scale) {
  __shared__ __attribute__((aligned(16))) uint8_t Ks[2][AB * 128];
  __shared__ __attribute__((aligned(16))) uint8_t Vs[2][AB * 128];
  int qb, h, b;
  block_coords(S, 64 * NQ, H, qb, h, b);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15;
  const int D = H * AH;
  const int64_t ld = 3 * (int64_t)D;
  const int64_t base = (int64_t)b * S;
  const int len = lens ? lens[b] : S;
  MLT_DCHECK(len >= 0 && len <= S);
  int q[NQ];
  bf16x8 qf[NQ][2];
#pragma unroll
  for (int n = 0; n < NQ; ++n) {
    q[n] = qb * (64 * NQ) + n * 64 + wid * 16 + i;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
      qf[n][kh] = q[n] < S ? *reinterpret_cast<const bf16x8*>(qkv + (base + q[n]) * ld + h * AH + kh * 32 + 8 * g)
                           : bf16x8{};
  }
  f32x4 o[NQ][4], lacc[NQ];
  float m[NQ];
#pragma unroll
  for (int n = 0; n < NQ; ++n) {
    m[n] = -INFINITY;
    lacc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int d = 0; d < 4; ++d) o[n][d] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const s16x8 ones_bits = {0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80};
  const bf16x8 ones = __builtin_bit_cast(bf16x8, ones_bits);
  const int nkb = (len + AB - 1) / AB;
  const float sl2 = scale * 1.4426950408889634f;  // exponents in base 2
  u32x4 kr[2], vr[2];
  // loop-invariant byte offsets of this thread's two 16-byte K chunks inside a 64-row block (V:
  // + 2 D elements): with the block base in the scalar descriptor, no per-iteration address VGPRs
  int voff[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int e = threadIdx.x + 256 * t;
    voff[t] = (int)(((int64_t)(e >> 3) * ld + D + h * AH + (e & 7) * 8) * 2);
  }
  if (nkb > 0) {
    stage_tile(Ks[0], qkv, ld, base, min(AB, S), D + h * AH);
    stage_tile(Vs[0], qkv, ld, base, min(AB, S), 2 * D + h * AH);
  }
  __syncthreads();
  // retire the Q fragment loads here, on every path into the loop: the waitcnt pass merges paths
  // at the loop header and would otherwise put this wait inside the loop, in front of every
  // block's first MFMA (an S_WAITCNT it can see, unlike an asm one: simm16 0x0F70 = vmcnt(0))
  __builtin_amdgcn_s_waitcnt(0x0F70);
  for (int kb = 0; kb < nkb; ++kb) {
    const int cur = kb & 1;
    const bool more = kb + 1 < nkb;
    if (more) {  // next K / V block -> registers (rows >= S read as 0), LDS after the math
      const int k1 = (kb + 1) * AB;
      const i32x4 rs = buffer_rsrc(qkv + (base + k1) * ld, (int64_t)(S - k1) * ld * 2);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        kr[t] = buffer_load_x4_asm(rs, voff[t]);
        vr[t] = buffer_load_x4_asm(rs, voff[t] + 2 * D);
      }
    }
    f32x4 s[NQ][4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
      for (int n = 0; n < NQ; ++n) s[n][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        const bf16x8 kfr = frag_row(Ks[cur], kt * 16, kh);
#pragma unroll
        for (int n = 0; n < NQ; ++n) s[n][kt] = mfma(kfr, qf[n][kh], s[n][kt]);
      }
    }
    if ((kb + 1) * AB > len) {  // the block holding the sequence end: mask the keys past it
#pragma unroll
      for (int n = 0; n < NQ; ++n)
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (kb * AB + kt * 16 + 4 * g + r >= len) s[n][kt][r] = -INFINITY;
    }
#pragma unroll
    for (int n = 0; n < NQ; ++n) {
      float bm = s[n][0][0];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) bm = fmaxf(bm, s[n][kt][r]);
      bm = fmaxf(bm, __shfl_xor(bm, 16, 64));
      bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
      const float cand = bm * sl2;  // this block's max, scaled (finite: the block has a valid key)
      if (__any(cand - m[n] > kFwdDeferThr)) {  // wave-uniform: rescale O and l to the new max
        const float mn = fmaxf(m[n], cand);
        const float alpha = fast_exp2(m[n] - mn);  // m = -inf on the first block -> 0
        m[n] = mn;
        lacc[n] *= alpha;
#pragma unroll
        for (int d = 0; d < 4; ++d) o[n][d] *= alpha;
      }
      const float nm = -m[n];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) s[n][kt][r] = fast_exp2(fmaf(s[n][kt][r], sl2, nm));
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 pb[NQ];
#pragma unroll
      for (int n = 0; n < NQ; ++n) {
        pb[n] = pack_acc(s[n][2 * ks], s[n][2 * ks + 1]);
        lacc[n] = mfma(ones, pb[n], lacc[n]);  // row sums of P on the MFMA pipe
      }
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const bf16x8 va = frag_tr(Vs[cur], 32 * ks + 4 * g, 32 * ks + 16 + 4 * g, d * 16);
#pragma unroll
        for (int n = 0; n < NQ; ++n) o[n][d] = mfma(va, pb[n], o[n][d]);
      }
    }
    if (more) {
      vmem_wait_tiles(kr, vr);
      store_tile_v(Ks[cur ^ 1], kr);
      store_tile_v(Vs[cur ^ 1], vr);
    }
    __syncthreads();
  }
#pragma unroll
  for (int n = 0; n < NQ; ++n) {
    if (q[n] < S) {
      const float l = lacc[n][0];
      const float inv = l > 0.f ? 1.f / l : 0.f;
      uint16_t* op = out + (base + q[n]) * (int64_t)D + h * AH;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        ushort4 u;
        u.x = f32_to_bf16(o[n][d][0] * inv);
        u.y = f32_to_bf16(o[n][d][1] * inv);
        u.z = f32_to_bf16(o[n][d][2] * inv);
        u.w = f32_to_bf16(o[n][d][3] * inv);
        *reinterpret_cast<ushort4*>(op + d * 16 + 4 * g) = u;
      }
      if (g == 0) lse[((int64_t)b * H + h) * S + q[n]] = m[n] + __log2f(l);
    }
  }
}

// delta[b,h,q] = sum_d dO[q, h, d] * O[q, h, d]
__global__ __launch_bounds__(256) void attn_delta_kernel(const uint16_t* __restrict__ dout,
                                                         const uint16_t* __restrict__ out, float* __restrict__ delta,
                                                         int64_t rows, int H) {
  const int64_t idx = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);  // (row, h) pair, 16 lanes each
  const int sub = threadIdx.x & 15;
  const int64_t row = idx / H;
  const int h = (int)(idx - row * H);
  float s = 0.f;
  if (row < rows) {
    const int64_t off = row * (int64_t)H * AH + h * AH + sub * 4;
    const ushort4 a = *reinterpret_cast<const ushort4*>(dout + off);
    const ushort4 c = *reinterpret_cast<const ushort4*>(out + off);
    s = bf16_to_f32(a.x) * bf16_to_f32(c.x) + bf16_to_f32(a.y) * bf16_to_f32(c.y) +
        bf16_to_f32(a.z) * bf16_to_f32(c.z) + bf16_to_f32(a.w) * bf16_to_f32(c.w);
  }
  s = group_sum<16>(s);
  if (sub == 0 && row < rows) {
    // layout [B, H, S] like lse: row = b*S + q -> needs S; the host passes rows = B*S and
    // we store by (row, h) then the backward indexes delta[row * H + h]
    delta[row * H + h] = s;
  }
}

// ---------------------------------------------------------------------------
// backward, dK / dV: one block per (64*NK-key block, head, batch); NK 16-key groups per wave
// ---------------------------------------------------------------------------
template <int NK>
__global__ __launch_bounds__(256) void attn_bwd_dkdv_kernel(const uint16_t* __restrict__ qkv,
                                                            const uint16_t* __restrict__ dout,
                                                            const float* __restrict__ lse,
                                                            const float* __restrict__ delta,
                                                            const int* __restrict__ lens, uint16_t* __restrict__ dqkv,
                                                            int S, int H, float scale) {
  __shared__ __attribute__((aligned(16))) uint8_t Qs[2][AB * 128];
  __shared__ __attribute__((aligned(16))) uint8_t Os[2][AB * 128];  // dO tiles
  __shared__ float lse_s[2][AB], del_s[2][AB];
  int kbk, h, b;
  block_coords(S, 64 * NK, H, kbk, h, b);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15;
  const int D = H * AH;
  const int64_t ld = 3 * (int64_t)D;
  const int64_t base = (int64_t)b * S;
  const int len = lens ? lens[b] : S;
  const int k0b = kbk * (64 * NK);
  if (k0b >= len) {  // fully masked key block: zero gradients
    for (int e = threadIdx.x; e < 64 * NK * AH; e += 256) {
      const int kk = k0b + e / AH, d = e % AH;
      if (kk < S) {
        dqkv[(base + kk) * ld + D + h * AH + d] = 0;
        dqkv[(base + kk) * ld + 2 * D + h * AH + d] = 0;
      }
    }
    return;
  }
  const float sl2 = scale * 1.4426950408889634f;
  int key[NK];
  bf16x8 kf[NK][2], vf[NK][2];  // B operands: K[key][32kh + 8g + j], V[key][...]
#pragma unroll
  for (int n = 0; n < NK; ++n) {
    key[n] = k0b + n * 64 + wid * 16 + i;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      kf[n][kh] = key[n] < S ? *reinterpret_cast<const bf16x8*>(qkv + (base + key[n]) * ld + D + h * AH + kh * 32 + 8 * g)
                             : bf16x8{};
      vf[n][kh] = key[n] < S
                      ? *reinterpret_cast<const bf16x8*>(qkv + (base + key[n]) * ld + 2 * D + h * AH + kh * 32 + 8 * g)
                      : bf16x8{};
    }
  }
  f32x4 dk[NK][4], dv[NK][4];  // dK^T / dV^T [d = dt*16 + 4g + r][key = lane]
#pragma unroll
  for (int n = 0; n < NK; ++n)
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      dk[n][d] = f32x4{0.f, 0.f, 0.f, 0.f};
      dv[n][d] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  const int nqb = (S + AB - 1) / AB;
  auto stage_stats = [&](int buf, int q0) {
    if (threadIdx.x < AB) {
      const int qq = q0 + threadIdx.x;
      lse_s[buf][threadIdx.x] = qq < S ? lse[((int64_t)b * H + h) * S + qq] : 0.f;
      del_s[buf][threadIdx.x] = qq < S ? delta[(base + qq) * H + h] : 0.f;
    }
  };
  stage_tile(Qs[0], qkv, ld, base, min(AB, S), h * AH);
  stage_tile(Os[0], dout, (int64_t)D, base, min(AB, S), h * AH);
  stage_stats(0, 0);
  __syncthreads();
  TileRegs qr, orr;
  for (int qb = 0; qb < nqb; ++qb) {
    const int cur = qb & 1, q0 = qb * AB;
    const bool more = qb + 1 < nqb;
    if (more) {
      const int q1 = q0 + AB;
      load_tile(qr, qkv, ld, base + q1, min(AB, S - q1), h * AH);
      load_tile(orr, dout, (int64_t)D, base + q1, min(AB, S - q1), h * AH);
    }
    f32x4 p[NK][4], ds[NK][4];  // rows q = qt*16 + 4g + r, column = key (lane)
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      // dP accumulates onto -delta (the MFMA's C operand): dS = P * dP' (as the ring kernel)
      const float4 d4 = *reinterpret_cast<const float4*>(&del_s[cur][qt * 16 + 4 * g]);
      f32x4 sv[NK], dp[NK];
#pragma unroll
      for (int n = 0; n < NK; ++n) {
        sv[n] = f32x4{0.f, 0.f, 0.f, 0.f};
        dp[n] = f32x4{-d4.x, -d4.y, -d4.z, -d4.w};
      }
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        const bf16x8 qa = frag_row(Qs[cur], qt * 16, kh), oa = frag_row(Os[cur], qt * 16, kh);
#pragma unroll
        for (int n = 0; n < NK; ++n) {
          sv[n] = mfma(qa, kf[n][kh], sv[n]);
          dp[n] = mfma(oa, vf[n][kh], dp[n]);
        }
      }
      const float4 l4 = *reinterpret_cast<const float4*>(&lse_s[cur][qt * 16 + 4 * g]);
      const float lr[4] = {l4.x, l4.y, l4.z, l4.w};
#pragma unroll
      for (int n = 0; n < NK; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ql = qt * 16 + 4 * g + r;
          const bool ok = key[n] < len && q0 + ql < S;
          const float pv = fast_exp2(ok ? sv[n][r] * sl2 - lr[r] : -INFINITY);
          p[n][qt][r] = pv;
          ds[n][qt][r] = pv * dp[n][r];
        }
    }
    // dV^T += dO^T . P ; dK^T += Q^T . dS  (k = queries, two 32-query steps)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 pb[NK], sb[NK];
#pragma unroll
      for (int n = 0; n < NK; ++n) {
        pb[n] = pack_acc(p[n][2 * ks], p[n][2 * ks + 1]);
        sb[n] = pack_acc(ds[n][2 * ks], ds[n][2 * ks + 1]);
      }
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const bf16x8 ot = frag_tr(Os[cur], 32 * ks + 4 * g, 32 * ks + 16 + 4 * g, d * 16);
        const bf16x8 qt = frag_tr(Qs[cur], 32 * ks + 4 * g, 32 * ks + 16 + 4 * g, d * 16);
#pragma unroll
        for (int n = 0; n < NK; ++n) {
          dv[n][d] = mfma(ot, pb[n], dv[n][d]);
          dk[n][d] = mfma(qt, sb[n], dk[n][d]);
        }
      }
    }
    if (more) {
      store_tile(Qs[cur ^ 1], qr);
      store_tile(Os[cur ^ 1], orr);
      stage_stats(cur ^ 1, q0 + AB);
    }
    __syncthreads();
  }
#pragma unroll
  for (int n = 0; n < NK; ++n) {
    if (key[n] < S) {
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        uint16_t* kp = dqkv + (base + key[n]) * ld + D + h * AH + d * 16 + 4 * g;
        uint16_t* vp = dqkv + (base + key[n]) * ld + 2 * D + h * AH + d * 16 + 4 * g;
        ushort4 uk, uv;
        uk.x = f32_to_bf16(dk[n][d][0] * scale);
        uk.y = f32_to_bf16(dk[n][d][1] * scale);
        uk.z = f32_to_bf16(dk[n][d][2] * scale);
        uk.w = f32_to_bf16(dk[n][d][3] * scale);
        uv.x = f32_to_bf16(dv[n][d][0]);
        uv.y = f32_to_bf16(dv[n][d][1]);
        uv.z = f32_to_bf16(dv[n][d][2]);
        uv.w = f32_to_bf16(dv[n][d][3]);
        *reinterpret_cast<ushort4*>(kp) = uk;
        *reinterpret_cast<ushort4*>(vp) = uv;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// backward, dQ: one block per (64*NQ-query block, head, batch); queries on lanes
// ---------------------------------------------------------------------------
template <int NQ>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(const uint16_t* __restrict__ qkv,
                                                          const uint16_t* __restrict__ dout,
                                                          const float* __restrict__ lse,
                                                          const float* __restrict__ delta,
                                                          const int* __restrict__ lens, uint16_t* __restrict__ dqkv,
                                                          int S, int H, float scale) {
  __shared__ __attribute__((aligned(16))) uint8_t Ks[2][AB * 128];
  __shared__ __attribute__((aligned(16))) uint8_t Vs[2][AB * 128];
  int qb, h, b;
  block_coords(S, 64 * NQ, H, qb, h, b);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15;
  const int D = H * AH;
  const int64_t ld = 3 * (int64_t)D;
  const int64_t base = (int64_t)b * S;
  const int len = lens ? lens[b] : S;
  const float sl2 = scale * 1.4426950408889634f;
  int q[NQ];
  bf16x8 qf[NQ][2], of[NQ][2];  // B operands: Q[q][32kh + 8g + j], dO[q][...]
  float lq[NQ], dl[NQ];
  f32x4 acc[NQ][4];
#pragma unroll
  for (int n = 0; n < NQ; ++n) {
    q[n] = qb * (64 * NQ) + n * 64 + wid * 16 + i;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      qf[n][kh] = q[n] < S ? *reinterpret_cast<const bf16x8*>(qkv + (base + q[n]) * ld + h * AH + kh * 32 + 8 * g)
                           : bf16x8{};
      of[n][kh] = q[n] < S
                      ? *reinterpret_cast<const bf16x8*>(dout + (base + q[n]) * (int64_t)D + h * AH + kh * 32 + 8 * g)
                      : bf16x8{};
    }
    lq[n] = q[n] < S ? lse[((int64_t)b * H + h) * S + q[n]] : 0.f;
    dl[n] = q[n] < S ? delta[(base + q[n]) * H + h] : 0.f;
#pragma unroll
    for (int d = 0; d < 4; ++d) acc[n][d] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int nkb = (len + AB - 1) / AB;
  TileRegs kr, vr;
  if (nkb > 0) {
    stage_tile(Ks[0], qkv, ld, base, min(AB, S), D + h * AH);
    stage_tile(Vs[0], qkv, ld, base, min(AB, S), 2 * D + h * AH);
  }
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    const int cur = kb & 1;
    const bool more = kb + 1 < nkb;
    if (more) {
      const int k1 = (kb + 1) * AB;
      load_tile(kr, qkv, ld, base + k1, min(AB, S - k1), D + h * AH);
      load_tile(vr, qkv, ld, base + k1, min(AB, S - k1), 2 * D + h * AH);
    }
    f32x4 ds[NQ][4];  // dS^T rows = keys kt*16 + 4g + r, column = query of group n
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      f32x4 sv[NQ], dp[NQ];
#pragma unroll
      for (int n = 0; n < NQ; ++n) {  // dP accumulates onto -delta: dS = P * dP'
        sv[n] = f32x4{0.f, 0.f, 0.f, 0.f};
        dp[n] = f32x4{-dl[n], -dl[n], -dl[n], -dl[n]};
      }
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        const bf16x8 ka = frag_row(Ks[cur], kt * 16, kh), va = frag_row(Vs[cur], kt * 16, kh);
#pragma unroll
        for (int n = 0; n < NQ; ++n) {
          sv[n] = mfma(ka, qf[n][kh], sv[n]);
          dp[n] = mfma(va, of[n][kh], dp[n]);
        }
      }
#pragma unroll
      for (int n = 0; n < NQ; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kb * AB + kt * 16 + 4 * g + r;
          const float pv = fast_exp2(key < len ? sv[n][r] * sl2 - lq[n] : -INFINITY);
          ds[n][kt][r] = pv * dp[n][r];
        }
    }
    // dQ^T[d][q] += K^T[d][key] . dS^T[key][q]
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 sb[NQ];
#pragma unroll
      for (int n = 0; n < NQ; ++n) sb[n] = pack_acc(ds[n][2 * ks], ds[n][2 * ks + 1]);
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const bf16x8 kt = frag_tr(Ks[cur], 32 * ks + 4 * g, 32 * ks + 16 + 4 * g, d * 16);
#pragma unroll
        for (int n = 0; n < NQ; ++n) acc[n][d] = mfma(kt, sb[n], acc[n][d]);
      }
    }
    if (more) {
      store_tile(Ks[cur ^ 1], kr);
      store_tile(Vs[cur ^ 1], vr);
    }
    __syncthreads();
  }
#pragma unroll
  for (int n = 0; n < NQ; ++n) {
    if (q[n] < S) {
      uint16_t* qp = dqkv + (base + q[n]) * ld + h * AH;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        ushort4 u;
        u.x = f32_to_bf16(acc[n][d][0] * scale);
        u.y = f32_to_bf16(acc[n][d][1] * scale);
        u.z = f32_to_bf16(acc[n][d][2] * scale);
        u.w = f32_to_bf16(acc[n][d][3] * scale);
        *reinterpret_cast<ushort4*>(qp + d * 16 + 4 * g) = u;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Ring-staged backward (MLT_ATTN_RING, default on). The register-staged kernels above hold
// ~180 VGPRs, i.e. 2 waves per SIMD, and wait at the end of every 64-row step for tile loads
// issued at its start: one HBM/L2 round trip exposed per step. Here the streamed tiles (Q, dO
// and the LSE / delta rows for dK/dV; K, V for dQ) go HBM -> LDS by global_load_lds into a
// 4-deep ring, so three steps are in flight while one is computed; a counted vmcnt + raw
// s_barrier retires one stage per step (cdna_hip_programming.md §5 "Pipelining across
// barriers"); all LDS lives in ONE __shared__ array (the second-object trap, §5 item 4a).
// The math and its order are those of the kernels above: bit-identical gradients.
// ---------------------------------------------------------------------------
constexpr int kTile = AB * 128;  // one 64 x 64 bf16 tile

// glds of a 64x64 bf16 tile into the (row & 7)-swizzled image tile_off() reads: lane-linear
// LDS destination, swizzle on the per-lane source; rows past nrows_valid re-read the last valid
// row (their products are masked by the callers). 2 glds per thread (256 threads).
__device__ __forceinline__ void glds_tile(uint8_t* lds, const uint16_t* __restrict__ g, int64_t ld, int64_t row0,
                                          int nrows_valid, int col0) {
  const int wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = threadIdx.x + 256 * i, r = e >> 3, c = (e & 7) ^ (r & 7);
    const int row = min(r, nrows_valid - 1);
    __builtin_amdgcn_global_load_lds((const void*)(g + (row0 + row) * ld + col0 + c * 8),
                                     (lds_void*)(lds + (i * 256 + wid * 64) * 16), 16, 0, 0);
  }
}

// The same tile copy from a uniform row base (SGPRs) + a per-thread 32-bit byte offset computed
// once per kernel (glds_off_row): the ring kernels' per-stage address math was ~45 VALU (64-bit
// row * ld products for 5 DMAs) in a loop whose VALU issue bounds it; the SADDR form also costs
// one VGPR per DMA instead of two. `wu` is the wave index as a scalar (readfirstlane), so the LDS
// destinations (M0) need no per-DMA readfirstlane either. Full tiles only (no row clamp).
__device__ __forceinline__ void glds_tile2(uint8_t* lds, const uint16_t* rowbase, uint32_t o0, uint32_t o1, int wu) {
  const uint8_t* b = reinterpret_cast<const uint8_t*>(rowbase);
  __builtin_amdgcn_global_load_lds((const void*)(b + o0), (lds_void*)(lds + wu * 64 * 16), 16, 0, 0);
  __builtin_amdgcn_global_load_lds((const void*)(b + o1), (lds_void*)(lds + (256 + wu * 64) * 16), 16, 0, 0);
}
// byte offset of this thread's DMA i of glds_tile(lds, g, ld, row0, 64, col0) from g + row0 * ld + col0
__device__ __forceinline__ uint32_t glds_off_row(int64_t ld, int i) {
  const int e = threadIdx.x + 256 * i, r = e >> 3, c = (e & 7) ^ (r & 7);
  return (uint32_t)((r * ld + c * 8) * 2);
}

// ds_read_b64_tr_b16 as inline asm for the ring kernels: through the builtin, hipcc cannot tell
// the read from the in-flight LDS-DMA writes and puts an s_waitcnt vmcnt(0) in front of it, which
// drains the whole ring every step. The asm read is invisible to the compiler's waitcnt pass, so
// its consumers go through frag_tr_wait (lgkmcnt(0) + "+v" dependence + sched_barrier, rule 18).
__device__ __forceinline__ s16x4 ds_tr_asm(const uint8_t* lds) {
  s16x4 r;
  const uint32_t a = (uint32_t)reinterpret_cast<uintptr_t>((lds_s16x4*)lds);
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return r;
}
__device__ __forceinline__ bf16x8 frag_tr_asm(const uint8_t* lds, int r0, int r1, int col) {
  const int lane = threadIdx.x & 63, i = lane & 15, q = i >> 2, p = i & 3;
  const int cc = col + 4 * p, chunk = cc >> 3, half = (cc & 7) * 2;
  const s16x4 lo = ds_tr_asm(lds + tile_off(r0 + q, chunk) + half);
  const s16x4 hi = ds_tr_asm(lds + tile_off(r1 + q, chunk) + half);
  const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}
// the same read at a compile-time byte offset from `base` (the instruction's offset field): rows
// r0 and r0 + 16 of a tile_off image share their XOR swizzle (16 = 0 mod 8), so the hi half is
// the lo address + 2048, and tiles a constant number of bytes apart share one address register
template <int OFF>
__device__ __forceinline__ s16x4 ds_tr_asm_off(uint32_t a) {
  s16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "n"(OFF));
  return r;
}
template <int OFF>  // fragment of the tile at `lds` + OFF, rows r0 .. and r0 + 16 .. (see frag_tr_asm)
__device__ __forceinline__ bf16x8 frag_tr16_off(uint32_t a) {
  const s16x4 lo = ds_tr_asm_off<OFF>(a);
  const s16x4 hi = ds_tr_asm_off<OFF + 16 * 128>(a);
  const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}
// lane address of frag_tr_asm(lds, r0, r0 + 16, col) as a 32-bit LDS byte address
__device__ __forceinline__ uint32_t frag_tr_addr(const uint8_t* lds, int r0, int col) {
  const int lane = threadIdx.x & 63, i = lane & 15, q = i >> 2, p = i & 3;
  const int cc = col + 4 * p, chunk = cc >> 3, half = (cc & 7) * 2;
  return (uint32_t)reinterpret_cast<uintptr_t>((lds_s16x4*)(lds + tile_off(r0 + q, chunk) + half));
}
template <int N>
__device__ __forceinline__ void frag_tr_wait(bf16x8 (&f)[N]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int k = 0; k < N; ++k) asm volatile("" : "+v"(f[k]));
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void ring_wait(int after) {  // `after` stages issued after the wanted one
  if (after >= 2)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * 5) : "memory");
  else if (after == 1)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(5) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void ring_wait4(int after) {  // dQ ring: 4 glds per stage
  if (after >= 2)
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (after == 1)
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void raw_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}


// Column sums over a block's rows of per-lane output fragments v[d][r] (head dims d*16 + 4g + r,
// one row per lane i of each 16-lane group): xor-shuffles over the 16 rows of a group, then the 4
// waves through LDS (`red`: 256 floats, free). Threads 0..63 write dims 0..63 to out[0..63].
// The bias gradient of the QKV projection falls out of the attention backward this way, with no
// separate pass over dQKV.
__device__ __forceinline__ void block_colsum64(float (&v)[4][4], float* red, float* __restrict__ out) {
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15;
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) v[d][r] += __shfl_xor(v[d][r], off);
  if (i == 0) {
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wid * 64 + d * 16 + 4 * g + r] = v[d][r];
  }
  __syncthreads();
  if (threadIdx.x < 64)
    out[threadIdx.x] = (red[threadIdx.x] + red[64 + threadIdx.x]) + (red[128 + threadIdx.x] + red[192 + threadIdx.x]);
}

// q8 epilogue of a ring backward kernel (AttnQ8): NT tensors (dK, dV: 2; dQ: 1) of this block's
// NR = 64 * groups rows x 64 head dims. v[t][n][d][r] is the fp32 value of row n * 64 + wid * 16 + i,
// dim d * 16 + 4 g + r. Each value is rounded to bf16 first (what the bf16 store would hold), so y,
// yt and amax are bitwise those of fp8_cast_transpose over the bf16 dQKV. Row-major bytes go
// straight out (4 dims per lane, one dword); the transpose is staged through LDS (the ring's
// space, free after the loop) so that each thread stores 16-byte runs of rows. (Staging dwords after
// a 4 x 4 byte transpose inside each lane quad, DPP, instead of the byte writes measured slower:
// profiles/r6/fp8_attn_q8_dpp_ab.jsonl.)
// col0[t]: first column of tensor t in the packed 3D layout (+ h * 64); rows beyond S are skipped.
template <int NT, int NG>
__device__ __forceinline__ void attn_q8_epilogue(const AttnQ8& q8, const float (&v)[NT][NG][4][4], uint8_t* smem,
                                                 int64_t base, int row0, int S, int D, const int (&col0)[NT]) {
  constexpr int NR = 64 * NG, TP = NR + 16;  // rows per block; LDS pitch of a transposed row
  constexpr int YP = 64 + 16, YOFF = NT * 64 * TP;  // row-major image: pitch, offset (both 16-B multiples)
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15;
  const float sc = *q8.scale;
  const int64_t ld3 = 3 * (int64_t)D;
  float mx = 0.f;
  __syncthreads();  // every wave is past its last ring-stage read
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int n = 0; n < NG; ++n) {
      const int rl = n * 64 + wid * 16 + i, row = row0 + rl;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        float f[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          f[r] = __uint_as_float((unsigned)f32_to_bf16(v[t][n][d][r]) << 16);
          mx = row < S ? fmaxf(mx, fabsf(f[r])) : mx;
        }
        const uint32_t q = pack4_fp8<1>(f[0] * sc, f[1] * sc, f[2] * sc, f[3] * sc);
        *reinterpret_cast<uint32_t*>(smem + YOFF + (t * NR + rl) * YP + d * 16 + 4 * g) = q;
#pragma unroll
        for (int r = 0; r < 4; ++r) smem[(t * 64 + d * 16 + 4 * g + r) * TP + rl] = (uint8_t)(q >> (8 * r));
      }
    }
  __syncthreads();
  // the row-major bytes: each row's 64 head dims as four 16-byte pieces
  for (int e = threadIdx.x; e < NT * NR * 4; e += blockDim.x) {
    const int tr = e >> 2, c = e & 3, t = tr / NR, rl = tr - t * NR;
    if (row0 + rl < S)
      *reinterpret_cast<uint4*>(q8.y + (base + row0 + rl) * ld3 + col0[t] + 16 * c) =
          *reinterpret_cast<const uint4*>(smem + YOFF + tr * YP + 16 * c);
  }
  // NT x 64 transposed rows of NR bytes: 16-byte runs
  constexpr int RUNS = NR / 16;
  for (int e = threadIdx.x; e < NT * 64 * RUNS; e += blockDim.x) {
    const int tr = e / RUNS, c = e - tr * RUNS, t = tr >> 6, dim = tr & 63;
    if (row0 + 16 * c < S) {
      const uint4 w = *reinterpret_cast<const uint4*>(smem + tr * TP + 16 * c);
      *reinterpret_cast<uint4*>(q8.yt + (int64_t)(col0[t] + dim) * q8.ldt + base + row0 + 16 * c) = w;
    }
  }
  mx = wave_max(mx);
  float* red = reinterpret_cast<float*>(smem + YOFF + NT * NR * YP);
  if (lane == 0) red[wid] = mx;
  __syncthreads();
  if (threadIdx.x == 0) atomic_max_pos(q8.amax, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
  __syncthreads();  // (the caller's column-sum pass reuses the LDS)
}

// FULLT: S % 64 == 0 (every ring stage a whole tile: the clamped-row copy path is compiled out, which
// keeps the 2-group kernel within 256 VGPRs)
template <int NK, int kRing, bool FULLT>
__global__ __launch_bounds__(256, 2) void attn_bwd_dkdv_ring_kernel(const uint16_t* __restrict__ qkv,
                                                                 const uint16_t* __restrict__ dout,
                                                                 const float* __restrict__ lse,
                                                                 const float* __restrict__ delta,
                                                                 const int* __restrict__ lens,
                                                                 uint16_t* __restrict__ dqkv, int S, int H,
                                                                 float scale, float* __restrict__ colpart, AttnQ8 q8) {
  constexpr int STAGE = 2 * kTile + 2 * AB * 4;  // Q tile, dO tile, lse[64], delta[64]
  __shared__ __attribute__((aligned(16))) uint8_t smem[kRing * STAGE];
  int kbk, h, b;
  block_coords(S, 64 * NK, H, kbk, h, b);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15;
  const int D = H * AH;
  const int64_t ld = 3 * (int64_t)D;
  const int64_t base = (int64_t)b * S;
  const int len = lens ? lens[b] : S;
  const int k0b = kbk * (64 * NK);
  // column partials [B * key blocks][2 D] (dK | dV) of the bias gradient, or nullptr
  float* cp = colpart ? colpart + ((int64_t)b * ((S + 64 * NK - 1) / (64 * NK)) + kbk) * 2 * D + h * AH : nullptr;
  if (k0b >= len) {  // fully masked key block: zero gradients
    for (int e = threadIdx.x; e < 64 * NK * AH; e += 256) {
      const int kk = k0b + e / AH, d = e % AH;
      if (kk < S) {
        if (q8.y) {
          q8.y[(base + kk) * ld + D + h * AH + d] = 0;
          q8.y[(base + kk) * ld + 2 * D + h * AH + d] = 0;
          q8.yt[(int64_t)(D + h * AH + d) * q8.ldt + base + kk] = 0;
          q8.yt[(int64_t)(2 * D + h * AH + d) * q8.ldt + base + kk] = 0;
        } else {
          dqkv[(base + kk) * ld + D + h * AH + d] = 0;
          dqkv[(base + kk) * ld + 2 * D + h * AH + d] = 0;
        }
      }
    }
    if (cp && threadIdx.x < 64) {
      cp[threadIdx.x] = 0.f;
      cp[D + threadIdx.x] = 0.f;
    }
    return;
  }
  const float sl2 = scale * 1.4426950408889634f;
  const int nqb = (S + AB - 1) / AB;
  // stage = 5 glds per thread: 2 (Q) + 2 (dO) + 1 (waves 0/2: LSE row, waves 1/3: delta row);
  // full stages from sources computed once (advance q0 rows per stage), the partial last one clamped
  const int wu = __builtin_amdgcn_readfirstlane(wid);
  const uint32_t oq0 = glds_off_row(ld, 0), oq1 = glds_off_row(ld, 1);
  const uint32_t oo0 = glds_off_row((int64_t)D, 0), oo1 = glds_off_row((int64_t)D, 1);
  const uint32_t ol = (uint32_t)lane * ((wu & 1) ? (uint32_t)H * 4u : 4u);  // this lane's LSE / delta entry
  auto issue = [&](int slot, int qb) {
    uint8_t* st = smem + slot * STAGE;
    const int q0 = qb * AB, nv = min(AB, S - q0);
    if constexpr (FULLT) {
      glds_tile2(st, qkv + (base + q0) * ld + h * AH, oq0, oq1, wu);
      glds_tile2(st + kTile, dout + (base + q0) * (int64_t)D + h * AH, oo0, oo1, wu);
      const float* rb = (wu & 1) ? delta + (base + q0) * H + h : lse + ((int64_t)b * H + h) * S + q0;
      __builtin_amdgcn_global_load_lds((const void*)(reinterpret_cast<const uint8_t*>(rb) + ol),
                                       (lds_void*)(st + 2 * kTile + (wu & 1) * AB * 4), 4, 0, 0);
      return;
    }
    glds_tile(st, qkv, ld, base + q0, nv, h * AH);
    glds_tile(st + kTile, dout, (int64_t)D, base + q0, nv, h * AH);
    const int qq = q0 + min(lane, nv - 1);
    const float* src = (wid & 1) ? delta + (base + qq) * H + h : lse + ((int64_t)b * H + h) * S + qq;
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(st + 2 * kTile + (wid & 1) * AB * 4), 4, 0, 0);
  };
  int key[NK];
  bf16x8 kf[NK][2], vf[NK][2];
#pragma unroll
  for (int n = 0; n < NK; ++n) {
    key[n] = k0b + n * 64 + wid * 16 + i;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      kf[n][kh] = key[n] < S ? *reinterpret_cast<const bf16x8*>(qkv + (base + key[n]) * ld + D + h * AH + kh * 32 + 8 * g)
                             : bf16x8{};
      vf[n][kh] = key[n] < S
                      ? *reinterpret_cast<const bf16x8*>(qkv + (base + key[n]) * ld + 2 * D + h * AH + kh * 32 + 8 * g)
                      : bf16x8{};
    }
  }
  const bool kfull = k0b + 64 * NK <= len;  // block-uniform: no key of this block is masked
  float sl2k[NK], kinf[NK];  // masked keys: scale 0 and +inf shift -> exp2(-inf) = 0
#pragma unroll
  for (int n = 0; n < NK; ++n) {
    sl2k[n] = key[n] < len ? sl2 : 0.f;
    kinf[n] = key[n] < len ? 0.f : INFINITY;
  }
  // the ring prologue goes out after the register loads above, so waiting for those is a
  // counted vmcnt that leaves the DMAs in flight
#pragma unroll
  for (int s0 = 0; s0 < kRing - 1; ++s0)
    if (s0 < nqb) issue(s0, s0);
  f32x4 dk[NK][4], dv[NK][4];
#pragma unroll
  for (int n = 0; n < NK; ++n)
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      dk[n][d] = f32x4{0.f, 0.f, 0.f, 0.f};
      dv[n][d] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  for (int qb = 0; qb < nqb; ++qb) {
    ring_wait(min(kRing - 2, nqb - 1 - qb));
    raw_barrier();  // stage qb visible to all waves; everyone is done with slot (qb - 1) % kRing
    if (qb + kRing - 1 < nqb) issue((qb + kRing - 1) % kRing, qb + kRing - 1);
    const uint8_t* Qs = smem + (qb % kRing) * STAGE;
    const uint8_t* Os = Qs + kTile;
    const float* lse_s = reinterpret_cast<const float*>(Qs + 2 * kTile);
    const float* del_s = lse_s + AB;
    const int q0 = qb * AB;
    const bool qfull = q0 + AB <= S;
    // P and dS leave the fp32 accumulators as bf16 MFMA operands as soon as a qt pair is done
    // (half the registers of keeping all four qt tiles in fp32), and the block-uniform score-path
    // choice is taken once outside the qt loop, so each path's qt iterations are ONE basic block in
    // which one tile's MFMAs interleave with the previous tile's exp / dS VALU work
    bf16x8 pbk[NK][2], sbk[NK][2];
    auto qtiles = [&](auto pathc) __attribute__((always_inline)) {
      constexpr int PATH = decltype(pathc)::value;  // 0 all valid, 1 key mask, 2 key + query mask
      f32x4 pe[NK], dse[NK];  // the even qt of the current pair
#pragma unroll
      for (int qt = 0; qt < 4; ++qt) {
        // dP accumulates onto -delta (the MFMA's C operand), so dS = P * dP' needs no subtraction
        const float4 d4 = *reinterpret_cast<const float4*>(del_s + qt * 16 + 4 * g);
        const f32x4 ndr = {-d4.x, -d4.y, -d4.z, -d4.w};
        f32x4 sv[NK], dp[NK];
#pragma unroll
        for (int n = 0; n < NK; ++n) {
          sv[n] = f32x4{0.f, 0.f, 0.f, 0.f};
          dp[n] = ndr;
        }
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
          const bf16x8 qa = frag_row(Qs, qt * 16, kh), oa = frag_row(Os, qt * 16, kh);
#pragma unroll
          for (int n = 0; n < NK; ++n) {
            sv[n] = mfma(qa, kf[n][kh], sv[n]);
            dp[n] = mfma(oa, vf[n][kh], dp[n]);
          }
        }
        const float4 l4 = *reinterpret_cast<const float4*>(lse_s + qt * 16 + 4 * g);
        const float lr[4] = {l4.x, l4.y, l4.z, l4.w};
        f32x4 pc[NK], dsc[NK];
        if constexpr (PATH == 0 && MLT_ATTN_PKF32) {
          const f32x2 nl01 = {-lr[0], -lr[1]}, nl23 = {-lr[2], -lr[3]};
#pragma unroll
          for (int n = 0; n < NK; ++n) {
            f32x2 pa, pb, da, db;
            pk_prob_ds(sv[n], dp[n], sl2, nl01, 0, pa, da);
            pk_prob_ds(sv[n], dp[n], sl2, nl23, 2, pb, db);
            pc[n] = f32x4{pa.x, pa.y, pb.x, pb.y};
            dsc[n] = f32x4{da.x, da.y, db.x, db.y};
          }
        } else {
#pragma unroll
        for (int n = 0; n < NK; ++n)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float pv;
            if constexpr (PATH == 0) {  // every key of the block valid: x = s * sl2 - lse (one fma per score)
              pv = fast_exp2(sv[n][r] * sl2 - lr[r]);
            } else if constexpr (PATH == 1) {  // key mask folded into per-lane constants
              pv = fast_exp2(sv[n][r] * sl2k[n] - (lr[r] + kinf[n]));
            } else {
              const int ql = qt * 16 + 4 * g + r;
              const bool ok = key[n] < len && q0 + ql < S;
              pv = fast_exp2(ok ? sv[n][r] * sl2 - lr[r] : -INFINITY);
            }
            pc[n][r] = pv;
            dsc[n][r] = pv * dp[n][r];
          }
        }
#pragma unroll
        for (int n = 0; n < NK; ++n) {
          if (qt & 1) {
            pbk[n][qt >> 1] = pack_acc(pe[n], pc[n]);
            sbk[n][qt >> 1] = pack_acc(dse[n], dsc[n]);
          } else {
            pe[n] = pc[n];
            dse[n] = dsc[n];
          }
        }
      }
    };
    if (qfull && kfull)
      qtiles(std::integral_constant<int, 0>{});
    else if (qfull)
      qtiles(std::integral_constant<int, 1>{});
    else
      qtiles(std::integral_constant<int, 2>{});
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 pb[NK], sb[NK];
#pragma unroll
      for (int n = 0; n < NK; ++n) {
        pb[n] = pbk[n][ks];
        sb[n] = sbk[n][ks];
      }
      bf16x8 tf[8];  // dO^T (d = 0..3), Q^T (d = 0..3)
#pragma unroll
      for (int d = 0; d < 4; ++d) {  // Q^T and dO^T (kTile bytes further) from one address
        const uint32_t a = frag_tr_addr(Qs, 32 * ks + 4 * g, d * 16);
        tf[d] = frag_tr16_off<kTile>(a);
        tf[4 + d] = frag_tr16_off<0>(a);
      }
      frag_tr_wait(tf);
#pragma unroll
      for (int d = 0; d < 4; ++d) {
#pragma unroll
        for (int n = 0; n < NK; ++n) {
          dv[n][d] = mfma(tf[d], pb[n], dv[n][d]);
          dk[n][d] = mfma(tf[4 + d], sb[n], dk[n][d]);
        }
      }
    }
  }
  if (q8.y) {  // fp8 training: e5m2 dK | dV and their transposes instead of the bf16 dQKV
    float v[2][NK][4][4];
#pragma unroll
    for (int n = 0; n < NK; ++n)
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[0][n][d][r] = dk[n][d][r] * scale;
          v[1][n][d][r] = dv[n][d][r];
        }
    const int col0[2] = {D + h * AH, 2 * D + h * AH};
    attn_q8_epilogue<2, NK>(q8, v, smem, base, k0b, S, D, col0);
  } else {
#pragma unroll
  for (int n = 0; n < NK; ++n) {
    if (key[n] < S) {
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        uint16_t* kp = dqkv + (base + key[n]) * ld + D + h * AH + d * 16 + 4 * g;
        uint16_t* vp = dqkv + (base + key[n]) * ld + 2 * D + h * AH + d * 16 + 4 * g;
        ushort4 uk, uv;
        uk.x = f32_to_bf16(dk[n][d][0] * scale);
        uk.y = f32_to_bf16(dk[n][d][1] * scale);
        uk.z = f32_to_bf16(dk[n][d][2] * scale);
        uk.w = f32_to_bf16(dk[n][d][3] * scale);
        uv.x = f32_to_bf16(dv[n][d][0]);
        uv.y = f32_to_bf16(dv[n][d][1]);
        uv.z = f32_to_bf16(dv[n][d][2]);
        uv.w = f32_to_bf16(dv[n][d][3]);
        *reinterpret_cast<ushort4*>(kp) = uk;
        *reinterpret_cast<ushort4*>(vp) = uv;
      }
    }
  }
  }
  if (cp) {  // bias-gradient partials of dK and dV over this block's keys
    float vk[4][4], vv[4][4];
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        vk[d][r] = 0.f;
        vv[d][r] = 0.f;
#pragma unroll
        for (int n = 0; n < NK; ++n) {
          vk[d][r] += key[n] < S ? dk[n][d][r] * scale : 0.f;
          vv[d][r] += key[n] < S ? dv[n][d][r] : 0.f;
        }
      }
    float* red = reinterpret_cast<float*>(smem);
    __syncthreads();  // every wave is past its last ring-stage read
    block_colsum64(vk, red, cp);
    block_colsum64(vv, red + 256, cp + D);
  }
}

// The dQ ring kernel runs FIRST and computes delta = rowsum(dO * O) for its own queries in its
// prologue (dO is in its registers anyway; O is one more 16-byte load per fragment), publishing it
// for the dK/dV kernel that follows -- no separate delta pass over dO and O.
template <int NQ, int kRing, bool FULLT>
__global__ __launch_bounds__(256) void attn_bwd_dq_ring_kernel(const uint16_t* __restrict__ qkv,
                                                               const uint16_t* __restrict__ dout,
                                                               const uint16_t* __restrict__ out,
                                                               const float* __restrict__ lse,
                                                               float* __restrict__ delta,
                                                               const int* __restrict__ lens,
                                                               uint16_t* __restrict__ dqkv, int S, int H, float scale,
                                                               float* __restrict__ colpart, AttnQ8 q8) {
  constexpr int STAGE = 2 * kTile;  // K tile, V tile
  __shared__ __attribute__((aligned(16))) uint8_t smem[kRing * STAGE];
  int qb, h, b;
  block_coords(S, 64 * NQ, H, qb, h, b);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15;
  (void)lane;
  const int D = H * AH;
  const int64_t ld = 3 * (int64_t)D;
  const int64_t base = (int64_t)b * S;
  const int len = lens ? lens[b] : S;
  const float sl2 = scale * 1.4426950408889634f;
  const int nkb = (len + AB - 1) / AB;
  const int wu = __builtin_amdgcn_readfirstlane(wid);
  const uint32_t ok0 = glds_off_row(ld, 0), ok1 = glds_off_row(ld, 1);
  auto issue = [&](int slot, int kb) {  // (K and V: the same rows, D columns apart)
    uint8_t* st = smem + slot * STAGE;
    const int k0 = kb * AB, nv = min(AB, S - k0);
    if constexpr (FULLT) {
      const uint16_t* kr = qkv + (base + k0) * ld + D + h * AH;
      glds_tile2(st, kr, ok0, ok1, wu);
      glds_tile2(st + kTile, kr + D, ok0, ok1, wu);
      return;
    }
    glds_tile(st, qkv, ld, base + k0, nv, D + h * AH);
    glds_tile(st + kTile, qkv, ld, base + k0, nv, 2 * D + h * AH);
  };
  int q[NQ];
  bf16x8 qf[NQ][2], of[NQ][2];
  float lq[NQ], dl[NQ];
  f32x4 acc[NQ][4];
#pragma unroll
  for (int n = 0; n < NQ; ++n) {
    q[n] = qb * (64 * NQ) + n * 64 + wid * 16 + i;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      qf[n][kh] = q[n] < S ? *reinterpret_cast<const bf16x8*>(qkv + (base + q[n]) * ld + h * AH + kh * 32 + 8 * g)
                           : bf16x8{};
      of[n][kh] = q[n] < S
                      ? *reinterpret_cast<const bf16x8*>(dout + (base + q[n]) * (int64_t)D + h * AH + kh * 32 + 8 * g)
                      : bf16x8{};
    }
    lq[n] = q[n] < S ? lse[((int64_t)b * H + h) * S + q[n]] : 0.f;
    {  // delta of query q[n], bit-identical to attn_delta_kernel: its 16 four-dim partials (dims 4 sub ..)
       // are this lane's (kh, half) quads, sub = 8 kh + 2 g + half, summed in group_sum<16>'s
       // butterfly order (xor 8 = kh in-lane, xor 4 = lane ^ 32, xor 2 = lane ^ 16, xor 1 = half)
      float s4[2][2];
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        const bf16x8 o8 = q[n] < S ? *reinterpret_cast<const bf16x8*>(out + (base + q[n]) * (int64_t)D + h * AH +
                                                                        kh * 32 + 8 * g)
                                   : bf16x8{};
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          const int j = 4 * hf;
          s4[kh][hf] = (float)of[n][kh][j] * (float)o8[j] + (float)of[n][kh][j + 1] * (float)o8[j + 1] +
                       (float)of[n][kh][j + 2] * (float)o8[j + 2] + (float)of[n][kh][j + 3] * (float)o8[j + 3];
        }
      }
      float w[2];
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        float v = s4[0][hf] + s4[1][hf];
        v += __shfl_xor(v, 32, 64);
        v += __shfl_xor(v, 16, 64);
        w[hf] = v;
      }
      const float sacc = w[0] + w[1];
      dl[n] = q[n] < S ? sacc : 0.f;
      if (g == 0 && q[n] < S) delta[(base + q[n]) * H + h] = sacc;
    }
#pragma unroll
    for (int d = 0; d < 4; ++d) acc[n][d] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int s0 = 0; s0 < kRing - 1; ++s0)
    if (s0 < nkb) issue(s0, s0);
  for (int kb = 0; kb < nkb; ++kb) {
    ring_wait4(min(kRing - 2, nkb - 1 - kb));
    raw_barrier();
    if (kb + kRing - 1 < nkb) issue((kb + kRing - 1) % kRing, kb + kRing - 1);
    const uint8_t* Ks = smem + (kb % kRing) * STAGE;
    const uint8_t* Vs = Ks + kTile;
    const bool kfull = (kb + 1) * AB <= len;
    f32x4 ds[NQ][4];
    // mask-path choice hoisted out of the kt loop (block-uniform): one basic block per path, so
    // MFMAs and the exp / dS VALU work of neighbouring kt tiles interleave (see the dK/dV kernel)
    auto ktiles = [&](auto fullc) __attribute__((always_inline)) {
      constexpr bool FULL = decltype(fullc)::value;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        f32x4 sv[NQ], dp[NQ];
#pragma unroll
        for (int n = 0; n < NQ; ++n) {  // dP accumulates onto -delta: dS = P * dP'
          sv[n] = f32x4{0.f, 0.f, 0.f, 0.f};
          dp[n] = f32x4{-dl[n], -dl[n], -dl[n], -dl[n]};
        }
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
          const bf16x8 ka = frag_row(Ks, kt * 16, kh), va = frag_row(Vs, kt * 16, kh);
#pragma unroll
          for (int n = 0; n < NQ; ++n) {
            sv[n] = mfma(ka, qf[n][kh], sv[n]);
            dp[n] = mfma(va, of[n][kh], dp[n]);
          }
        }
        if constexpr (FULL && MLT_ATTN_PKF32) {
#pragma unroll
          for (int n = 0; n < NQ; ++n) {
            const f32x2 nl = {-lq[n], -lq[n]};
            f32x2 pa, pb, da, db;
            pk_prob_ds(sv[n], dp[n], sl2, nl, 0, pa, da);
            pk_prob_ds(sv[n], dp[n], sl2, nl, 2, pb, db);
            ds[n][kt] = f32x4{da.x, da.y, db.x, db.y};
          }
        } else
#pragma unroll
        for (int n = 0; n < NQ; ++n)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float pv;
            if constexpr (FULL) {  // every key of this block is valid
              pv = fast_exp2(sv[n][r] * sl2 - lq[n]);
            } else {
              const int key = kb * AB + kt * 16 + 4 * g + r;
              pv = fast_exp2(key < len ? sv[n][r] * sl2 - lq[n] : -INFINITY);
            }
            ds[n][kt][r] = pv * dp[n][r];
          }
      }
    };
    if (kfull)
      ktiles(std::true_type{});
    else
      ktiles(std::false_type{});
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 sb[NQ];
#pragma unroll
      for (int n = 0; n < NQ; ++n) sb[n] = pack_acc(ds[n][2 * ks], ds[n][2 * ks + 1]);
      bf16x8 tf[4];
#pragma unroll
      for (int d = 0; d < 4; ++d) tf[d] = frag_tr16_off<0>(frag_tr_addr(Ks, 32 * ks + 4 * g, d * 16));
      frag_tr_wait(tf);
#pragma unroll
      for (int d = 0; d < 4; ++d) {
#pragma unroll
        for (int n = 0; n < NQ; ++n) acc[n][d] = mfma(tf[d], sb[n], acc[n][d]);
      }
    }
  }
  if (q8.y) {  // fp8 training: e5m2 dQ and its transpose instead of the bf16 dQKV
    float v[1][NQ][4][4];
#pragma unroll
    for (int n = 0; n < NQ; ++n)
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[0][n][d][r] = acc[n][d][r] * scale;
    const int col0[1] = {h * AH};
    attn_q8_epilogue<1, NQ>(q8, v, smem, base, qb * (64 * NQ), S, D, col0);
  } else {
#pragma unroll
  for (int n = 0; n < NQ; ++n) {
    if (q[n] < S) {
      uint16_t* qp = dqkv + (base + q[n]) * ld + h * AH;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        ushort4 u;
        u.x = f32_to_bf16(acc[n][d][0] * scale);
        u.y = f32_to_bf16(acc[n][d][1] * scale);
        u.z = f32_to_bf16(acc[n][d][2] * scale);
        u.w = f32_to_bf16(acc[n][d][3] * scale);
        *reinterpret_cast<ushort4*>(qp + d * 16 + 4 * g) = u;
      }
    }
  }
  }
  if (colpart) {  // bias-gradient partials of dQ over this block's queries: [B * query blocks][D]
    float vq[4][4];
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        vq[d][r] = 0.f;
#pragma unroll
        for (int n = 0; n < NQ; ++n) vq[d][r] += q[n] < S ? acc[n][d][r] * scale : 0.f;
      }
    __syncthreads();  // every wave is past its last ring-stage read
    block_colsum64(vq, reinterpret_cast<float*>(smem),
                   colpart + ((int64_t)b * ((S + 64 * NQ - 1) / (64 * NQ)) + qb) * D + h * AH);
  }
}

// 32 rows per wave (2 x 16-row groups) once the sequence fills a 128-row block.
// MLT_ATTN_FWD_GROUPS / MLT_ATTN_DKDV_GROUPS / MLT_ATTN_DQ_GROUPS = 1|2 override the choice
// Measured (B32 / B128, S512, H12): lean forward 2 groups (44.7 vs 49.7 us, 161 vs 185 us), dQ 2 groups. dK/dV: with the
// register-staged kernel 1 group (2 need > 256 VGPRs and halve the occupancy); with the ring
// kernels (the default) 2 groups, 10-14 % faster backward at B16..B128 (B32 198 -> 176 us,
// B128 727 -> 629 us: each Q / dO ring stage feeds twice the MFMAs).
static int attn_groups(const char* env, int S, int dflt = 2) {
  const char* v = getenv(env);
  if (v && (v[0] == '1' || v[0] == '2')) return S >= 128 ? v[0] - '0' : 1;
  return S >= 128 ? dflt : 1;
}

void launch_attn_fwd(const uint16_t* qkv, uint16_t* out, float* lse, const int* lens, int B, int S, int H,
                     float scale, hipStream_t st) {
  if (B <= 0 || S <= 0) return;
  const unsigned g2 = (unsigned)((S + 127) / 128 * H * B), g1 = (unsigned)((S + 63) / 64 * H * B);
  if (attn_groups("MLT_ATTN_FWD_GROUPS", S, 2) == 2)
    hipLaunchKernelGGL(attn_fwd_lean_kernel<2>, dim3(g2), dim3(256), 0, st, qkv, out, lse, lens, S, H, scale);
  else
    hipLaunchKernelGGL(attn_fwd_lean_kernel<1>, dim3(g1), dim3(256), 0, st, qkv, out, lse, lens, S, H, scale);
}

bool launch_attn_bwd(const uint16_t* qkv, const uint16_t* out, const uint16_t* dout, const float* lse, float* delta,
                     const int* lens, uint16_t* dqkv, int B, int S, int H, float scale, hipStream_t st,
                     float* colpart_q, float* colpart_kv, int* rows_q, int* rows_kv, const AttnQ8& q8) {
  if (B <= 0 || S <= 0) return false;
  const int64_t pairs = (int64_t)B * S * H;
  const dim3 g2((S + 127) / 128 * H * B), g1((S + 63) / 64 * H * B);
  // MLT_ATTN_RING: 0 = register-staged kernels, 3 / 4 = ring depth (default 4)
  const char* rv = getenv("MLT_ATTN_RING");
  const int ring = rv ? atoi(rv) : 4;
  if (ring == 3 || ring == 4) {
    const bool k2 = attn_groups("MLT_ATTN_DKDV_GROUPS", S, 2) == 2, q2 = attn_groups("MLT_ATTN_DQ_GROUPS", S) == 2;
#define MLT_RING_LAUNCH(RD, FL)                                                                                       \
  {                                                                                                                   \
    if (q2)                                                                                                           \
      hipLaunchKernelGGL((attn_bwd_dq_ring_kernel<2, RD, FL>), g2, dim3(256), 0, st, qkv, dout, out, lse, delta, lens, \
                         dqkv, S, H, scale, colpart_q, q8);                                                           \
    else                                                                                                              \
      hipLaunchKernelGGL((attn_bwd_dq_ring_kernel<1, RD, FL>), g1, dim3(256), 0, st, qkv, dout, out, lse, delta, lens, \
                         dqkv, S, H, scale, colpart_q, q8);                                                           \
    if (k2)                                                                                                           \
      hipLaunchKernelGGL((attn_bwd_dkdv_ring_kernel<2, RD, FL>), g2, dim3(256), 0, st, qkv, dout, lse, delta, lens,   \
                         dqkv, S, H, scale, colpart_kv, q8);                                                          \
    else                                                                                                              \
      hipLaunchKernelGGL((attn_bwd_dkdv_ring_kernel<1, RD, FL>), g1, dim3(256), 0, st, qkv, dout, lse, delta, lens,   \
                         dqkv, S, H, scale, colpart_kv, q8);                                                          \
  }
    const bool full = S % AB == 0;
    if (ring == 3) {
      if (full) MLT_RING_LAUNCH(3, true) else MLT_RING_LAUNCH(3, false)
    } else {
      if (full) MLT_RING_LAUNCH(4, true) else MLT_RING_LAUNCH(4, false)
    }
#undef MLT_RING_LAUNCH
    // partial rows actually written: B x (row blocks of the chosen group count)
    if (rows_kv) *rows_kv = B * ((S + (k2 ? 127 : 63)) / (k2 ? 128 : 64));
    if (rows_q) *rows_q = B * ((S + (q2 ? 127 : 63)) / (q2 ? 128 : 64));
    return colpart_q != nullptr && colpart_kv != nullptr;
  }
  if (q8.y) throw std::runtime_error("attn_bwd: the fp8 (q8) outputs need the ring kernels (MLT_ATTN_RING=3|4)");
  hipLaunchKernelGGL(attn_delta_kernel, dim3((unsigned)((pairs + 15) / 16)), dim3(256), 0, st, dout, out, delta,
                     (int64_t)B * S, H);
  if (attn_groups("MLT_ATTN_DKDV_GROUPS", S, 1) == 2)
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<2>, g2, dim3(256), 0, st, qkv, dout, lse, delta, lens, dqkv, S, H, scale);
  else
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<1>, g1, dim3(256), 0, st, qkv, dout, lse, delta, lens, dqkv, S, H, scale);
  if (attn_groups("MLT_ATTN_DQ_GROUPS", S) == 2)
    hipLaunchKernelGGL(attn_bwd_dq_kernel<2>, g2, dim3(256), 0, st, qkv, dout, lse, delta, lens, dqkv, S, H, scale);
  else
    hipLaunchKernelGGL(attn_bwd_dq_kernel<1>, g1, dim3(256), 0, st, qkv, dout, lse, delta, lens, dqkv, S, H, scale);
  return false;  // register-staged kernels: no column partials (the caller reduces dQKV itself)
}

}  // namespace mlt
