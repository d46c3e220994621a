// 4-wave 256x256x64 bf16 GEMM for gfx950 (planner cfg 7): C = A . B^T with A [M][K] k-contiguous and
// B [N][K] (forward layout of a linear layer) or B [K][N] (b_mn: the input-gradient layout, read
// through ds_read_b64_tr_b16), one output tile per 256-thread workgroup, ONE wave per SIMD holding
// a 128 x 128 wave tile in 256 AGPR accumulators.
//
// Why this shape (rocprofv3 --pmc on the box, profiles/r4/gemm_pmc_*.jsonl): at 8192^3 hipBLASLt's
// MT256x256x64 kernel runs 4 waves per workgroup and keeps the matrix cores busy 87.5 % of the
// cycles (SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x 4 SIMDs)), while the 8-wave ping-pong
// kernel (gemm_tile.hip, cfg 5: 2 waves per SIMD, 128 x 64 wave tiles, two barriers per 16-MFMA
// phase) reaches 67 % -- its waves sit parked at barriers / waitcnts 26 % of their cycles. A 128 x
// 128 wave tile reads 64 FLOP per LDS byte (43 for 128 x 64), and with one barrier per K-tile
// (2,048 MFMA cycles per SIMD) the fill / drain of the barrier is amortised over 128 MFMAs.
//
// The main loop is generated asm (scripts/gen_gemm_w4.py -> gemm_w4_loop.inc): fixed fragment
// registers v[0:127], accumulators a[0:255], DMA source pointers s[88:91]; fragment reads one per
// MFMA gap of a phase's first half, the LDS-DMA pieces one per 4 MFMAs over the second phase, the
// first K-tile's MFMAs start from C = 0. This file computes the per-lane addresses, runs the loop
// and applies the fused epilogue from the accumulators through a per-wave LDS image (16-byte row
// stores). MFMA operands are swapped (D = B_tile . A_tile^T): a lane holds 4 columns of one row.
// Requirements (host-checked, else the caller falls back): M, N multiples of 256, K a multiple of
// 128 and >= 256, 16-byte aligned rows, no split-K / accumulate / fp8 scales.
#include "mlt_common.h"
#include "mlt_fp8.h"
#include "mlt_gemm.h"
#include "mlt_gemm_tile.h"
#include "gemm_w4_loop.inc"

namespace mlt {


// W4_Q8GELU / W4_Q8DGELU: the quantising ("q8") epilogues of the fp8 FFN (OutT = fp8 bytes): GELU /
// dGELU as W4_GELU / W4_DGELU, then amax, scale, fp8 Y (e4m3 / e5m2) and fp8 Y^T from the same LDS image
enum W4Epi { W4_PLAIN = 0, W4_GELU = 1, W4_RES = 2, W4_DGELU = 3, W4_Q8GELU = 4, W4_Q8DGELU = 5 };
template <int EK>
constexpr bool w4_gel() { return EK == W4_GELU || EK == W4_Q8GELU; }
template <int EK>
constexpr bool w4_dgel() { return EK == W4_DGELU || EK == W4_Q8DGELU; }
template <int EK>
constexpr bool w4_q8() { return EK == W4_Q8GELU || EK == W4_Q8DGELU; }

typedef __attribute__((address_space(3))) uint8_t lds_u8;
// LDS: two K-tile stages of 64 KB; after the loop, four per-wave 64 x 132 fp32 epilogue images
__device__ __forceinline__ uint32_t pack2(uint16_t lo, uint16_t hi) { return (uint32_t)lo | ((uint32_t)hi << 16); }
constexpr int kW4Pitch = 132, kW4Smem = 4 * 64 * kW4Pitch * 4 > 131072 ? 4 * 64 * kW4Pitch * 4 : 131072;

// GELU / GELU' of the (b)GELU epilogues from exact tables at the bf16 input points (scripts/
// gen_gelu_table.py: layout, accuracy, why) instead of the A&S erf of mlt_gemm.h; the table sits in
// LDS behind the epilogue images (158,736 B of the 160 KB). Build switch -DMLT_W4_GELU_TAB=0: the
// erf polynomial. Same-box A/B at 256 K tokens (profiles/r5/gemm_gelu_tab_attn_pkf32_ab.jsonl): bias +
// GELU 832 -> 862-870 TF, dGELU 839-842 -> 914-917, dGELU + column sums 809-812 -> 880-887 (plain
// epilogue 1,097-1,107); BERT-base 3,038-3,040 -> 3,070-3,074 samples/s.
#ifndef MLT_W4_GELU_TAB
#define MLT_W4_GELU_TAB 1
#endif
template <int EK>
constexpr bool w4_gelu_tab() {
  return MLT_W4_GELU_TAB && (w4_gel<EK>() || w4_dgel<EK>());
}
template <int EK>
constexpr int w4_smem() {
  return kW4Smem + (w4_gelu_tab<EK>() ? kGeluTabBytes : 0);
}
static_assert(kW4Smem + kGeluTabBytes <= 160 * 1024, "GELU table must fit beside the epilogue images");
// workgroup copy of the epilogue's table into LDS (read only after the epilogue's first barrier)
template <int EK>
__device__ __forceinline__ void w4_load_gelu_tab(uint8_t* smem) {
  if constexpr (w4_gelu_tab<EK>()) gelu_tab_load(smem + kW4Smem, w4_dgel<EK>(), 256);
}

// ---- epilogue through LDS: a lane's accumulator fragment holds 4 columns of one row, so direct
// stores would be 64 x 8 bytes per lane in 32-byte row pieces (store-issue bound). Each wave
// instead writes its 128 x 128 fp32 tile to its own LDS image in two 64-row halves (pitch 132
// floats: the 16 rows of a fragment write land 4 banks apart) and reads it back as 8 consecutive
// columns per lane: 32 x 16-byte stores per lane (bf16), side operands as 16-byte loads.
template <typename OutT, int EK>
__device__ __forceinline__ void w4_epilogue(OutT* __restrict__ C, int64_t ldc, const GemmEpi& epi, float alpha, int m0,
                                            int n0, int N, int w, int lane, uint8_t* smem) {
  const int wr = w >> 1, wc = w & 1, g = lane >> 4, rl = lane & 15;
  __syncthreads();  // every wave is past its last read of the K-tile stages
  constexpr int P = kW4Pitch;
  float* img = reinterpret_cast<float*>(smem) + w * 64 * P;
  const int rsub = lane >> 4, cc = lane & 15;  // read side: row 4 * it + rsub, columns 8 cc .. + 7
  constexpr int QF = EK == W4_Q8DGELU ? 1 : 0;  // q8 output format: e4m3 (GELU: FFN2's input) / e5m2 (dGELU: a dY)
  float q_amx = 0.f, q_s = 1.f;
  if constexpr (w4_q8<EK>()) q_s = *epi.q_scale;
  const int gn = n0 + wc * 128 + 8 * cc;
  float bs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bs[e] = 0.f;
  if (epi.bias) {
    const float4 b0 = *reinterpret_cast<const float4*>(epi.bias + gn);
    const float4 b1 = *reinterpret_cast<const float4*>(epi.bias + gn + 4);
    bs[0] = b0.x, bs[1] = b0.y, bs[2] = b0.z, bs[3] = b0.w, bs[4] = b1.x, bs[5] = b1.y, bs[6] = b1.z, bs[7] = b1.w;
  }
  // side operands: the residual of BOTH halves issued first (one HBM round trip under the image
  // writes instead of one per half); the dGELU pre-activation per half -- with the column partials
  // beside it, both halves' 128 registers would push the kernel past 256 VGPRs into spills to AGPRs,
  // which hold the not-yet-read accumulators (scripts/check_w4_agpr.py guards every build)
  constexpr int SH = EK == W4_RES ? 2 : 1;
  uint4 sd[SH][16];
  // (the quantising dGELU form loads them in two 8-row batches, its row loop unrolled by 8 to match:
  // fully unrolled, the compiler spilled 108-207 values into the accumulator AGPRs)
  constexpr int SB = EK == W4_Q8DGELU ? 8 : 16;
  auto side_loads = [&](int h, uint4 (&dst)[16], int it0 = 0) __attribute__((always_inline)) {
    const uint16_t* sx = EK == W4_RES ? epi.res : epi.aux;
    const int64_t ldx = EK == W4_RES ? epi.ldres : epi.ldaux;
#pragma unroll
    for (int i = 0; i < SB; ++i) {
      const int it = it0 + i;
      const int gm = m0 + wr * 128 + 64 * h + 4 * it + rsub;
      dst[i] = *reinterpret_cast<const uint4*>(sx + (int64_t)gm * ldx + gn);
    }
  };
  if constexpr (EK == W4_RES) {
    side_loads(0, sd[0]);
    side_loads(1, sd[SH - 1]);
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    // the half's 32 fragments -> image rows 16 i + rl, columns 16 j + 4 g (ds_write from the AGPRs)
    const uint32_t va = (uint32_t)(uintptr_t)(lds_u8*)(smem + 4 * (w * 64 * P + rl * P + 4 * g));
    if (h == 0)
      asm volatile(MLT_W4_IMG_H0 ::[va] "v"(va) : "memory");
    else
      asm volatile(MLT_W4_IMG_H1 ::[va] "v"(va) : "memory");
    if constexpr (w4_dgel<EK>()) side_loads(h, sd[0]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own image: no barrier needed
    float csum[8];  // dGELU + q_colpart: the half's column sums (bias gradient of the dGELU output)
#pragma unroll
    for (int e = 0; e < 8; ++e) csum[e] = 0.f;
#pragma unroll SB
    for (int it = 0; it < 16; ++it) {
      const int row = 4 * it + rsub, gm = m0 + wr * 128 + 64 * h + row;
      if constexpr (SB < 16) {
        if (it > 0 && it % SB == 0) side_loads(h, sd[0], it);
      }
      const float4 lo = *reinterpret_cast<const float4*>(img + row * P + 8 * cc);
      const float4 hi = *reinterpret_cast<const float4*>(img + row * P + 8 * cc + 4);
      float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = v[e] * alpha + bs[e];
      if constexpr (w4_gel<EK>()) {  // keep the (bf16-rounded) pre-activation for the backward
        uint32_t a[4];                // (two-wide GELU: this epilogue is VALU-bound, mlt_gemm.h)
        f32x2 x2[4];
#pragma unroll
        for (int q2 = 0; q2 < 4; ++q2) {
          a[q2] = cvt_pk_bf16(f32x2{v[2 * q2], v[2 * q2 + 1]});
          x2[q2] = unpack_bf16x2(a[q2]);
        }
        *reinterpret_cast<uint4*>(const_cast<uint16_t*>(epi.aux) + (int64_t)gm * epi.ldaux + gn) =
            make_uint4(a[0], a[1], a[2], a[3]);
        if constexpr (w4_gelu_tab<EK>()) {
#pragma unroll
          for (int q2 = 0; q2 < 4; ++q2) x2[q2] = x2[q2] * gelu_tab2(a[q2], smem + kW4Smem);
        } else {
          gelu2<4>(x2);
        }
#pragma unroll
        for (int q2 = 0; q2 < 4; ++q2) v[2 * q2] = x2[q2].x, v[2 * q2 + 1] = x2[q2].y;
      } else if constexpr (w4_dgel<EK>()) {
        const uint4 sv = sd[0][it % SB];
        f32x2 x2[4];
        if constexpr (w4_gelu_tab<EK>()) {
          const uint32_t sw4[4] = {sv.x, sv.y, sv.z, sv.w};
#pragma unroll
          for (int q2 = 0; q2 < 4; ++q2) x2[q2] = gelu_tab2(sw4[q2], smem + kW4Smem);
        } else {
          x2[0] = unpack_bf16x2(sv.x), x2[1] = unpack_bf16x2(sv.y), x2[2] = unpack_bf16x2(sv.z);
          x2[3] = unpack_bf16x2(sv.w);
          gelu_grad2<4>(x2);
        }
#pragma unroll
        for (int q2 = 0; q2 < 4; ++q2) {
          const f32x2 gv = f32x2{v[2 * q2], v[2 * q2 + 1]} * x2[q2];
          v[2 * q2] = gv.x, v[2 * q2 + 1] = gv.y;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) csum[e] += v[e];
      } else if constexpr (EK == W4_RES) {
        const uint4 sv = sd[h][it];
        const uint32_t sw4[4] = {sv.x, sv.y, sv.z, sv.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += bf16_to_f32((uint16_t)(sw4[e >> 1] >> (16 * (e & 1))));
      }
      if constexpr (w4_q8<EK>()) {
        // amax of the unscaled output, then the SCALED values: fp8 row store, and back into the
        // image for the transposed pass below
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          q_amx = fmaxf(q_amx, fabsf(v[e]));
          v[e] *= q_s;
        }
        *reinterpret_cast<float4*>(img + row * P + 8 * cc) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(img + row * P + 8 * cc + 4) = make_float4(v[4], v[5], v[6], v[7]);
        *reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(C) + (int64_t)gm * ldc + gn) =
            make_uint2(pack4_fp8<QF>(v[0], v[1], v[2], v[3]), pack4_fp8<QF>(v[4], v[5], v[6], v[7]));
        continue;
      }
      OutT* cp = C + (int64_t)gm * ldc + gn;
      if constexpr (sizeof(OutT) == 4) {
        *reinterpret_cast<float4*>(cp) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(cp + 4) = make_float4(v[4], v[5], v[6], v[7]);
      } else {
        *reinterpret_cast<uint4*>(cp) =
            make_uint4(cvt_pk_bf16(f32x2{v[0], v[1]}), cvt_pk_bf16(f32x2{v[2], v[3]}),
                       cvt_pk_bf16(f32x2{v[4], v[5]}), cvt_pk_bf16(f32x2{v[6], v[7]}));
      }
    }
    if constexpr (w4_dgel<EK>()) {
      if (epi.q_colpart) {  // the 4 lanes of a column group (rsub) hold 16 rows each: one 64-row block
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          csum[e] += __shfl_xor(csum[e], 16);
          csum[e] += __shfl_xor(csum[e], 32);
        }
        if (rsub == 0) {
          float* cp = epi.q_colpart + (int64_t)((m0 + wr * 128 + 64 * h) >> 6) * N + gn;
          *reinterpret_cast<float4*>(cp) = make_float4(csum[0], csum[1], csum[2], csum[3]);
          *reinterpret_cast<float4*>(cp + 4) = make_float4(csum[4], csum[5], csum[6], csum[7]);
        }
      }
    }
    if constexpr (w4_q8<EK>()) {
      // Y^T: per pass p, lane (kq = lane / 16, cq = lane % 16) takes columns 32 p + 2 cq, + 1 and
      // rows 16 kq .. + 15 of the half's image: one 16-byte store per column, the 4 kq lanes of a
      // column covering its 64 contiguous bytes of the consumer's k-contiguous operand
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the row pass's image writes (this wave's own)
      const int kq = lane >> 4, cq = lane & 15;
      const int qoff = 2 * cq * (int)epi.ldqt + 16 * kq;  // the lane's part: a 32-bit offset off a wave-uniform base
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const float* cimg = img + (16 * kq) * P + 32 * p + 2 * cq;
        uint8_t* const qt0 = epi.qt + (int64_t)(n0 + wc * 128 + 32 * p) * epi.ldqt + (m0 + wr * 128 + 64 * h) + qoff;
        uint32_t w0[4], w1[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float2 x0 = *reinterpret_cast<const float2*>(cimg + (4 * k + 0) * P);
          const float2 x1 = *reinterpret_cast<const float2*>(cimg + (4 * k + 1) * P);
          const float2 x2 = *reinterpret_cast<const float2*>(cimg + (4 * k + 2) * P);
          const float2 x3 = *reinterpret_cast<const float2*>(cimg + (4 * k + 3) * P);
          w0[k] = pack4_fp8<QF>(x0.x, x1.x, x2.x, x3.x);
          w1[k] = pack4_fp8<QF>(x0.y, x1.y, x2.y, x3.y);
        }
        *reinterpret_cast<uint4*>(qt0) = make_uint4(w0[0], w0[1], w0[2], w0[3]);
        *reinterpret_cast<uint4*>(qt0 + epi.ldqt) = make_uint4(w1[0], w1[1], w1[2], w1[3]);
      }
    }
    if (h == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the image is rewritten
  }
  if constexpr (w4_q8<EK>()) {  // this wave's amax into the output's slots
    q_amx = wave_max(q_amx);
    if (lane == 0) atomic_max_pos(epi.q_amax, q_amx);
  }
}

// AN / BN: A stored [K][M] / B stored [K][N] (mn-contiguous: weight-gradient / input-gradient
// layouts, read through ds_read_b64_tr_b16); nkt = this workgroup's K-tiles (even, >= 4), kz = its
// first K element (split-K)
template <typename OutT, int EK, bool AN, bool BN>
__device__ __forceinline__ void gemm_w4_tile(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                             OutT* __restrict__ C, int nkt, int64_t kz, int64_t lda, int64_t ldb,
                                             int64_t ldc, const GemmEpi& epi, int id, int gm_, int tiles_m, int tiles_n,
                                             uint8_t* smem) {
  const int per_group = gm_ * tiles_n, grp = id / per_group, first_m = grp * gm_;
  const int gsize = min(tiles_m - first_m, gm_), rr = id - grp * per_group;
  const int m0 = (first_m + rr % gsize) * 256, n0 = (rr / gsize) * 256;

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 1, wc = w & 1;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_u8*)smem;

  // fragment reads: lane (g, rl) of a 16-row block reads row rl, 16-B chunk kh*4 + g, stored at
  // chunk ^ ((row >> 1) & 7) (rows 128 B apart; the XOR spreads a 16-lane group over all 64 banks)
  const int g = lane >> 4, rl = lane & 15, sw = (rl >> 1) & 7;
  auto raddr = [&](int stage, int isb, int kh) {
    const int row = (isb ? wc : wr) * 128 + rl;
    return lds0 + stage * 65536 + isb * 32768 + row * 128 + (((kh * 4 + g) ^ sw) << 4);
  };
  const uint32_t ra00 = raddr(0, 0, 0), ra01 = raddr(0, 0, 1), ra10 = raddr(1, 0, 0), ra11 = raddr(1, 0, 1);
  const uint32_t rb00 = raddr(0, 1, 0), rb01 = raddr(0, 1, 1), rb10 = raddr(1, 1, 0), rb11 = raddr(1, 1, 1);
  // DMA sources: wave w's p-th piece fills 1 KB of the image (lane-linear). k-contiguous image
  // [256 rows][128 B]: rows (4p + w) * 8 .. + 7, lane L fetches row + (L >> 3), the global chunk that
  // lands on position L & 7 under the swizzle. mn-contiguous image [64 k][256 mn]: 32 chunks per
  // 512-B k-row, chunk ^ (2 (k & 3) + 8 ((k >> 3) & 1)) (conflict-free transposed reads).
  uint32_t ga[8], gb[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int r = (p * 4 + w) * 8 + (lane >> 3);
    const int kc = (lane & 7) ^ ((r >> 1) & 7);
    const int e = (p * 4 + w) * 64 + lane, kk = e >> 5;
    const int c = (e & 31) ^ (((kk & 3) << 1) | (((kk >> 3) & 1) << 3));
    ga[p] = AN ? (uint32_t)((kk * lda + c * 8) * 2) : (uint32_t)((r * lda + kc * 8) * 2);
    gb[p] = BN ? (uint32_t)((kk * ldb + c * 8) * 2) : (uint32_t)((r * ldb + kc * 8) * 2);
  }
  const uint64_t sa = (uint64_t)(uintptr_t)(A + (AN ? kz * lda + m0 : (int64_t)m0 * lda + kz) * 2);
  const uint64_t sb = (uint64_t)(uintptr_t)(B + (BN ? kz * ldb + n0 : (int64_t)n0 * ldb + kz) * 2);
  const uint32_t lw = __builtin_amdgcn_readfirstlane(lds0 + w * 1024);
  int np = (nkt >> 1) - 2;  // full K-tile pairs of the loop (the first and the last pair are peeled)
  // transposed fragment reads (as gemm_tile's tfrag_mn): lane (g, q = rl >> 2, p = rl & 3) reads
  // k-rows kh*32 + 8g + q (+ 4) at column w{r,c}*128 + 16 j + 4p; with the swizzle the byte address is
  // R + (32 j ^ X), R = row + column-pair + half, X = 16 * (2q + 8 (g & 1)) -- built in the asm
  const int q = rl >> 2, pp = rl & 3;
  const uint32_t rbx = (uint32_t)(32 * q + 128 * (g & 1));
  const uint32_t rcol = lds0 + (8 * g + q) * 512 + 16 * (pp >> 1) + 8 * (pp & 1);
  const uint32_t rbr = rcol + wc * 256, rar = rcol + wr * 256;
  const uint32_t astep = (uint32_t)(64 * lda * 2), bstep = (uint32_t)(64 * ldb * 2);
  if constexpr (!AN && !BN) {
    asm volatile(MLT_W4_LOOP_ASM
                 : [np] "+s"(np)
                 : [sa] "s"(sa), [sb] "s"(sb), [lw] "s"(lw), [ra00] "v"(ra00), [ra01] "v"(ra01), [ra10] "v"(ra10),
                   [ra11] "v"(ra11), [rb00] "v"(rb00), [rb01] "v"(rb01), [rb10] "v"(rb10), [rb11] "v"(rb11),
                   [ga0] "v"(ga[0]), [ga1] "v"(ga[1]), [ga2] "v"(ga[2]), [ga3] "v"(ga[3]), [ga4] "v"(ga[4]),
                   [ga5] "v"(ga[5]), [ga6] "v"(ga[6]), [ga7] "v"(ga[7]), [gb0] "v"(gb[0]), [gb1] "v"(gb[1]),
                   [gb2] "v"(gb[2]), [gb3] "v"(gb[3]), [gb4] "v"(gb[4]), [gb5] "v"(gb[5]), [gb6] "v"(gb[6]),
                   [gb7] "v"(gb[7])
                 : MLT_W4_CLOBBERS, "memory");
  } else if constexpr (!AN) {
    asm volatile(MLT_W4_LOOP_ASM_BN
                 : [np] "+s"(np)
                 : [sa] "s"(sa), [sb] "s"(sb), [lw] "s"(lw), [bstep] "s"(bstep), [ra00] "v"(ra00), [ra01] "v"(ra01),
                   [ra10] "v"(ra10), [ra11] "v"(ra11), [rbr] "v"(rbr), [rbx] "v"(rbx), [ga0] "v"(ga[0]),
                   [ga1] "v"(ga[1]), [ga2] "v"(ga[2]), [ga3] "v"(ga[3]), [ga4] "v"(ga[4]), [ga5] "v"(ga[5]),
                   [ga6] "v"(ga[6]), [ga7] "v"(ga[7]), [gb0] "v"(gb[0]), [gb1] "v"(gb[1]), [gb2] "v"(gb[2]),
                   [gb3] "v"(gb[3]), [gb4] "v"(gb[4]), [gb5] "v"(gb[5]), [gb6] "v"(gb[6]), [gb7] "v"(gb[7])
                 : MLT_W4_CLOBBERS_BN, "memory");
  } else {
    static_assert(BN, "mn-contiguous A is built with an mn-contiguous B (the weight-gradient layout)");
    asm volatile(MLT_W4_LOOP_ASM_ANBN
                 : [np] "+s"(np)
                 : [sa] "s"(sa), [sb] "s"(sb), [lw] "s"(lw), [astep] "s"(astep), [bstep] "s"(bstep), [rar] "v"(rar),
                   [rbr] "v"(rbr), [rbx] "v"(rbx), [ga0] "v"(ga[0]), [ga1] "v"(ga[1]), [ga2] "v"(ga[2]),
                   [ga3] "v"(ga[3]), [ga4] "v"(ga[4]), [ga5] "v"(ga[5]), [ga6] "v"(ga[6]), [ga7] "v"(ga[7]),
                   [gb0] "v"(gb[0]), [gb1] "v"(gb[1]), [gb2] "v"(gb[2]), [gb3] "v"(gb[3]), [gb4] "v"(gb[4]),
                   [gb5] "v"(gb[5]), [gb6] "v"(gb[6]), [gb7] "v"(gb[7])
                 : MLT_W4_CLOBBERS_ANBN, "memory");
  }

  w4_epilogue<OutT, EK>(C, ldc, epi, epi.alpha, m0, n0, tiles_n * 256, w, lane, smem);
}

// fp8 operands (OCP e4m3 = 0 / e5m2 = 1 each; A [M][K], B [N][K] bytes): the block-scaled MFMA with
// unit scales, K-tile = 128 elements = the same 128-byte LDS rows; a fragment is the lane's 32
// bytes (chunks 2g and 2g + 1 of its row). Main loop: MLT_W4F8_LOOP_ASM (scripts/gen_gemm_w4.py).
template <typename OutT, int EK, int FA, int FB>
__device__ __forceinline__ void gemm_w4f8_tile(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                               OutT* __restrict__ C, int nkt, int64_t kz, int64_t lda, int64_t ldb,
                                               int64_t ldc, const GemmEpi& epi, int id, int gm_, int tiles_m,
                                               int tiles_n, uint8_t* smem) {
  const int per_group = gm_ * tiles_n, grp = id / per_group, first_m = grp * gm_;
  const int gsize = min(tiles_m - first_m, gm_), rr = id - grp * per_group;
  const int m0 = (first_m + rr % gsize) * 256, n0 = (rr / gsize) * 256;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 1, wc = w & 1;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_u8*)smem;
  const int g = lane >> 4, rl = lane & 15, sw = (rl >> 1) & 7;
  auto raddr = [&](int stage, int isb, int hi) {
    const int row = (isb ? wc : wr) * 128 + rl;
    return lds0 + stage * 65536 + isb * 32768 + row * 128 + (((2 * g + hi) ^ sw) << 4);
  };
  const uint32_t raL0 = raddr(0, 0, 0), raH0 = raddr(0, 0, 1), raL1 = raddr(1, 0, 0), raH1 = raddr(1, 0, 1);
  const uint32_t rbL0 = raddr(0, 1, 0), rbH0 = raddr(0, 1, 1), rbL1 = raddr(1, 1, 0), rbH1 = raddr(1, 1, 1);
  uint32_t ga[8], gb[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int r = (p * 4 + w) * 8 + (lane >> 3);
    const int kc = (lane & 7) ^ ((r >> 1) & 7);
    ga[p] = (uint32_t)(r * lda + kc * 16);
    gb[p] = (uint32_t)(r * ldb + kc * 16);
  }
  const uint64_t sa = (uint64_t)(uintptr_t)(A + (int64_t)m0 * lda + kz);
  const uint64_t sb = (uint64_t)(uintptr_t)(B + (int64_t)n0 * ldb + kz);
  const uint32_t lw = __builtin_amdgcn_readfirstlane(lds0 + w * 1024);
  int np = (nkt >> 1) - 2;  // full K-tile pairs of the loop (the first and the last pair are peeled)
  asm volatile(MLT_W4F8_LOOP_ASM
               : [np] "+s"(np)
               : [sa] "s"(sa), [sb] "s"(sb), [lw] "s"(lw), [raL0] "v"(raL0), [raH0] "v"(raH0), [raL1] "v"(raL1),
                 [raH1] "v"(raH1), [rbL0] "v"(rbL0), [rbH0] "v"(rbH0), [rbL1] "v"(rbL1), [rbH1] "v"(rbH1),
                 [ga0] "v"(ga[0]), [ga1] "v"(ga[1]), [ga2] "v"(ga[2]), [ga3] "v"(ga[3]), [ga4] "v"(ga[4]),
                 [ga5] "v"(ga[5]), [ga6] "v"(ga[6]), [ga7] "v"(ga[7]), [gb0] "v"(gb[0]), [gb1] "v"(gb[1]),
                 [gb2] "v"(gb[2]), [gb3] "v"(gb[3]), [gb4] "v"(gb[4]), [gb5] "v"(gb[5]), [gb6] "v"(gb[6]),
                 [gb7] "v"(gb[7]), [fa] "n"(FA), [fb] "n"(FB)
               : MLT_W4F8_CLOBBERS, "memory");
  float alpha = epi.alpha;
  if (epi.inv_scale_a) alpha *= *epi.inv_scale_a;
  if (epi.inv_scale_b) alpha *= *epi.inv_scale_b;
  w4_epilogue<OutT, EK>(C, ldc, epi, alpha, m0, n0, tiles_n * 256, w, lane, smem);
}

template <typename OutT, int EK, int FA, int FB>
__global__ __launch_bounds__(256, 1) void gemm_w4f8_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                           OutT* __restrict__ C, int M, int N, int nk, int ksteps,
                                                           int64_t lda, int64_t ldb, int64_t ldc, int64_t cstride,
                                                           GemmEpi epi, int group_m) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tiles_m = M >> 8, tiles_n = N >> 8;
  const int gm_ = group_m > 0 ? group_m : tiles_m;
  const int z = blockIdx.y, kt0 = z * ksteps, nkt = min(ksteps, nk - kt0);  // split z (see gemm_w4_kernel)
  const int T = tiles_m * tiles_n, G = gridDim.x;
  w4_load_gelu_tab<EK>(smem);
  if (G >= T) {
    gemm_w4f8_tile<OutT, EK, FA, FB>(A, B, C + (int64_t)z * cstride, nkt, (int64_t)kt0 * 128, lda, ldb, ldc, epi,
                                     xcd_remap(blockIdx.x, G), gm_, tiles_m, tiles_n, smem);
    return;
  }
  // persistent: XCD x walks its contiguous run of tile ids (as gemm_w4_kernel)
  const int x = blockIdx.x % 8, l = blockIdx.x / 8, per = G / 8, q = T / 8, r = T % 8;
  const int start = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q, end = start + q + (x < r ? 1 : 0);
  for (int id = start + l; id < end; id += per) {
    if (id != start + l) __syncthreads();
    gemm_w4f8_tile<OutT, EK, FA, FB>(A, B, C + (int64_t)z * cstride, nkt, (int64_t)kt0 * 128, lda, ldb, ldc, epi, id,
                                     gm_, tiles_m, tiles_n, smem);
  }
}

// Persistent by default: 256 workgroups (one per CU), XCD x walking ITS contiguous run of tile ids
// (the run xcd_remap gives it in a one-tile-per-workgroup launch, so the L2 reuse pattern is kept),
// the next tile's DMAs issued right behind the previous epilogue's stores: +0.5-2 % per shape,
// BERT-base 2,925 / 2,932 -> 2,945 / 2,956 (profiles/r4/gemm_w4_persist_xcd_ab.jsonl). (A first
// persistent version striding ids by 256 broke that locality and lost: QKV 950 vs 988 TF.)
// MLT_W4_PERSIST=0: one tile per workgroup.
template <typename OutT, int EK, bool AN, bool BN>
__global__ __launch_bounds__(256, 1) void gemm_w4_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                         OutT* __restrict__ C, int M, int N, int nk, int ksteps,
                                                         int64_t lda, int64_t ldb, int64_t ldc, int64_t cstride,
                                                         GemmEpi epi, int group_m) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tiles_m = M >> 8, tiles_n = N >> 8;
  const int gm_ = group_m > 0 ? group_m : tiles_m;
  // split z = blockIdx.y: K-tiles [z * ksteps, min(nk, (z + 1) * ksteps)), output slab z (cstride)
  const int z = blockIdx.y, kt0 = z * ksteps, nkt = min(ksteps, nk - kt0);
  const int T = tiles_m * tiles_n, G = gridDim.x;
  w4_load_gelu_tab<EK>(smem);
  if (G >= T) {
    gemm_w4_tile<OutT, EK, AN, BN>(A, B, C + (int64_t)z * cstride, nkt, (int64_t)kt0 * 64, lda, ldb, ldc, epi,
                                   xcd_remap(blockIdx.x, G), gm_, tiles_m, tiles_n, smem);
    return;
  }
  // persistent (G = 256 = 8 XCDs x 32): XCD x walks its contiguous run of tile ids
  const int x = blockIdx.x % 8, l = blockIdx.x / 8, per = G / 8, q = T / 8, r = T % 8;
  const int start = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q, end = start + q + (x < r ? 1 : 0);
  for (int id = start + l; id < end; id += per) {
    if (id != start + l) __syncthreads();  // the previous epilogue's LDS reads are done
    gemm_w4_tile<OutT, EK, AN, BN>(A, B, C + (int64_t)z * cstride, nkt, (int64_t)kt0 * 64, lda, ldb, ldc, epi, id,
                                   gm_, tiles_m, tiles_n, smem);
  }
}

template <typename OutT, int EK, bool AN, bool BN>
static void launch_w4_ek(const uint8_t* A, const uint8_t* B, OutT* C, int M, int N, int K, int64_t lda, int64_t ldb,
                         int64_t ldc, const GemmEpi& e, int group_m, int splits, int ksteps, int64_t cstride,
                         hipStream_t st) {
  constexpr int SMEM = w4_smem<EK>();
  auto kern = gemm_w4_kernel<OutT, EK, AN, BN>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    attr_set = true;
  }
  const int tiles = (M / 256) * (N / 256);
  static const bool persist = [] {
    const char* v = getenv("MLT_W4_PERSIST");
    return !(v && atoi(v) == 0);
  }();
  const int grid = persist && splits == 1 && tiles > 256 ? 256 : tiles;
  hipLaunchKernelGGL(kern, dim3(grid, splits), dim3(256), SMEM, st, A, B, C, M, N, K / 64, ksteps, lda, ldb, ldc,
                     cstride, e, group_m);
}

template <typename OutT, bool AN, bool BN>
static void launch_w4_bn(const uint8_t* A, const uint8_t* B, OutT* C, int M, int N, int K, int64_t lda, int64_t ldb,
                         int64_t ldc, const GemmEpi& e, int group_m, hipStream_t st) {
  const int nk = K / 64;
  if constexpr (sizeof(OutT) == 4) {  // fp32 outputs: the plain epilogue only (host-checked)
    launch_w4_ek<OutT, W4_PLAIN, AN, BN>(A, B, C, M, N, K, lda, ldb, ldc, e, group_m, 1, nk, 0, st);
  } else {
    if (e.mode == 1)
      launch_w4_ek<OutT, W4_GELU, AN, BN>(A, B, C, M, N, K, lda, ldb, ldc, e, group_m, 1, nk, 0, st);
    else if (e.mode == 2)
      launch_w4_ek<OutT, W4_DGELU, AN, BN>(A, B, C, M, N, K, lda, ldb, ldc, e, group_m, 1, nk, 0, st);
    else if (e.res)
      launch_w4_ek<OutT, W4_RES, AN, BN>(A, B, C, M, N, K, lda, ldb, ldc, e, group_m, 1, nk, 0, st);
    else
      launch_w4_ek<OutT, W4_PLAIN, AN, BN>(A, B, C, M, N, K, lda, ldb, ldc, e, group_m, 1, nk, 0, st);
  }
}

template <typename OutT>
void launch_gemm_w4(const uint8_t* A, const uint8_t* B, OutT* C, int M, int N, int K, int64_t lda, int64_t ldb,
                    int64_t ldc, const GemmEpi& e, int group_m, bool b_mn, hipStream_t st) {
  if (b_mn)
    launch_w4_bn<OutT, false, true>(A, B, C, M, N, K, lda, ldb, ldc, e, group_m, st);
  else
    launch_w4_bn<OutT, false, false>(A, B, C, M, N, K, lda, ldb, ldc, e, group_m, st);
}

bool gemm_w4_supported(int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int out_bytes, const GemmEpi& e,
                       bool b_mn) {
  auto al = [](const void* p, int64_t ld, int esz) {
    return p == nullptr || ((((uintptr_t)p) % 16) == 0 && (ld * esz) % 16 == 0);
  };
  if (M % 256 || N % 256 || K % 128 || K < 256) return false;
  if ((lda * 2) % 16 || (ldb * 2) % 16 || (ldc * out_bytes) % 16) return false;
  if (lda * 2 * 256 > (int64_t)1 << 31 || ldb * 2 * 256 > (int64_t)1 << 31) return false;  // 32-bit DMA offsets
  if (b_mn && (N % 8 || ldb < N)) return false;
  if (e.accumulate || e.inv_scale_a || e.inv_scale_b || e.qt || e.mode == 3) return false;
  if (e.q_colpart && e.mode != 2) return false;  // column partials: the dGELU epilogue only
  if (!al(e.res, e.ldres, 2) || !al(e.aux, e.ldaux, 2) || (e.bias && ((uintptr_t)e.bias) % 16)) return false;
  if (out_bytes == 4 && (e.mode != 0 || e.res)) return false;
  if (e.mode != 0 && e.res) return false;
  return true;
}

// weight-gradient layout (A [K][M], B [K][N]): split-K raw fp32 partials ws[z][M][N] (the caller's
// split-reduce applies alpha / bias / accumulate), or (splits == 1) straight through the epilogue
template <typename OutT>
void launch_gemm_w4_wgrad(const uint8_t* A, const uint8_t* B, OutT* C, float* ws, int M, int N, int K, int64_t lda,
                          int64_t ldb, int64_t ldc, const GemmEpi& e, int group_m, int splits, int ksteps,
                          hipStream_t st) {
  if (splits > 1) {
    GemmEpi raw{};
    raw.alpha = 1.f;
    launch_w4_ek<float, W4_PLAIN, true, true>(A, B, ws, M, N, K, lda, ldb, N, raw, group_m, splits, ksteps,
                                              (int64_t)M * N, st);
  } else {
    launch_w4_bn<OutT, true, true>(A, B, C, M, N, K, lda, ldb, ldc, e, group_m, st);
  }
}
bool gemm_w4_wgrad_supported(int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int out_bytes,
                             const GemmEpi& e, int splits, int ksteps) {
  const int nk = K / 64;
  if (M % 256 || N % 256 || K % 64 || splits < 1 || ksteps % 2 || ksteps < 4) return false;
  if ((int64_t)(splits - 1) * ksteps >= nk) return false;
  const int last = nk - (splits - 1) * ksteps;
  if (last % 2 || last < 4 || last > ksteps) return false;
  if ((lda * 2) % 16 || (ldb * 2) % 16 || lda < M || ldb < N) return false;
  if (lda * 2 * 64 > (int64_t)1 << 31 || ldb * 2 * 64 > (int64_t)1 << 31) return false;
  if (splits > 1) return N % 4 == 0;  // the raw partials; the split-reduce handles the epilogue
  return gemm_w4_supported(M, N, K, lda, ldb, ldc, out_bytes, e, true) && !e.accumulate;
}

template <typename OutT, int EK, int FA, int FB>
static void launch_w4f8_ek(const uint8_t* A, const uint8_t* B, OutT* C, int M, int N, int K, int64_t lda, int64_t ldb,
                           int64_t ldc, const GemmEpi& e, int group_m, hipStream_t st, int splits = 1, int ksteps = 0,
                           int64_t cstride = 0) {
  constexpr int SMEM = w4_smem<EK>();
  auto kern = gemm_w4f8_kernel<OutT, EK, FA, FB>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    attr_set = true;
  }
  static const bool persist = [] {
    const char* v = getenv("MLT_W4_PERSIST");
    return !(v && atoi(v) == 0);
  }();
  const int tiles = (M / 256) * (N / 256);
  const int grid = persist && splits == 1 && tiles > 256 ? 256 : tiles;
  hipLaunchKernelGGL(kern, dim3(grid, splits), dim3(256), SMEM, st, A, B, C, M, N, K / 128,
                     ksteps > 0 ? ksteps : K / 128, lda, ldb, ldc, cstride, e, group_m);
}
template <typename OutT, int FA, int FB>
void launch_gemm_w4_f8(const uint8_t* A, const uint8_t* B, OutT* C, int M, int N, int K, int64_t lda, int64_t ldb,
                       int64_t ldc, const GemmEpi& e, int group_m, hipStream_t st) {
  if constexpr (sizeof(OutT) == 4) {  // fp32 outputs: the plain epilogue only (host-checked)
    launch_w4f8_ek<OutT, W4_PLAIN, FA, FB>(A, B, C, M, N, K, lda, ldb, ldc, e, group_m, st);
  } else {
    if (e.mode == 1)
      launch_w4f8_ek<OutT, W4_GELU, FA, FB>(A, B, C, M, N, K, lda, ldb, ldc, e, group_m, st);
    else if (e.mode == 2)
      launch_w4f8_ek<OutT, W4_DGELU, FA, FB>(A, B, C, M, N, K, lda, ldb, ldc, e, group_m, st);
    else if (e.res)
      launch_w4f8_ek<OutT, W4_RES, FA, FB>(A, B, C, M, N, K, lda, ldb, ldc, e, group_m, st);
    else
      launch_w4f8_ek<OutT, W4_PLAIN, FA, FB>(A, B, C, M, N, K, lda, ldb, ldc, e, group_m, st);
  }
}
// split-K raw fp32 partials ws[z][M][N] (alpha, the fp8 inverse scales and the epilogue are the
// split-reduce's): the fp8 weight gradients (few tiles, K = tokens)
template <int FA, int FB>
void launch_gemm_w4_f8_splitk(const uint8_t* A, const uint8_t* B, float* ws, int M, int N, int K, int64_t lda,
                              int64_t ldb, int group_m, int splits, int ksteps, hipStream_t st) {
  GemmEpi raw{};
  raw.alpha = 1.f;
  launch_w4f8_ek<float, W4_PLAIN, FA, FB>(A, B, ws, M, N, K, lda, ldb, N, raw, group_m, st, splits, ksteps,
                                          (int64_t)M * N);
}
template void launch_gemm_w4_f8_splitk<0, 0>(const uint8_t*, const uint8_t*, float*, int, int, int, int64_t, int64_t,
                                              int, int, int, hipStream_t);
template void launch_gemm_w4_f8_splitk<1, 0>(const uint8_t*, const uint8_t*, float*, int, int, int, int64_t, int64_t,
                                              int, int, int, hipStream_t);
template void launch_gemm_w4_f8_splitk<0, 1>(const uint8_t*, const uint8_t*, float*, int, int, int, int64_t, int64_t,
                                              int, int, int, hipStream_t);
bool gemm_w4_f8_splitk_supported(int M, int N, int K, int64_t lda, int64_t ldb, int splits, int ksteps) {
  const int nk = K / 128;
  if (M % 256 || N % 256 || K % 128 || splits < 2 || ksteps % 2 || ksteps < 4 || N % 4) return false;
  if ((int64_t)(splits - 1) * ksteps >= nk) return false;
  const int last = nk - (splits - 1) * ksteps;
  if (last % 2 || last < 4 || last > ksteps) return false;
  if (lda % 16 || ldb % 16 || lda * 256 > (int64_t)1 << 31 || ldb * 256 > (int64_t)1 << 31) return false;
  return true;
}

bool gemm_w4_f8_supported(int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int out_bytes,
                          const GemmEpi& e) {
  auto al = [](const void* p, int64_t ld, int esz) {
    return p == nullptr || ((((uintptr_t)p) % 16) == 0 && (ld * esz) % 16 == 0);
  };
  if (M % 256 || N % 256 || K % 256 || K < 512) return false;
  if (lda % 16 || ldb % 16 || (ldc * out_bytes) % 16) return false;
  if (lda * 256 > (int64_t)1 << 31 || ldb * 256 > (int64_t)1 << 31) return false;
  if (e.accumulate || e.qt || e.mode == 3) return false;
  if (e.q_colpart && e.mode != 2) return false;
  if (!al(e.res, e.ldres, 2) || !al(e.aux, e.ldaux, 2) || (e.bias && ((uintptr_t)e.bias) % 16)) return false;
  if (out_bytes == 4 && (e.mode != 0 || e.res)) return false;
  if (e.mode != 0 && e.res) return false;
  return true;
}
// the quantising fp8 FFN epilogues on the 4-wave kernel (gemm_f8_q): FFN1's GELU (e4m3 A, e4m3 out)
// and FFN2-dgrad's dGELU (e5m2 A, e5m2 out, column partials); false when the shape / layout /
// formats do not fit
bool launch_gemm_w4_f8_q(int fmt_a, const uint8_t* A, const uint8_t* B, uint8_t* Y, int M, int N, int K,
                         int64_t lda, int64_t ldb, int64_t ldy, const GemmEpi& e, int group_m, hipStream_t st) {
  if (M % 256 || N % 256 || K % 256 || K < 512) return false;
  if (lda % 16 || ldb % 16 || ldy % 16 || e.ldqt % 16 || e.ldqt * 32 >= (int64_t)1 << 31) return false;
  if (lda * 256 > (int64_t)1 << 31 || ldb * 256 > (int64_t)1 << 31) return false;
  if (!e.aux || !e.qt || !e.q_scale || !e.q_amax || e.res || e.accumulate) return false;
  if ((e.ldaux * 2) % 16 || ((uintptr_t)e.aux) % 16 || ((uintptr_t)e.qt) % 16 || ((uintptr_t)Y) % 16) return false;
  if (e.bias && ((uintptr_t)e.bias) % 16) return false;
  if (e.mode == 1 && fmt_a == 0 && e.q_fmt == 0 && !e.q_colpart) {
    launch_w4f8_ek<uint8_t, W4_Q8GELU, 0, 0>(A, B, Y, M, N, K, lda, ldb, ldy, e, group_m, st);
    return true;
  }
  if (e.mode == 2 && fmt_a == 1 && e.q_fmt == 1) {
    launch_w4f8_ek<uint8_t, W4_Q8DGELU, 1, 0>(A, B, Y, M, N, K, lda, ldb, ldy, e, group_m, st);
    return true;
  }
  return false;
}

#define MLT_W4F8_INST(OT, FA, FB)                                                                                   \
  template void launch_gemm_w4_f8<OT, FA, FB>(const uint8_t*, const uint8_t*, OT*, int, int, int, int64_t, int64_t, \
                                              int64_t, const GemmEpi&, int, hipStream_t);
MLT_W4F8_INST(uint16_t, 0, 0)
MLT_W4F8_INST(uint16_t, 1, 0)
MLT_W4F8_INST(uint16_t, 0, 1)
MLT_W4F8_INST(float, 0, 0)
MLT_W4F8_INST(float, 1, 0)
MLT_W4F8_INST(float, 0, 1)
#undef MLT_W4F8_INST

template void launch_gemm_w4<uint16_t>(const uint8_t*, const uint8_t*, uint16_t*, int, int, int, int64_t, int64_t,
                                       int64_t, const GemmEpi&, int, bool, hipStream_t);
template void launch_gemm_w4<float>(const uint8_t*, const uint8_t*, float*, int, int, int, int64_t, int64_t, int64_t,
                                    const GemmEpi&, int, bool, hipStream_t);
template void launch_gemm_w4_wgrad<float>(const uint8_t*, const uint8_t*, float*, float*, int, int, int, int64_t,
                                          int64_t, int64_t, const GemmEpi&, int, int, int, hipStream_t);
template void launch_gemm_w4_wgrad<uint16_t>(const uint8_t*, const uint8_t*, uint16_t*, float*, int, int, int, int64_t,
                                             int64_t, int64_t, const GemmEpi&, int, int, int, hipStream_t);

}  // namespace mlt
