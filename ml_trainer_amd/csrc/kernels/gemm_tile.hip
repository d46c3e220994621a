// Large-tile bf16 GEMM for gfx950: 512 threads (8 waves), 256x256 / 256x192 / 256x128 / 128x256 block
// tiles, BK = 64, operands staged HBM -> LDS with global_load_lds_dwordx4 (no VGPR round
// trip, 16 B per lane per instruction) into two LDS buffers: tile k+1's DMA is issued before
// the MFMAs of tile k and retired by the one barrier per K-step
// (cdna_hip_programming.md §5 "glds vs register staging": the 256^2, ~1 block/CU regime).
//
// LDS images are lane-linear (a glds writes base + lane*16), so the bank-conflict swizzle is
// applied to the per-lane SOURCE address and undone on the read (rule 21):
//   k-contiguous operand  [rows][64 k]  : position p of row r holds 16-B chunk p ^ (r & 7)
//   mn-contiguous operand [64 k][BM|BN] : position p of k-row kk holds chunk p ^ (kk & 15)
// and fragments are read with ds_read_b128 (k-contiguous) or the gfx950 transpose read
// ds_read_b64_tr_b16 (mn-contiguous: dgrad / wgrad operands need no transpose pass).
//
// M / N tails: source rows / columns are clamped into the matrix (garbage lands only in
// output rows / columns >= M / N, which are never stored); K must be a multiple of 64.
//
// Split-K (gridDim.y = splits): each split writes its fp32 accumulators to a workspace slab
// in fragment order (coalesced 16-B stores), publishes with an agent-scope release and a
// relaxed ticket; the last arriver (acquire) sums the slabs in split order -- deterministic
// for any arrival order and any XCD placement -- and runs the fused epilogue
// (§5 "Projection GEMM" item 2; §6 Guideline 16).
//
// Epilogue: each wave stages 64-row halves of its sub-tile through a padded LDS image and
// writes 4 consecutive columns per lane (bias, GELU / dGELU, residual, accumulate fused).
#include <cstdlib>
#include <type_traits>

#include "mlt_common.h"
#include "mlt_fp8.h"
#include "mlt_gemm.h"
#include "mlt_gemm_tile.h"
#include "mlt_kernels.h"

namespace mlt {

// exact GELU / GELU' at the bf16 input points for the quantising epilogue (scripts/gen_gelu_table.py;
// the 4-wave kernel's epilogues use the same tables, gemm_w4.hip). Build switch -DMLT_Q8_GELU_TAB=0:
// the A&S erf polynomial of mlt_gemm.h. Same-box A/B at the large config's FFN (262 K tokens,
// profiles/r5/fp8_q8_gelu_tab_ab.jsonl): q8 GELU forward 2.37 -> 2.28 ms, q8 dGELU 2.49-2.50 ->
// 2.37-2.38 ms; fp8 `large` 1,183-1,184 -> 1,202-1,205 samples/s.
#ifndef MLT_Q8_GELU_TAB
#define MLT_Q8_GELU_TAB 1
#endif

template <int V>
using PIC = std::integral_constant<int, V>;

template <int BM, int BN, int WARPS_M>
struct TileGeom {
  static constexpr int A_BYTES = BM * T_BK * 2, B_BYTES = BN * T_BK * 2, BUF = A_BYTES + B_BYTES;
  static constexpr int WTN = BN / (8 / WARPS_M);
  static constexpr int EPR = WTN <= 64 ? 64 : 32;        // epilogue rows per pass per wave
  static constexpr int EPS = WTN + 4;                     // padded fp32 row stride of the image
  static constexpr int EPI_BYTES = 8 * EPR * EPS * 4;
  static constexpr int SMEM = 2 * BUF > EPI_BYTES ? 2 * BUF : EPI_BYTES;
};

// F8A / F8B: -1 = bf16 operands; 0 = fp8 e4m3, 1 = bf8 e5m2 (OCP) through the MX-scaled
// 16x16x128 MFMA at unit block scales (per-tensor scales are folded into the epilogue alpha).
template <int BM, int BN, int WARPS_M, bool AM, bool BNL, typename OutT, int F8A = -1, int F8B = -1>
__global__ __launch_bounds__(T_NT, 1) void gemm_tile_kernel(const uint8_t* __restrict__ A,
                                                             const uint8_t* __restrict__ B, OutT* __restrict__ C,
                                                             int M, int N, int K, int64_t lda, int64_t ldb,
                                                             int64_t ldc, GemmEpi epi, float* __restrict__ ws,
                                                             unsigned* __restrict__ cnt, int ksteps, int group_m) {
  using G = TileGeom<BM, BN, WARPS_M>;
  constexpr int WARPS_N = 8 / WARPS_M, WTM = BM / WARPS_M, WTN = BN / WARPS_N, TI = WTM / 16, TJ = WTN / 16;
  constexpr int A_CH = G::A_BYTES / 16 / T_NT, B_CH = G::B_BYTES / 16 / T_NT;
  static_assert(A_CH * 16 * T_NT == G::A_BYTES && B_CH * 16 * T_NT == G::B_BYTES, "glds chunking");
  static_assert(WTM % G::EPR == 0 && (G::EPR * WTN / 4) % 64 == 0, "epilogue geometry");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int tiles = gridDim.x, tiles_n = (N + BN - 1) / BN;
  // XCD-aware remap over the whole (tiles x splits) grid: workgroups are dealt to the 8 XCDs
  // round-robin in linear order (blockIdx.y * tiles + blockIdx.x). After the remap the ids one XCD
  // runs at once are consecutive and split-major: tiles of the SAME K-range, which share A / B
  // panels in that XCD's L2 (remapping blockIdx.x alone scattered them over XCDs in split-K grids)
  const int lin = xcd_remap((int)(blockIdx.y * tiles + blockIdx.x), tiles * (int)gridDim.y);
  const int id = lin % tiles, ksplit = lin / tiles;
  // grouped raster: runs of `group_m` tile-rows are walked column by column, so the ~32 blocks
  // an XCD runs at once share a few A row-panels AND a few B column-panels in its L2
  const int tiles_m = tiles / tiles_n;
  int tm, tn;
  {
    const int gm = group_m > 0 ? group_m : tiles_m;
    const int per_group = gm * tiles_n, grp = id / per_group, first_m = grp * gm;
    const int gsize = min(tiles_m - first_m, gm), r = id - grp * per_group;
    tm = first_m + r % gsize;
    tn = r / gsize;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  MLT_DCHECK(m0 < M && n0 < N && tiles % tiles_n == 0);  // tile grid = ceil(M/BM) x ceil(N/BN)
  MLT_DCHECK(K % (F8A >= 0 ? 128 : T_BK) == 0 && ksplit * ksteps < (K / (F8A >= 0 ? 128 : T_BK)));
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = (wid / WARPS_N) * WTM, wn = (wid % WARPS_N) * WTN;
  constexpr bool F8 = F8A >= 0;
  constexpr int ES = F8 ? 1 : 2;
  static_assert(!F8 || (F8B >= 0 && !AM && !BNL), "fp8 operands must both be fp8 and k-contiguous");
  const int nk = K / (F8 ? 128 : T_BK);
  const int kt0 = ksplit * ksteps, kt1 = min(nk, kt0 + ksteps);

  const uint8_t* asrc[A_CH];
  const uint8_t* bsrc[B_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) asrc[i] = glds_src<BM, AM, ES>(A, lda, i, m0, M);
#pragma unroll
  for (int i = 0; i < B_CH; ++i) bsrc[i] = glds_src<BN, BNL, ES>(B, ldb, i, n0, N);
  // bytes per K-step: a k-contiguous row advances 128 B; an mn-contiguous image 64 k-rows
  const int64_t astep = AM ? (int64_t)T_BK * lda * ES : 128, bstep = BNL ? (int64_t)T_BK * ldb * ES : 128;

  auto stage = [&](int buf, int kt) {
    uint8_t* base = smem + buf * G::BUF;
#pragma unroll
    for (int i = 0; i < A_CH; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + kt * astep),
                                       (lds_void*)(base + (i * T_NT + wid * 64) * 16), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < B_CH; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + kt * bstep),
                                       (lds_void*)(base + G::A_BYTES + (i * T_NT + wid * 64) * 16), 16, 0, 0);
  };

  f32x4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (kt0 < kt1) stage(0, kt0);
  __syncthreads();  // waits the DMA (vmcnt(0)) and publishes buffer 0
  for (int kt = kt0; kt < kt1; ++kt) {
    const int cur = (kt - kt0) & 1;
    if (kt + 1 < kt1) stage(cur ^ 1, kt + 1);
    const uint8_t* As = smem + cur * G::BUF;
    const uint8_t* Bs = As + G::A_BYTES;
    if constexpr (F8) {
      i32x8 bfr[TJ];
#pragma unroll
      for (int j = 0; j < TJ; ++j) bfr[j] = tfrag_f8(Bs, wn + 16 * j);
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const i32x8 af = tfrag_f8(As, wm + 16 * i);
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, bfr[j], acc[i][j], F8A, F8B, 0, 127, 0, 127);
      }
    } else
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      bf16x8 bfr[TJ];
#pragma unroll
      for (int j = 0; j < TJ; ++j) bfr[j] = BNL ? tfrag_mn<2 * BN>(Bs, wn + 16 * j, kh) : tfrag_k(Bs, wn + 16 * j, kh);
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const bf16x8 af = AM ? tfrag_mn<2 * BM>(As, wm + 16 * i, kh) : tfrag_k(As, wm + 16 * i, kh);
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();  // retires tile kt+1's DMA and frees buffer `cur` for tile kt+2
  }

  // ---- split-K: slab publish / last-arriver reduction --------------------------------------
  // (no counters = external mode: every split stores its raw fp32 partial tile row-major into
  // ws[split][M][N] through the epilogue below and splitk_reduce_kernel finishes the job)
  const bool ext = gridDim.y > 1 && cnt == nullptr;
  if (gridDim.y > 1 && !ext) {
    constexpr int SLAB = BM * BN;
    float* slab = ws + ((int64_t)ksplit * tiles + id) * SLAB;
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        *reinterpret_cast<f32x4*>(slab + ((int64_t)wid * TI * TJ * 64 + lane) * 4 + (i * TJ + j) * 256) = acc[i][j];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(smem);
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned t = __hip_atomic_fetch_add(cnt + id, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = t == gridDim.y - 1;
      if (last) __hip_atomic_store(cnt + id, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // sum the slabs in split order (own slab re-read: same order whoever arrives last)
    const int64_t fo = ((int64_t)wid * TI * TJ * 64 + lane) * 4;
    {
      const float* sl = ws + (int64_t)id * SLAB + fo;
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = *reinterpret_cast<const f32x4*>(sl + (i * TJ + j) * 256);
    }
    for (int z = 1; z < (int)gridDim.y; ++z) {
      const float* sl = ws + ((int64_t)z * tiles + id) * SLAB + fo;
      f32x4 v[TI][TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) v[i][j] = *reinterpret_cast<const f32x4*>(sl + (i * TJ + j) * 256);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] += v[i][j];
    }
  }

  // ---- epilogue ----------------------------------------------------------------------------
  constexpr int EPR = G::EPR, EPS = G::EPS, RI = EPR / 16;
  float alpha = epi.alpha;
  if (epi.inv_scale_a) alpha *= *epi.inv_scale_a;
  if (epi.inv_scale_b) alpha *= *epi.inv_scale_b;
  if (ext) alpha = 1.f;
  float* const wsz = ws + (int64_t)ksplit * M * N;
  const int g = lane >> 4, cl = lane & 15;
  float* cs = reinterpret_cast<float*>(smem) + wid * (EPR * EPS);
  float bv[TJ];
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int gn = n0 + wn + 16 * j + cl;
    bv[j] = (epi.bias && gn < N && !ext) ? epi.bias[gn] : 0.f;
  }
  constexpr int EIT = EPR * WTN / 4 / 64;  // float4 groups per lane per pass
  const EpiSide side = epi_side<OutT>(epi, C, ldc, N, ext);
  // the image is per wave and the main loop ended with a workgroup barrier (no DMA in flight):
  // wave-level hand-offs only, so the block's waves run their epilogues independently
  auto stage_pass = [&](int h) __attribute__((always_inline)) {
    wave_lds_sync();  // this wave's reads of the previous pass are done
#pragma unroll
    for (int ii = 0; ii < RI; ++ii)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          cs[(16 * ii + 4 * g + r) * EPS + 16 * j + cl] = acc[RI * h + ii][j][r] * alpha + bv[j];
    wave_lds_sync();
  };
  // side operands (residual / dGELU input / accumulate target) prefetched across the LDS round trip
  const int sk = epi_side_kind<OutT>(side, epi, m0 + BM <= M && n0 + BN <= N);
  const bool st8 = sk == 0 && epi_store8_ok(epi, C, ldc, N, m0 + BM <= M && n0 + BN <= N, ext);
  constexpr int HF = WTN % 3 == 0 ? EIT / 3 : EIT / 2;
#pragma unroll
  for (int h = 0; h < TI / RI; ++h) {
    auto rc = [&](int it, int& gm, int& gn, int& off) __attribute__((always_inline)) {
      const int e = it * 64 + lane, row = e / (WTN / 4), c4 = (e % (WTN / 4)) * 4;
      gm = m0 + wm + EPR * h + row;
      gn = n0 + wn + c4;
      off = row * EPS + c4;
    };
    auto stg = [&]() __attribute__((always_inline)) { stage_pass(h); };
    if (sk == EPI_RES) {
      epi_pass_side<EPI_RES, OutT, EIT, HF>(C, ldc, side, cs, rc, stg);
      continue;
    }
    if (sk == EPI_DGELU) {
      epi_pass_side<EPI_DGELU, OutT, EIT, HF>(C, ldc, side, cs, rc, stg);
      continue;
    }
    if constexpr (sizeof(OutT) == 4) {
      if (sk == EPI_ACC) {
        epi_pass_side<EPI_ACC, OutT, EIT, HF>(C, ldc, side, cs, rc, stg);
        continue;
      }
    }
    stage_pass(h);
    if constexpr (sizeof(OutT) == 2 && (WTN % 8) == 0 && EIT % 2 == 0) {
      if (st8) {
        epi_store8<EIT / 2>(reinterpret_cast<uint16_t*>(C), ldc, epi, cs,
                            [&](int it, int& gm, int& gn, int& off) __attribute__((always_inline)) {
                              const int e = it * 64 + lane, row = e / (WTN / 8), c8 = (e % (WTN / 8)) * 8;
                              gm = m0 + wm + EPR * h + row;
                              gn = n0 + wn + c8;
                              off = row * EPS + c8;
                            });
        continue;
      }
    }
#pragma unroll 4
    for (int it = 0; it < EIT; ++it) {
      const int e = it * 64 + lane, row = e / (WTN / 4), c4 = (e % (WTN / 4)) * 4;
      const int gm = m0 + wm + EPR * h + row, gn = n0 + wn + c4;
      if (gm >= M || gn >= N) continue;
      const float4 v = *reinterpret_cast<const float4*>(cs + row * EPS + c4);
      if (ext) {
        *reinterpret_cast<float4*>(wsz + (int64_t)gm * N + gn) = v;
        continue;
      }
      float vv[4] = {v.x, v.y, v.z, v.w};
      epilogue_store4<OutT>(C, ldc, epi, gm, gn, N, vv);
    }
  }
}

// External split-K reduction: out = epilogue(alpha * sum_z ws[z] + bias), summed in split order
// (bit-identical to the in-kernel last-arriver path), one float4 of a row per thread -- the
// whole chip reduces, instead of one block per tile reading every slab of its tile serially.
template <typename OutT>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, int S, int M, int N,
                                                            OutT* __restrict__ C, int64_t ldc, GemmEpi epi) {
  const int64_t total = (int64_t)M * N / 4;
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= total) return;
  const float4* w = reinterpret_cast<const float4*>(ws);
  float4 s = w[q];
#pragma unroll 4
  for (int z = 1; z < S; ++z) {
    const float4 v = w[(int64_t)z * total + q];
    s.x += v.x;
    s.y += v.y;
    s.z += v.z;
    s.w += v.w;
  }
  float alpha = epi.alpha;
  if (epi.inv_scale_a) alpha *= *epi.inv_scale_a;
  if (epi.inv_scale_b) alpha *= *epi.inv_scale_b;
  const int64_t e = q * 4;
  const int gm = (int)(e / N), gn = (int)(e % N);
  float vv[4] = {s.x * alpha, s.y * alpha, s.z * alpha, s.w * alpha};
  if (epi.bias) {
#pragma unroll
    for (int k = 0; k < 4; ++k) vv[k] += epi.bias[gn + k];
  }
  epilogue_store4<OutT>(C, ldc, epi, gm, gn, N, vv);
}

// ---------------------------------------------------------------------------------------------
// Ping-pong 256x256 kernel (config 5): the two waves that share a SIMD alternate between an
// MFMA cluster and a load section, and operand DMAs stay in flight across barriers.
//
//   * waves 0-3 (group 0) and 4-7 (group 1) sit on the four SIMDs in pairs; group 1 executes
//     one extra s_barrier up front, so while one group runs the 16 MFMAs of a phase the other
//     issues its fragment ds_reads and its share of the next DMA (cdna_hip_programming.md §5,
//     "The 256^2 8-phase template"; T3-T5);
//   * a K-tile (64 bf16 / 128 fp8 of K) is four phases, one per 64x32 quadrant of the wave's
//     output (rows {qm*128 + wr*64 ..+64}, cols {qn*128 + wc*32 ..+32}), visited in the order
//     (0,0) (0,1) (1,1) (1,0) so each phase reads either the A or the B fragments (or both);
//   * the LDS image of a K-tile is four 16 KiB half-tiles [A0 A1 B0 B1] (128 rows or columns
//     each), two K-tiles resident (even buffer E, odd buffer O). Each phase stages ONE
//     half-tile (2 glds per thread): the half whose last ds_read was the previous phase
//     (WAR: those reads were retired by an lgkmcnt(0) before that phase's first barrier):
//        phase: 1      2      3      4      5      6      7      8
//        reads: E q0   E q1   E q2   E q3   O q0   O q1   O q2   O q3
//        stage: O.B0   E.A0   E.B1   E.A1   E.B0   O.A0   O.B1   O.A1
//               (t+1)  (t+2)  (t+2)  (t+2)  (t+2)  (t+3)  (t+3)  (t+3)
//   * RAW: phase 4 waits vmcnt(6) (the three newest half-tiles stay in flight) which retires
//     all of O; phase 8 likewise retires all of E; the waits precede the phase's first barrier
//     and the buffer is read one phase later (one barrier more than the stagger needs);
//   * raw s_barrier (inline asm) -- __syncthreads would drain vmcnt(0) every phase.
// ---------------------------------------------------------------------------------------------
#define MLT_PP_SYNC_READS()                                              \
  do {                                                                   \
    __builtin_amdgcn_sched_barrier(0);                                   \
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");      \
    __builtin_amdgcn_sched_barrier(0);                                   \
  } while (0)
#define MLT_PP_BARRIER()                                                 \
  do {                                                                   \
    __builtin_amdgcn_sched_barrier(0);                                   \
    asm volatile("s_barrier" ::: "memory");                              \
    __builtin_amdgcn_sched_barrier(0);                                   \
  } while (0)

template <int V>
using IC = std::integral_constant<int, V>;

// ---- quantising ("q8") epilogue of one 64x32 quadrant -------------------------------------
// cs: the wave's staged fp32 image of the quadrant (row stride 36, alpha and bias applied),
// rows gm0 + 0..63, columns gn0 + 0..31, wholly inside C. Row pass: 2 lanes per row, 16 columns
// each -- the activation (GELU: pre-activation saved as bf16; dGELU: times gelu'(aux)), amax, one
// 16-byte fp8 store of C; the final fp32 values go back into the image. Column pass: one column
// per lane, 32 rows per half-wave (conflict-free: the 32 lanes of a half read 32 consecutive
// banks) -> two 16-byte stores of C^T (the consumer GEMM's k-contiguous operand) and the
// column partial sum of the quadrant (bias gradient), both halves combined by one shuffle.
template <int FMT>
__device__ __forceinline__ void q8_quadrant(uint8_t* __restrict__ C, int64_t ldc, const GemmEpi& epi, float* cs,
                                            int gm0, int gn0, int N, int lane, float& amx, const uint8_t* tab) {
  constexpr int EPS = 36;
  const float s = *epi.q_scale;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int row = it * 32 + (lane >> 1), c16 = (lane & 1) * 16;
    float* p = cs + row * EPS + c16;
    float v[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 t = reinterpret_cast<const float4*>(p)[q];
      v[4 * q] = t.x;
      v[4 * q + 1] = t.y;
      v[4 * q + 2] = t.z;
      v[4 * q + 3] = t.w;
    }
    const int64_t gm = gm0 + row;
    const int gn = gn0 + c16;
    if (epi.mode == 1) {  // GELU: save the bf16 pre-activation, activate its rounded value
      uint16_t* ap = const_cast<uint16_t*>(epi.aux) + gm * epi.ldaux + gn;
      uint32_t pr[8];  // (two-wide GELU, mlt_gemm.h)
#pragma unroll
      for (int q = 0; q < 8; ++q) pr[q] = cvt_pk_bf16(f32x2{v[2 * q], v[2 * q + 1]});
      reinterpret_cast<uint4*>(ap)[0] = make_uint4(pr[0], pr[1], pr[2], pr[3]);
      reinterpret_cast<uint4*>(ap)[1] = make_uint4(pr[4], pr[5], pr[6], pr[7]);
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        f32x2 x2[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) x2[q] = unpack_bf16x2(pr[4 * hh + q]);
        if constexpr (MLT_Q8_GELU_TAB) {
#pragma unroll
          for (int q = 0; q < 4; ++q) x2[q] = x2[q] * gelu_tab2(pr[4 * hh + q], tab);
        } else {
          gelu2<4>(x2);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) v[8 * hh + 2 * q] = x2[q].x, v[8 * hh + 2 * q + 1] = x2[q].y;
      }
    } else if (epi.mode == 2) {  // dGELU: times gelu'(pre-activation)
      const uint4* ap = reinterpret_cast<const uint4*>(epi.aux + gm * epi.ldaux + gn);
      const uint4 a0 = ap[0], a1 = ap[1];
      const uint32_t w[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        f32x2 x2[4];
        if constexpr (MLT_Q8_GELU_TAB) {
#pragma unroll
          for (int q = 0; q < 4; ++q) x2[q] = gelu_tab2(w[4 * hh + q], tab);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) x2[q] = unpack_bf16x2(w[4 * hh + q]);
          gelu_grad2<4>(x2);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) v[8 * hh + 2 * q] *= x2[q].x, v[8 * hh + 2 * q + 1] *= x2[q].y;
      }
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      amx = fmaxf(amx, fabsf(v[q]));
      v[q] *= s;  // the image keeps the SCALED values: the column pass only converts
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
      reinterpret_cast<float4*>(p)[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    uint32_t o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = pack4_fp8<FMT>(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    *reinterpret_cast<uint4*>(C + gm * ldc + gn) = make_uint4(o[0], o[1], o[2], o[3]);
  }
  wave_lds_sync();  // the image is this wave's own
  const int col = lane & 31, r0 = (lane >> 5) * 32;
  const float* p = cs + r0 * EPS + col;
  uint4* tp = reinterpret_cast<uint4*>(epi.qt + (int64_t)(gn0 + col) * epi.ldqt + gm0 + r0);
  auto column = [&](auto csc) __attribute__((always_inline)) {
    constexpr bool CS = decltype(csc)::value;
    uint32_t w[8];
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float x[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) x[j] = p[(4 * k + j) * EPS];
      if constexpr (CS) sum += (x[0] + x[1]) + (x[2] + x[3]);
      w[k] = pack4_fp8<FMT>(x[0], x[1], x[2], x[3]);
    }
    tp[0] = make_uint4(w[0], w[1], w[2], w[3]);
    tp[1] = make_uint4(w[4], w[5], w[6], w[7]);
    if constexpr (CS) {  // column sums of the unscaled output: one multiply by 1/scale
      sum += __shfl_xor(sum, 32);
      if (lane < 32) epi.q_colpart[(int64_t)(gm0 >> 6) * N + gn0 + col] = sum * __builtin_amdgcn_rcpf(s);
    }
  };
  if (epi.q_colpart)
    column(std::true_type{});
  else
    column(std::false_type{});
}

template <bool AM, bool BNL, typename OutT, int F8A = -1, int F8B = -1>
__global__ __launch_bounds__(T_NT, 1) void gemm_pp_kernel(const uint8_t* __restrict__ A,
                                                          const uint8_t* __restrict__ B, OutT* __restrict__ C,
                                                          int M, int N, int K, int64_t lda, int64_t ldb,
                                                          int64_t ldc, GemmEpi epi, float* __restrict__ ws,
                                                          unsigned* __restrict__ cnt, int ksteps, int group_m) {
  constexpr int BM = 256, BN = 256, HALF = 16384, BUF = 4 * HALF, NF = 32;
  constexpr bool F8 = F8A >= 0;
  constexpr int ES = F8 ? 1 : 2;
  static_assert(!F8 || (F8B >= 0 && !AM && !BNL), "fp8 operands must both be fp8 and k-contiguous");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int tiles = gridDim.x, tiles_n = (N + BN - 1) / BN;
  // XCD-aware remap over the whole (tiles x splits) grid: workgroups are dealt to the 8 XCDs
  // round-robin in linear order (blockIdx.y * tiles + blockIdx.x). After the remap the ids one XCD
  // runs at once are consecutive and split-major: tiles of the SAME K-range, which share A / B
  // panels in that XCD's L2 (remapping blockIdx.x alone scattered them over XCDs in split-K grids)
  const int lin = xcd_remap((int)(blockIdx.y * tiles + blockIdx.x), tiles * (int)gridDim.y);
  const int id = lin % tiles, ksplit = lin / tiles;
  int tm, tn;
  {
    const int tiles_m = tiles / tiles_n;
    const int gm = group_m > 0 ? group_m : tiles_m;
    const int per_group = gm * tiles_n, grp = id / per_group, first_m = grp * gm;
    const int gsize = min(tiles_m - first_m, gm), r = id - grp * per_group;
    tm = first_m + r % gsize;
    tn = r / gsize;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  MLT_DCHECK(m0 < M && n0 < N && tiles % tiles_n == 0);  // tile grid = ceil(M/BM) x ceil(N/BN)
  MLT_DCHECK(K % (F8A >= 0 ? 128 : T_BK) == 0 && ksplit * ksteps < (K / (F8A >= 0 ? 128 : T_BK)));
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wid >> 2, wc = wid & 3;
  const int nk = K / (F8 ? 128 : T_BK);
  const int kt0 = ksplit * ksteps, kt1 = min(nk, kt0 + ksteps);
  if constexpr (sizeof(OutT) == 1 && MLT_Q8_GELU_TAB) {  // quantising GELU / dGELU epilogue: its table
    if (epi.mode == 1 || epi.mode == 2) gelu_tab_load(smem + 2 * BUF, epi.mode == 2, T_NT);
  }

  // glds sources of the four half-tiles (0 A0, 1 A1, 2 B0, 3 B1), two 16-B chunks per thread
  // each: 32-bit offsets from the uniform operand bases (the host guarantees < 4 GiB spans)
  uint32_t src[4][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    src[0][i] = glds_off<128, AM, ES>(lda, i, m0, M);
    src[1][i] = glds_off<128, AM, ES>(lda, i, m0 + 128, M);
    src[2][i] = glds_off<128, BNL, ES>(ldb, i, n0, N);
    src[3][i] = glds_off<128, BNL, ES>(ldb, i, n0 + 128, N);
  }
  const int64_t astep = AM ? (int64_t)T_BK * lda * ES : 128, bstep = BNL ? (int64_t)T_BK * ldb * ES : 128;
  auto stage = [&](auto hc, int buf, int kt) {
    constexpr int h = decltype(hc)::value;
    const uint8_t* base = h < 2 ? A + (int64_t)kt * astep : B + (int64_t)kt * bstep;
    uint8_t* dst = smem + buf * BUF + h * HALF;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(base + src[h][i]), (lds_void*)(dst + (i * T_NT + wid * 64) * 16),
                                       16, 0, 0);
  };

  f32x4 acc[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[4][2], bfr[2][2];
  i32x8 af8[4], bf8[2];
  auto read_a = [&](const uint8_t* h) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (F8) {
        af8[i] = tfrag_f8(h, wr * 64 + 16 * i);
      } else {
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
          af[i][kh] = AM ? tfrag_mn<256>(h, wr * 64 + 16 * i, kh) : tfrag_k(h, wr * 64 + 16 * i, kh);
      }
    }
  };
  auto read_b = [&](const uint8_t* h) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if constexpr (F8) {
        bf8[j] = tfrag_f8(h, wc * 32 + 16 * j);
      } else {
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
          bfr[j][kh] = BNL ? tfrag_mn<256>(h, wc * 32 + 16 * j, kh) : tfrag_k(h, wc * 32 + 16 * j, kh);
      }
    }
  };
  auto mma = [&](auto qmc, auto qnc) {
    constexpr int qm = decltype(qmc)::value, qn = decltype(qnc)::value, f0 = (qm * 2 + qn) * 8;
    __builtin_amdgcn_s_setprio(1);
    if constexpr (F8) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[f0 + i * 2 + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af8[i], bf8[j], acc[f0 + i * 2 + j],
                                                                                  F8A, F8B, 0, 127, 0, 127);
    } else {
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[f0 + i * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][kh], bfr[j][kh], acc[f0 + i * 2 + j], 0, 0, 0);
    }
    // pin the cluster between its barriers: IR-level passes ignore sched_barrier and may sink
    // MFMAs past the (volatile-asm) barrier, which stretches operand live ranges into spills
#pragma unroll
    for (int f = 0; f < 8; ++f) asm volatile("" ::"v"(acc[f0 + f]));
    __builtin_amdgcn_s_setprio(0);
  };
  // one phase: reads of quadrant q from `rb`, stage half `sh` of K-tile `skt` into buffer `sbuf`,
  // optional counted DMA wait, barrier, MFMA cluster, barrier
  auto phase = [&](auto qc, auto shc, const uint8_t* rb, int sbuf, int skt, bool do_stage, int wait, bool compute) {
    constexpr int q = decltype(qc)::value;
    if (compute) {
      if constexpr (q == 0) {
        read_b(rb + 2 * HALF);
        read_a(rb);
      } else if constexpr (q == 1) {
        read_b(rb + 3 * HALF);
      } else if constexpr (q == 2) {
        read_a(rb + HALF);
      } else {
        read_b(rb + 2 * HALF);
      }
    }
    if (do_stage) stage(shc, sbuf, skt);
    if (wait == 6)
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (wait == 0)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    MLT_PP_SYNC_READS();
    if (compute) {
      if constexpr (q == 0) mma(IC<0>{}, IC<0>{});
      else if constexpr (q == 1) mma(IC<0>{}, IC<1>{});
      else if constexpr (q == 2) mma(IC<1>{}, IC<1>{});
      else mma(IC<1>{}, IC<0>{});
    }
    MLT_PP_BARRIER();
  };

  // prologue: K-tile kt0 -> E (all four halves), kt0+1 -> O (A0, B1, A1; B0 comes in phase 1)
  if (kt0 < kt1) {
    stage(IC<0>{}, 0, kt0);
    stage(IC<3>{}, 0, kt0);
    stage(IC<1>{}, 0, kt0);
    stage(IC<2>{}, 0, kt0);
  }
  if (kt0 + 1 < kt1) {
    stage(IC<0>{}, 1, kt0 + 1);
    stage(IC<3>{}, 1, kt0 + 1);
    stage(IC<1>{}, 1, kt0 + 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  MLT_PP_BARRIER();
  const bool late = __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256;  // group 1: wave-uniform branch
  if (late) MLT_PP_BARRIER();
  const uint8_t* E = smem;
  const uint8_t* O = smem + BUF;
  for (int t = kt0; t < kt1; t += 2) {
    const bool o1 = t + 1 < kt1, e2 = t + 2 < kt1, o3 = t + 3 < kt1;
    phase(IC<0>{}, IC<2>{}, E, 1, t + 1, o1, -1, true);
    phase(IC<1>{}, IC<0>{}, E, 0, t + 2, e2, -1, true);
    phase(IC<2>{}, IC<3>{}, E, 0, t + 2, e2, -1, true);
    phase(IC<3>{}, IC<1>{}, E, 0, t + 2, e2, e2 ? 6 : 0, true);
    phase(IC<0>{}, IC<2>{}, O, 0, t + 2, e2, -1, o1);
    phase(IC<1>{}, IC<0>{}, O, 1, t + 3, o3, -1, o1);
    phase(IC<2>{}, IC<3>{}, O, 1, t + 3, o3, -1, o1);
    phase(IC<3>{}, IC<1>{}, O, 1, t + 3, o3, o3 ? 6 : 0, o1);
  }
  if (!late) MLT_PP_BARRIER();  // both groups have now executed the same number of barriers
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- split-K: slab publish / last-arriver reduction (as gemm_tile_kernel) ------------------
  const bool ext = gridDim.y > 1 && cnt == nullptr;
  if (gridDim.y > 1 && !ext) {
    constexpr int SLAB = BM * BN;
    const int64_t fo = ((int64_t)wid * NF * 64 + lane) * 4;
    float* slab = ws + ((int64_t)ksplit * tiles + id) * SLAB + fo;
#pragma unroll
    for (int f = 0; f < NF; ++f) *reinterpret_cast<f32x4*>(slab + f * 256) = acc[f];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(smem);
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned tk = __hip_atomic_fetch_add(cnt + id, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = tk == gridDim.y - 1;
      if (last) __hip_atomic_store(cnt + id, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    {
      const float* sl = ws + (int64_t)id * SLAB + fo;
#pragma unroll
      for (int f = 0; f < NF; ++f) acc[f] = *reinterpret_cast<const f32x4*>(sl + f * 256);
    }
    for (int z = 1; z < (int)gridDim.y; ++z) {
      const float* sl = ws + ((int64_t)z * tiles + id) * SLAB + fo;
      f32x4 v[NF];
#pragma unroll
      for (int f = 0; f < NF; ++f) v[f] = *reinterpret_cast<const f32x4*>(sl + f * 256);
#pragma unroll
      for (int f = 0; f < NF; ++f) acc[f] += v[f];
    }
  }

  // ---- epilogue: one 64x32 quadrant per pass through a padded per-wave LDS image -----------
  constexpr int EPS = 36;
  float alpha = epi.alpha;
  if (epi.inv_scale_a) alpha *= *epi.inv_scale_a;
  if (epi.inv_scale_b) alpha *= *epi.inv_scale_b;
  if (ext) alpha = 1.f;
  float* const wsz = ws + (int64_t)ksplit * M * N;
  const int g = lane >> 4, cl = lane & 15;
  float* cs = reinterpret_cast<float*>(smem) + wid * (64 * EPS);
  const EpiSide side = epi_side<OutT>(epi, C, ldc, N, ext);
  // quadrant qd of the wave's output: rows gm0(qd) + 0..63, columns gn0(qd) + 0..31
  auto q_gm0 = [&](int qd) __attribute__((always_inline)) { return m0 + (qd >> 1) * 128 + wr * 64; };
  auto q_gn0 = [&](int qd) __attribute__((always_inline)) { return n0 + (qd & 1) * 128 + wc * 32; };
  auto stage_q = [&](int qd) __attribute__((always_inline)) {
    float bv[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int gn = q_gn0(qd) + 16 * j + cl;
      bv[j] = (epi.bias && gn < N && !ext) ? epi.bias[gn] : 0.f;
    }
    // per-wave image after the post-loop workgroup barrier: wave-level hand-offs only
    wave_lds_sync();
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          cs[(16 * i + 4 * g + r) * EPS + 16 * j + cl] = acc[qd * 8 + i * 2 + j][r] * alpha + bv[j];
    wave_lds_sync();
  };
  // side operands (residual / dGELU input / accumulate target) prefetched across the LDS round trip
  const int sk = epi_side_kind<OutT>(side, epi, m0 + 256 <= M && n0 + 256 <= N);
  const bool st8 = sk == 0 && epi_store8_ok(epi, C, ldc, N, m0 + 256 <= M && n0 + 256 <= N, ext);
  // one quadrant per call with a compile-time index: the accumulator array must stay in registers
  // (a runtime quadrant index -- e.g. a loop the compiler declines to unroll -- puts it on the stack)
  float q_amx = 0.f;  // q8: max |output| over this wave's quadrants
  auto quadrant = [&](auto qc) __attribute__((always_inline)) {
    constexpr int qd = decltype(qc)::value;
    auto rc = [&](int it, int& gm, int& gn, int& off) __attribute__((always_inline)) {
      const int e = it * 64 + lane, row = e >> 3, c4 = (e & 7) * 4;
      gm = q_gm0(qd) + row;
      gn = q_gn0(qd) + c4;
      off = row * EPS + c4;
    };
    if constexpr (sizeof(OutT) == 1) {  // quantising epilogue (interior tiles, no split: host-checked)
      stage_q(qd);
      if (epi.q_fmt == 0)
        q8_quadrant<0>(reinterpret_cast<uint8_t*>(C), ldc, epi, cs, q_gm0(qd), q_gn0(qd), N, lane, q_amx,
                       smem + 2 * BUF);
      else
        q8_quadrant<1>(reinterpret_cast<uint8_t*>(C), ldc, epi, cs, q_gm0(qd), q_gn0(qd), N, lane, q_amx,
                       smem + 2 * BUF);
      return;
    } else {
    auto stg = [&]() __attribute__((always_inline)) { stage_q(qd); };
    if (sk == EPI_RES) {
      epi_pass_side<EPI_RES, OutT, 8, 4>(C, ldc, side, cs, rc, stg);
      return;
    }
    if (sk == EPI_DGELU) {
      if (epi.q_colpart) {  // + column sums (bias gradient): lanes with equal lane & 7 share 4 columns
        float csum[4] = {0.f, 0.f, 0.f, 0.f};
        epi_pass_side<EPI_DGELU, OutT, 8, 4, true>(C, ldc, side, cs, rc, stg, csum);
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int off = 8; off < 64; off <<= 1) csum[q] += __shfl_xor(csum[q], off);
        if (lane < 8)
          *reinterpret_cast<float4*>(epi.q_colpart + (int64_t)(q_gm0(qd) >> 6) * N + q_gn0(qd) + lane * 4) =
              make_float4(csum[0], csum[1], csum[2], csum[3]);
      } else {
        epi_pass_side<EPI_DGELU, OutT, 8, 4>(C, ldc, side, cs, rc, stg);
      }
      return;
    }
    MLT_DCHECK(epi.q_colpart == nullptr);  // the host guarantees the dGELU side pass for column sums
    if constexpr (sizeof(OutT) == 4) {
      if (sk == EPI_ACC) {
        epi_pass_side<EPI_ACC, OutT, 8, 4>(C, ldc, side, cs, rc, stg);
        return;
      }
    }
    stage_q(qd);
    const int gm0 = q_gm0(qd), gn0 = q_gn0(qd);
    if constexpr (sizeof(OutT) == 2) {
      if (st8) {  // 64 x 32 quadrant: 4 lanes per row, 8 columns each
        const int row0 = lane >> 2, c8 = (lane & 3) * 8;
        epi_store8<4>(reinterpret_cast<uint16_t*>(C), ldc, epi, cs,
                      [=](int it, int& gm, int& gn, int& off) __attribute__((always_inline)) {
                        gm = gm0 + 16 * it + row0;
                        gn = gn0 + c8;
                        off = (16 * it + row0) * EPS + c8;
                      });
        return;
      }
    }
#pragma unroll 4
    for (int it = 0; it < 8; ++it) {
      const int e = it * 64 + lane, row = e >> 3, c4 = (e & 7) * 4;
      const int gm = gm0 + row, gn = gn0 + c4;
      if (gm >= M || gn >= N) continue;
      const float4 v = *reinterpret_cast<const float4*>(cs + row * EPS + c4);
      if (ext) {
        *reinterpret_cast<float4*>(wsz + (int64_t)gm * N + gn) = v;
        continue;
      }
      float vv[4] = {v.x, v.y, v.z, v.w};
      epilogue_store4<OutT>(C, ldc, epi, gm, gn, N, vv);
    }
    }
  };
  quadrant(PIC<0>{});
  quadrant(PIC<1>{});
  quadrant(PIC<2>{});
  quadrant(PIC<3>{});
  if constexpr (sizeof(OutT) == 1) {
    if (epi.q_amax) {
      q_amx = wave_max(q_amx);
      if (lane == 0) atomic_max_pos(epi.q_amax, q_amx);
    }
  }
}
#undef MLT_PP_SYNC_READS
#undef MLT_PP_BARRIER

// ---------------------------------------------------------------------------------------------
// host: planning + dispatch
// ---------------------------------------------------------------------------------------------
void launch_gemm_bf16_128(int a_mn, int b_mn, bool out_f32, const uint16_t* A, const uint16_t* B, void* C, int M,
                          int N, int K, int64_t lda, int64_t ldb, int64_t ldc, const GemmEpi& e, hipStream_t st);

namespace {
constexpr int kCUs = 256;
struct CfgDesc {
  int bm, bn;
  double rate;   // sustained FLOP/s per CU (relative model, measured ordering)
  int per_cu;    // resident blocks per CU
  double fixed;  // per-block fixed cost (prologue fill + epilogue), s
};
constexpr int kNumCfg = 8;
// cfg 5 (ping-pong) fitted to the 64K-token BERT shapes (profiles/gemm_bf16_64k_tokens.jsonl):
// 8-10 % faster than cfg 1 at K = 2304-3072; since the 16-byte-store epilogue also 3-8 % faster
// at K = 768 (profiles/gemm_epi16_64k_tokens.jsonl) -> a faster steady state, a small extra
// fixed cost.
const CfgDesc kCfg[kNumCfg] = {{128, 128, 0.62e15 / kCUs, 2, 1.0e-6},
                               {256, 256, 1.15e15 / kCUs, 1, 1.0e-6},
                               {256, 128, 0.92e15 / kCUs, 1, 1.0e-6},
                               {128, 256, 0.92e15 / kCUs, 1, 1.0e-6},
                               {256, 192, 1.05e15 / kCUs, 1, 1.0e-6},
                               {256, 256, 1.335e15 / kCUs, 1, 2.5e-6},   // 5: ping-pong
                               {256, 256, 1.335e15 / kCUs, 1, 5.6e-6},   // 6: persistent ping-pong (fill once)
                               {256, 256, 1.335e15 / kCUs, 1, 2.5e-6}};  // 7: 4-wave asm main loop (gemm_w4.hip)

// split-K combine override: -1 planner, 0 in-kernel, 1 external (env MLT_GEMM_SPLIT_EXT, or
// set_gemm_split_mode() from tests / benchmarks)
int g_split_mode = -2;
int gemm_split_mode() {
  if (g_split_mode == -2) {
    const char* v = getenv("MLT_GEMM_SPLIT_EXT");
    g_split_mode = v ? atoi(v) : -1;
  }
  return g_split_mode;
}

// Cost of combining split-K partials (fitted to benchmarks/wgrad_bench.py on MI355X). In-kernel:
// the last-arriving block of each tile reads every slab of its tile on its own -- measured
// ~40 GB/s effective for that one block, i.e. serial. External: every split writes a row-major
// partial (overlapped with the other splits' compute) and one grid-wide reduce launch sums them
// at ~6 TB/s (+ a launch). `ext` receives the cheaper choice.
double split_cost(int cfg, int splits, int M, int N, int* ext) {
  const CfgDesc& c = kCfg[cfg];
  const double slab = (double)c.bm * c.bn * 4.0;
  const double t_in = splits * slab / 40.0e9 + 1.0e-6;
  const double t_ext = (double)M * N * 4.0 * (splits + 1.0) / 6.0e12 + 3.0e-6;
  const bool use_ext = N % 4 == 0 && t_ext < t_in;
  if (ext) *ext = use_ext ? 1 : 0;
  return use_ext ? t_ext : t_in;
}

// kstep = K elements per 128-byte row step (64 bf16, 128 fp8); speed = MFMA-rate factor
double est_time(int cfg, int splits, int M, int N, int K, int kstep, double speed) {
  const CfgDesc& c = kCfg[cfg];
  const int64_t tiles = (int64_t)((M + c.bm - 1) / c.bm) * ((N + c.bn - 1) / c.bn);
  const int64_t blocks = tiles * splits;
  const int64_t slots = (int64_t)kCUs * c.per_cu;
  const int64_t rounds = (blocks + slots - 1) / slots;
  const int nk = (K + kstep - 1) / kstep, ks = (nk + splits - 1) / splits;
  const double fixed = c.fixed;
  const double t_block = 2.0 * c.bm * c.bn * kstep * ks / (speed * c.rate / c.per_cu) + fixed;
  double t = rounds * t_block;
  if (cfg == 6) t = rounds * (t_block - fixed) + fixed;  // prologue / epilogue overlap the next tile
  if (splits > 1) t += split_cost(cfg, splits, M, N, nullptr);
  return t;
}

// grouped tile raster: runs of kGroupM M-tiles walk the N tiles together (MLT_GEMM_GROUP_M
// overrides). 4 measured >= 8 everywhere on MI355X (profiles/gemm_group_m_r2.txt: BERT-base b512
// +1.0 %, fp8 large b512 +1.1 %, BERT-base b128 equal); 16 lost 2-3 % at b128 (ab_gemm_group_m.txt)
constexpr int kGroupM = 4;
// cfg 7 runs one 256 x 256 tile per workgroup and never splits K: below about one tile per CU the
// split-K tiles win (the fp8 weight gradients of the `large` config: 16-256 tiles at K = 256K
// tokens ran 1,064 -> 621 samples/s end to end when cfg 7 took them)
constexpr int kW4MinTiles = 240;
// one workgroup's 256 x 256 x 64 K-tile at ~1.4 PF / 256 CUs (planner model for the split choice;
// the fp8 K-tile of 128 takes the same cycles)
constexpr double kW4KtileSec = 2.0 * 256 * 256 * 64 / (1.4e15 / 256);
// split count for cfg 7 over nk K-tiles: rounds of workgroups x K-tiles each + the partials' traffic
void w4_pick_splits(int tiles, int nk, int M, int N, int& bs, int& bks) {
  double best = 1e30;
  bs = bks = 0;
  for (int S = 1; S <= 64; ++S) {
    int ks = (nk + S - 1) / S;
    ks += ks & 1;
    if (ks < 4) break;
    const int last = nk - (S - 1) * ks;
    if (last < 4 || last % 2) continue;
    const int64_t rounds = ((int64_t)tiles * S + kCUs - 1) / kCUs;
    const double t = (double)rounds * ks * kW4KtileSec + (S > 1 ? (double)M * N * 4.0 * (S + 1) / 5.0e12 + 3.0e-6 : 0.0);
    if (t < best) {
      best = t;
      bs = S;
      bks = ks;
    }
  }
}

GemmPlan plan_tiles(int M, int N, int K, int force_cfg, int force_splits, int kstep, bool allow_legacy,
                    bool allow_pp = true, bool allow_persist = true) {
  GemmPlan p{0, 1, 0, 0, 0};
  const bool big_ok = K % kstep == 0 && K >= kstep && M >= 64 && N >= 64;
  const double speed = kstep == 128 ? 1.8 : 1.0;
  int best_cfg = 0, best_s = 1;
  if (force_cfg >= 0) {
    best_cfg = (force_cfg >= 1 && force_cfg < kNumCfg && big_ok) ? force_cfg : 0;
    if (best_cfg == 6 && !allow_persist) best_cfg = 1;
    best_s = best_cfg ? (force_splits > 0 && best_cfg < 6 ? force_splits : 1) : 1;
  } else if (big_ok) {
    double best = allow_legacy ? est_time(0, 1, M, N, K, 64, 1.0) : 1e30;
    const int nk = K / kstep;
    for (int cfg = 1; cfg < kNumCfg; ++cfg)
      for (int s = 1; s <= 16; ++s) {
        if (cfg == 5 && !allow_pp) break;
        // persistent ping-pong (cfg 6): only when forced. It won 4-12 % on the fp8 K = 768 / 1024
        // shapes while the tile kernels stored 8 bytes per lane; with their 16-byte-store
        // epilogue the ping-pong tile beats it by 13-20 % there (profiles/gemm_epi16_64k_tokens.jsonl,
        // profiles/fp8_cfg_large_131k_tokens.jsonl), and at K >= 3072 it already lost by 8-11 %.
        if (cfg >= 6) break;
        if (s > nk) break;
        const int ks = (nk + s - 1) / s;
        if ((int64_t)ks * (s - 1) >= nk) continue;  // no empty split
        if (s > 1 && ks < 4) continue;
        const double t = est_time(cfg, s, M, N, K, kstep, speed);
        if (t < best * 0.97) {
          best = t;
          best_cfg = cfg;
          best_s = s;
        }
      }
    if (force_splits > 0 && best_cfg) {
      if (best_cfg == 6) best_cfg = 1;  // an explicit split-K request takes the split-capable tile
      best_s = force_splits;
    }
  }
  p.cfg = best_cfg;
  p.splits = best_s;
  if (best_cfg) {
    const int nk = K / kstep;
    if (p.splits > nk) p.splits = nk;
    p.ksteps = (nk + p.splits - 1) / p.splits;
    const CfgDesc& c = kCfg[best_cfg];
    const int64_t tiles = (int64_t)((M + c.bm - 1) / c.bm) * ((N + c.bn - 1) / c.bn);
    if (p.splits > 1) {
      split_cost(best_cfg, p.splits, M, N, &p.ext);
      const int mode = gemm_split_mode();
      if (mode >= 0) p.ext = (mode > 0 && N % 4 == 0) ? 1 : 0;
      if (p.ext) {
        p.ws_floats = (int64_t)p.splits * M * N;
        p.cnt_ints = 0;
      } else {
        p.ws_floats = tiles * p.splits * c.bm * c.bn;
        p.cnt_ints = tiles;
      }
    }
  }
  return p;
}

// Split-K tile counters: one zero-initialised device pool (allocated on first use, i.e. in an
// eager warm-up call, never inside a graph capture), handed out as a ring of slices. Every
// launch leaves its slice zeroed (the last arriver of each tile resets its counter), so no
// per-call memset node is needed; a ring of kCntSlices slices keeps split GEMMs that are in
// flight on different streams apart.
constexpr int kCntSlices = 16, kCntSlice = 1 << 14;
unsigned* split_counters(int64_t need) {
  static unsigned* pool = nullptr;
  static int next = 0;
  if (need > kCntSlice) return nullptr;
  if (!pool) {
    if (hipMalloc(&pool, sizeof(unsigned) * kCntSlices * kCntSlice) != hipSuccess) return nullptr;
    if (hipMemset(pool, 0, sizeof(unsigned) * kCntSlices * kCntSlice) != hipSuccess) return nullptr;
  }
  unsigned* s = pool + (int64_t)(next % kCntSlices) * kCntSlice;
  ++next;
  return s;
}

template <int BM, int BN, int WARPS_M, bool AM, bool BNL, typename OutT, int F8A, int F8B>
void launch_tile(const GemmPlan& p, const uint8_t* A, const uint8_t* B, OutT* C, int M, int N, int K, int64_t lda,
                 int64_t ldb, int64_t ldc, const GemmEpi& e, float* ws, unsigned* cnt, hipStream_t st) {
  using G = TileGeom<BM, BN, WARPS_M>;
  auto kern = gemm_tile_kernel<BM, BN, WARPS_M, AM, BNL, OutT, F8A, F8B>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, G::SMEM);
    attr_set = true;
  }
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  static const int group_m = [] {
    const char* v = getenv("MLT_GEMM_GROUP_M");
    return v ? atoi(v) : kGroupM;
  }();
  hipLaunchKernelGGL(kern, dim3(tiles, p.splits), dim3(T_NT), G::SMEM, st, A, B, C, M, N, K, lda, ldb, ldc, e, ws,
                     cnt, p.ksteps, group_m);
}

template <bool AM, bool BNL, typename OutT, int F8A, int F8B>
void launch_pp(const GemmPlan& p, const uint8_t* A, const uint8_t* B, OutT* C, int M, int N, int K, int64_t lda,
               int64_t ldb, int64_t ldc, const GemmEpi& e, float* ws, unsigned* cnt, hipStream_t st) {
  // two K-tiles; the epilogue image (8 x 64 x 36 fp32) fits inside; + the GELU table (quantising epilogue)
  constexpr int SMEM = 2 * 4 * 16384 + (sizeof(OutT) == 1 && MLT_Q8_GELU_TAB ? kGeluTabBytes : 0);
  auto kern = gemm_pp_kernel<AM, BNL, OutT, F8A, F8B>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    attr_set = true;
  }
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  static const int group_m = [] {
    const char* v = getenv("MLT_GEMM_GROUP_M");
    return v ? atoi(v) : kGroupM;
  }();
  hipLaunchKernelGGL(kern, dim3(tiles, p.splits), dim3(T_NT), SMEM, st, A, B, C, M, N, K, lda, ldb, ldc, e, ws, cnt,
                     p.ksteps, group_m);
}

template <bool AM, bool BNL, typename OutT, int F8A, int F8B>
void launch_cfg(const GemmPlan& p, const uint8_t* A, const uint8_t* B, OutT* C, int M, int N, int K, int64_t lda,
                int64_t ldb, int64_t ldc, const GemmEpi& e, float* ws, unsigned* cnt, hipStream_t st) {
  switch (p.cfg) {
    case 1: launch_tile<256, 256, 2, AM, BNL, OutT, F8A, F8B>(p, A, B, C, M, N, K, lda, ldb, ldc, e, ws, cnt, st); break;
    case 2: launch_tile<256, 128, 4, AM, BNL, OutT, F8A, F8B>(p, A, B, C, M, N, K, lda, ldb, ldc, e, ws, cnt, st); break;
    case 3: launch_tile<128, 256, 2, AM, BNL, OutT, F8A, F8B>(p, A, B, C, M, N, K, lda, ldb, ldc, e, ws, cnt, st); break;
    case 4: launch_tile<256, 192, 4, AM, BNL, OutT, F8A, F8B>(p, A, B, C, M, N, K, lda, ldb, ldc, e, ws, cnt, st); break;
    case 5: launch_pp<AM, BNL, OutT, F8A, F8B>(p, A, B, C, M, N, K, lda, ldb, ldc, e, ws, cnt, st); break;
    case 6:
      // persistent ping-pong (gemm_persist.hip): k-contiguous A, an even K-tile count, no split
      if constexpr (!AM) {
        if ((K / (F8A >= 0 ? 128 : T_BK)) % 2 == 0 && p.splits == 1) {
          static const int group_m = [] {
            const char* v = getenv("MLT_GEMM_GROUP_M");
            return v ? atoi(v) : kGroupM;
          }();
          launch_gemm_persist<AM, BNL, OutT, F8A, F8B>(A, B, C, M, N, K, lda, ldb, ldc, e, group_m, kCUs, st);
          break;
        }
      }
      launch_pp<AM, BNL, OutT, F8A, F8B>(p, A, B, C, M, N, K, lda, ldb, ldc, e, ws, cnt, st);
      break;
    case 7:
      // 4-wave asm main loop (gemm_w4.hip): bf16, k-contiguous A, full 256 tiles
      if constexpr (!AM && F8A < 0 && (sizeof(OutT) == 2 || sizeof(OutT) == 4)) {
        if (p.splits == 1 && gemm_w4_supported(M, N, K, lda, ldb, ldc, (int)sizeof(OutT), e, BNL)) {
          static const int group_m = [] {
            const char* v = getenv("MLT_GEMM_GROUP_M");
            return v ? atoi(v) : kGroupM;
          }();
          launch_gemm_w4<OutT>(A, B, C, M, N, K, lda, ldb, ldc, e, group_m, BNL, st);
          break;
        }
      } else if constexpr (AM && BNL && F8A < 0 && (sizeof(OutT) == 2 || sizeof(OutT) == 4)) {
        // weight gradients: both operands transposed in LDS, split-K raw partials (external reduce)
        if (gemm_w4_wgrad_supported(M, N, K, lda, ldb, ldc, (int)sizeof(OutT), e, p.splits, p.ksteps) &&
            (p.splits == 1 || (ws != nullptr && cnt == nullptr))) {
          static const int group_m = [] {
            const char* v = getenv("MLT_GEMM_GROUP_M");
            return v ? atoi(v) : kGroupM;
          }();
          launch_gemm_w4_wgrad<OutT>(A, B, C, ws, M, N, K, lda, ldb, ldc, e, group_m, p.splits, p.ksteps, st);
          break;
        }
        launch_tile<256, 256, 2, AM, BNL, OutT, F8A, F8B>(p, A, B, C, M, N, K, lda, ldb, ldc, e, ws, cnt, st);
        break;
      } else if constexpr (!AM && !BNL && F8A >= 0 && (sizeof(OutT) == 2 || sizeof(OutT) == 4)) {
        static const int group_m = [] {
          const char* v = getenv("MLT_GEMM_GROUP_M");
          return v ? atoi(v) : kGroupM;
        }();
        if (p.splits == 1 && gemm_w4_f8_supported(M, N, K, lda, ldb, ldc, (int)sizeof(OutT), e)) {
          launch_gemm_w4_f8<OutT, F8A, F8B>(A, B, C, M, N, K, lda, ldb, ldc, e, group_m, st);
          break;
        }
        if (p.splits > 1 && ws != nullptr && cnt == nullptr &&
            gemm_w4_f8_splitk_supported(M, N, K, lda, ldb, p.splits, p.ksteps)) {
          launch_gemm_w4_f8_splitk<F8A, F8B>(A, B, ws, M, N, K, lda, ldb, group_m, p.splits, p.ksteps, st);
          break;
        }
      }
      launch_pp<AM, BNL, OutT, F8A, F8B>(p, A, B, C, M, N, K, lda, ldb, ldc, e, ws, cnt, st);
      break;
    default: break;
  }
}

// split-K plan without workspace / counters -> unsplit
bool resolve_split(GemmPlan& p, float* ws, unsigned*& cnt, int K, int kstep) {
  if (p.splits > 1 && p.ext) {
    cnt = nullptr;  // external mode is signalled to the kernels by the missing counters
    if (ws == nullptr) {
      p.splits = 1;
      p.ksteps = K / kstep;
    }
    return p.splits > 1;
  }
  if (p.splits > 1 && cnt == nullptr) cnt = split_counters(p.cnt_ints);
  if (p.splits > 1 && (cnt == nullptr || ws == nullptr)) {
    p.splits = 1;
    p.ksteps = K / kstep;
  }
  return p.splits > 1;
}

template <typename OutT>
void launch_split_reduce(const GemmPlan& p, const float* ws, OutT* C, int M, int N, int64_t ldc, const GemmEpi& e,
                         hipStream_t st) {
  const int64_t q = (int64_t)M * N / 4;
  hipLaunchKernelGGL(splitk_reduce_kernel<OutT>, dim3((unsigned)((q + 255) / 256)), dim3(256), 0, st, ws, p.splits, M,
                     N, C, ldc, e);
}
}  // namespace

void set_gemm_split_mode(int mode) { g_split_mode = mode; }

// which kernel runs gemm_f8_q's GELU epilogue: 1 the 4-wave one, 0 the ping-pong one, -1 MLT_GEMM_W4Q8
static int g_w4q8 = -1;
void set_gemm_w4q8(int on) { g_w4q8 = on; }

GemmPlan plan_gemm_bf16(int a_mn, int b_mn, int M, int N, int K, int force_cfg, int force_splits, int accumulate) {
  (void)b_mn;
  // (the 4-wave kernel's in-kernel epilogue cannot accumulate into C: an accumulating GEMM takes it
  // only with split-K partials, whose external reduce accumulates; otherwise the fitted planner)
  // the 4-wave asm kernel (cfg 7) takes every k-contiguous-A (forward / input-gradient) shape it
  // covers: 3-17 % over the ping-pong tile on the BERT forward shapes, 98-101 % of hipBLASLt at
  // 4096^3 / 8192^3 (profiles/r4/gemm_w4_*.jsonl). MLT_GEMM_W4=0 restores the fitted planner.
  static const bool w4 = [] {
    const char* v = getenv("MLT_GEMM_W4");
    return !(v && atoi(v) == 0);
  }();
  // (only with enough tiles to fill the chip: few-tile / long-K shapes keep the split-K planner)
  if (w4 && !accumulate && force_cfg < 0 && force_splits <= 0 && a_mn == 0 && M % 256 == 0 && N % 256 == 0 &&
      K % 128 == 0 && K >= 256 && (int64_t)(M / 256) * (N / 256) >= kW4MinTiles) {
    GemmPlan p{7, 1, K / 64, 0, 0};
    return p;
  }
  // weight gradients (both operands mn-contiguous, few tiles, K = tokens): cfg 7 with split-K raw
  // partials reduced by one grid-wide launch; splits from a rounds x K-steps + reduce-traffic model
  if (w4 && force_cfg < 0 && force_splits <= 0 && a_mn == 1 && b_mn == 1 && M % 256 == 0 && N % 256 == 0 &&
      K % 128 == 0 && K >= 256) {
    int bs = 0, bks = 0;
    w4_pick_splits((M / 256) * (N / 256), K / 64, M, N, bs, bks);
    if (bs > 1 || (bs == 1 && !accumulate)) {
      GemmPlan p{7, bs, bks, bs > 1 ? (int64_t)bs * M * N : 0, 0};
      p.ext = bs > 1 ? 1 : 0;
      return p;
    }
  }
  // the ping-pong kernel's fit covers the k-contiguous-A (forward / dgrad) shapes; weight
  // gradients (A = dY^T, mn-contiguous) stay on the 256-wide tiles with split-K
  return plan_tiles(M, N, K, force_cfg, force_splits, 64, true, a_mn == 0, a_mn == 0);
}

GemmPlan plan_gemm_f8(int M, int N, int K, int force_cfg, int force_splits) {
  // the 4-wave asm kernel's fp8 form (cfg 7) where it applies; MLT_GEMM_W4=0 / MLT_GEMM_W4F8=0 opt out
  static const bool w4 = [] {
    const char* v = getenv("MLT_GEMM_W4");
    const char* v8 = getenv("MLT_GEMM_W4F8");
    return !(v && atoi(v) == 0) && !(v8 && atoi(v8) == 0);
  }();
  if (w4 && force_cfg < 1 && force_splits <= 0 && M % 256 == 0 && N % 256 == 0 && K % 256 == 0 && K >= 512 &&
      (int64_t)(M / 256) * (N / 256) >= kW4MinTiles) {
    GemmPlan p{7, 1, K / 128, 0, 0};
    return p;
  }
  // few tiles, long K (the fp8 weight gradients): cfg 7 split-K raw partials + the external reduce
  if (w4 && force_cfg < 1 && force_splits <= 0 && M % 256 == 0 && N % 256 == 0 && N % 4 == 0 && K % 256 == 0 &&
      K >= 1024) {
    int bs = 0, bks = 0;
    w4_pick_splits((M / 256) * (N / 256), K / 128, M, N, bs, bks);
    if (bs > 1) {
      GemmPlan p{7, bs, bks, (int64_t)bs * M * N, 0};
      p.ext = 1;
      return p;
    }
  }
  GemmPlan p = plan_tiles(M, N, K, force_cfg < 1 ? -1 : force_cfg, force_splits, 128, false);
  if (p.cfg == 0) p.cfg = -1;  // not runnable (K % 128 != 0 or too small)
  return p;
}

void launch_gemm_bf16(const GemmPlan& plan, int a_mn, int b_mn, bool out_f32, const uint16_t* A, const uint16_t* B,
                      void* C, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc, const float* bias,
                      const uint16_t* aux, int64_t ldaux, const uint16_t* res, int64_t ldres, float alpha, int mode,
                      int accumulate, float* ws, unsigned* cnt, hipStream_t st, float* colpart) {
  if (M <= 0 || N <= 0) return;
  GemmEpi e{bias, aux, res, ldaux, ldres, alpha, mode, accumulate};
  e.q_colpart = colpart;  // dGELU column partials (host: ping-pong plan, interior tiles only)
  if (plan.cfg == 0) {
    launch_gemm_bf16_128(a_mn, b_mn, out_f32, A, B, C, M, N, K, lda, ldb, ldc, e, st);
    return;
  }
  GemmPlan p = plan;
  const bool ext = resolve_split(p, ws, cnt, K, 64) && p.ext;
  const uint8_t* a8 = reinterpret_cast<const uint8_t*>(A);
  const uint8_t* b8 = reinterpret_cast<const uint8_t*>(B);
#define MLT_TILE_CASE(AMV, BNV)                                                                                  \
  if (a_mn == AMV && b_mn == BNV) {                                                                              \
    if (out_f32)                                                                                                 \
      launch_cfg<AMV, BNV, float, -1, -1>(p, a8, b8, (float*)C, M, N, K, lda, ldb, ldc, e, ws, cnt, st);         \
    else                                                                                                         \
      launch_cfg<AMV, BNV, uint16_t, -1, -1>(p, a8, b8, (uint16_t*)C, M, N, K, lda, ldb, ldc, e, ws, cnt, st);   \
    if (ext && out_f32) launch_split_reduce<float>(p, ws, (float*)C, M, N, ldc, e, st);                          \
    if (ext && !out_f32) launch_split_reduce<uint16_t>(p, ws, (uint16_t*)C, M, N, ldc, e, st);                   \
    return;                                                                                                      \
  }
  MLT_TILE_CASE(0, 0)
  MLT_TILE_CASE(0, 1)
  MLT_TILE_CASE(1, 0)
  MLT_TILE_CASE(1, 1)
#undef MLT_TILE_CASE
}

void launch_gemm_f8(const GemmPlan& plan, int fmt_a, int fmt_b, bool out_f32, const uint8_t* A, const uint8_t* B,
                    void* C, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc, const float* inv_scale_a,
                    const float* inv_scale_b, const float* bias, const uint16_t* aux, int64_t ldaux,
                    const uint16_t* res, int64_t ldres, float alpha, int mode, int accumulate, float* ws,
                    unsigned* cnt, hipStream_t st) {
  if (M <= 0 || N <= 0 || plan.cfg < 1) return;
  GemmEpi e{bias, aux, res, ldaux, ldres, alpha, mode, accumulate, inv_scale_a, inv_scale_b};
  GemmPlan p = plan;
  const bool ext = resolve_split(p, ws, cnt, K, 128) && p.ext;
#define MLT_F8_CASE(FA, FB)                                                                                      \
  if (fmt_a == FA && fmt_b == FB) {                                                                              \
    if (out_f32)                                                                                                 \
      launch_cfg<false, false, float, FA, FB>(p, A, B, (float*)C, M, N, K, lda, ldb, ldc, e, ws, cnt, st);       \
    else                                                                                                         \
      launch_cfg<false, false, uint16_t, FA, FB>(p, A, B, (uint16_t*)C, M, N, K, lda, ldb, ldc, e, ws, cnt, st); \
    if (ext && out_f32) launch_split_reduce<float>(p, ws, (float*)C, M, N, ldc, e, st);                          \
    if (ext && !out_f32) launch_split_reduce<uint16_t>(p, ws, (uint16_t*)C, M, N, ldc, e, st);                   \
    return;                                                                                                      \
  }
  MLT_F8_CASE(0, 0)
  MLT_F8_CASE(1, 0)
  MLT_F8_CASE(0, 1)
#undef MLT_F8_CASE
}

void launch_gemm_f8_q(int fmt_a, int fmt_b, const uint8_t* A, const uint8_t* B, uint8_t* Y, uint8_t* Yt, int M, int N,
                      int K, int64_t lda, int64_t ldb, int64_t ldy, int64_t ldyt, const float* inv_scale_a,
                      const float* inv_scale_b, const float* bias, const uint16_t* aux, int64_t ldaux, int mode,
                      int out_fmt, const float* out_scale, float* out_amax, float* colpart, hipStream_t st) {
  if (M <= 0 || N <= 0) return;  // the host binding checks M % 256, N % 256, K % 128
  GemmEpi e{bias, aux, nullptr, ldaux, 0, 1.f, mode, 0, inv_scale_a, inv_scale_b};
  e.qt = Yt;
  e.ldqt = ldyt;
  e.q_scale = out_scale;
  e.q_amax = out_amax;
  e.q_colpart = colpart;
  e.q_fmt = out_fmt;
  // the 4-wave kernel's quantising epilogues when they fit (MLT_GEMM_W4Q8=0 / set_gemm_w4q8(0): the
  // ping-pong kernel's): 1.93 vs 2.27 ms per FFN1 (GELU) call and 1.97 vs 2.37 ms per FFN2-dgrad
  // (dGELU) call of the fp8 `large` step (262144 x 4096 x 1024), 1,262 vs 1,204 samples/s for the
  // step (profiles/r5/fp8_q8_w4_ab.jsonl). Its first form, Y^T stored as 64 rows x 16 bytes per
  // instruction, took 2.63 ms: the 4-wave epilogue is not hidden behind another wave group's main
  // loop, so the Y^T pass is stored as 16 columns x 64 contiguous bytes per instruction instead.
  // (Round 4's 4-wave q8 form, on the erf GELU, had lost too: 2.73 vs 2.43 ms.)
  if (g_w4q8 < 0) {
    const char* v = getenv("MLT_GEMM_W4Q8");
    g_w4q8 = (v && atoi(v) == 0) ? 0 : 1;
  }
  // raster group width 4 (MLT_GEMM_W4Q8_GROUP_M overrides): in isolation 2 M-tiles ran the GELU
  // form faster (1.91 vs 1.96 ms) and the dGELU form slower (2.08 vs 1.97), 8 / 16 lost on both;
  // in the fp8 `large` step GELU at 2 lost (1,254 vs 1,263 samples/s) -- profiles/r5/fp8_q8_w4_group_m.jsonl
  static const int q_group_m = [] {
    const char* v = getenv("MLT_GEMM_W4Q8_GROUP_M");
    return v ? atoi(v) : 0;
  }();
  const int gm_q = q_group_m > 0 ? q_group_m : kGroupM;
  if (g_w4q8 && launch_gemm_w4_f8_q(fmt_a, A, B, Y, M, N, K, lda, ldb, ldy, e, gm_q, st)) return;
  GemmPlan p{5, 1, K / 128, 0, 0};
  if (fmt_a == 0 && fmt_b == 0)
    launch_pp<false, false, uint8_t, 0, 0>(p, A, B, Y, M, N, K, lda, ldb, ldy, e, nullptr, nullptr, st);
  else if (fmt_a == 1 && fmt_b == 0)
    launch_pp<false, false, uint8_t, 1, 0>(p, A, B, Y, M, N, K, lda, ldb, ldy, e, nullptr, nullptr, st);
}

}  // namespace mlt
