// Persistent ping-pong 256x256 bf16 / fp8 GEMM for gfx950 (planner cfg 6): one 512-thread
// workgroup per CU walks a static list of output tiles, and neither the operand pipeline nor the
// CUs stop at a tile boundary.
//
// Why: with one tile per workgroup (gemm_tile.hip) every CU finishes its tile at about the same
// moment, writes its 128 KB C tile through LDS passes with no MFMA work under it, and starts the
// next tile with an empty pipeline. At K = 768 (12 K-steps per tile: BERT-base QKV / out-proj /
// FFN1 forward, FFN2 dgrad) that fill + drain is the difference to hipBLASLt
// (profiles/gemm_bf16_64k_tokens.jsonl: 870-880 TF vs 1,220-1,280).
//
// Structure = the ping-pong schedule of gemm_tile.hip's gemm_pp_kernel (wave groups 0-3 / 4-7
// staggered by one barrier, one 64x32 quadrant per phase, 8 phases per pair of K-tiles, half-tile
// DMAs staged 1-3 K-tiles ahead with counted vmcnt waits and raw s_barriers) run over the
// CONCATENATED K-tile stream of all the workgroup's tiles: the DMAs of the next tile's first
// K-tiles are issued during the current tile's last phases, so its MFMAs start without a fill.
// After the phase that completes a tile the epilogue runs straight from registers:
//   * the MFMA operands are swapped (D = B_tile . A_tile^T), so each lane's accumulator holds 4
//     CONSECUTIVE COLUMNS of one C row -> 8-byte bf16 / 16-byte fp32 vector stores, no LDS, no
//     barrier (the other wave group keeps computing), and the stores drain under the next tile;
//   * the epilogue kind is a template parameter: on gfx9 vmcnt counts stores AND loads, so any
//     load or data-dependent branch between stores makes hipcc wait for every earlier store
//     (a per-fragment call of the runtime-moded epilogue_store4 measured 590 vs 810 TF). Side
//     operands (residual / dGELU pre-activation) of a quarter tile are loaded first, then its 8
//     stores go out back to back; edge tiles and rare combinations take epilogue_store4.
// Tiles are dealt round-robin over the workgroups after the XCD-aware remap and the grouped
// raster, so the ~32 tiles an XCD works on at once share A / B panels in its L2.
// Requirements (host-checked, else cfg 5 / 1 run): an even number of K-tiles, splits = 1.
#include <type_traits>

#include "mlt_common.h"
#include "mlt_gemm.h"
#include "mlt_gemm_tile.h"
#include "mlt_kernels.h"

namespace mlt {

enum PersistEpi { PE_PLAIN = 0, PE_GELU = 1, PE_RES = 2, PE_DGELU = 3, PE_GENERIC = 4 };

#define MLT_PPP_SYNC_READS()                                             \
  do {                                                                   \
    __builtin_amdgcn_sched_barrier(0);                                   \
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");      \
    __builtin_amdgcn_sched_barrier(0);                                   \
  } while (0)
#define MLT_PPP_BARRIER()                                                \
  do {                                                                   \
    __builtin_amdgcn_sched_barrier(0);                                   \
    asm volatile("s_barrier" ::: "memory");                              \
    __builtin_amdgcn_sched_barrier(0);                                   \
  } while (0)

template <int V>
using PIC = std::integral_constant<int, V>;

template <bool BNL, typename OutT, int F8A, int F8B, int EK>
__global__ __launch_bounds__(T_NT, 1) void gemm_ppp_kernel(const uint8_t* __restrict__ A,
                                                           const uint8_t* __restrict__ B, OutT* __restrict__ C, int M,
                                                           int N, int K, int64_t lda, int64_t ldb, int64_t ldc,
                                                           GemmEpi epi, int group_m) {
  constexpr int BM = 256, BN = 256, HALF = 16384, BUF = 4 * HALF, NF = 32;
  constexpr bool F8 = F8A >= 0;
  constexpr int ES = F8 ? 1 : 2;
  static_assert(!F8 || (F8B >= 0 && !BNL), "fp8 operands must both be fp8 and k-contiguous");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN, T = tiles_m * tiles_n;
  const int G = gridDim.x;
  const int id = xcd_remap(blockIdx.x, G);
  if (id >= T) return;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, cl = lane & 15;
  const int wr = wid >> 2, wc = wid & 3;
  const int nk = K / (F8 ? 128 : T_BK);
  const int U = ((T - id + G - 1) / G) * nk;  // K-tiles of all this workgroup's tiles, in order
  MLT_DCHECK(nk >= 2 && nk % 2 == 0 && K % (F8 ? 128 : T_BK) == 0);
  const int gm_ = group_m > 0 ? group_m : tiles_m;
  // origin of the workgroup's j-th tile (wave-uniform scalar math with divisions: evaluated once
  // per tile transition, never per stage -- the load sections of the ping-pong phases have to
  // fit under the other wave group's MFMA cluster)
  auto origin_j = [&](int j, int& m0, int& n0) __attribute__((always_inline)) {
    const int t = id + j * G;
    const int per_group = gm_ * tiles_n, grp = t / per_group, first_m = grp * gm_;
    const int gsize = min(tiles_m - first_m, gm_), r = t - grp * per_group;
    m0 = (first_m + r % gsize) * BM;
    n0 = (r / gsize) * BN;
  };
  int jt = 0, ukt = 0;  // current tile (index in this workgroup's list) and its K-tile of the stream position
  int cm0, cn0, nm0, nn0;
  origin_j(0, cm0, cn0);
  origin_j(1, nm0, nn0);  // (past the end: never staged, the loop bound stops first)
  const int64_t astep = 128, bstep = BNL ? (int64_t)T_BK * ldb * ES : 128;
  // stage half h (0 A0, 1 A1, 2 B0, 3 B1) of the K-tile d positions ahead of the current one
  auto stage = [&](auto hc, int buf, int d) __attribute__((always_inline)) {
    constexpr int h = decltype(hc)::value;
    int kt = ukt + d;
    const bool nxt = kt >= nk;
    kt -= nxt ? nk : 0;
    const int m0 = nxt ? nm0 : cm0, n0 = nxt ? nn0 : cn0;
    uint8_t* dst = smem + buf * BUF + h * HALF;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const uint32_t off = h < 2 ? glds_off<128, false, ES>(lda, i, m0 + (h & 1) * 128, M)
                                 : glds_off<128, BNL, ES>(ldb, i, n0 + (h & 1) * 128, N);
      const uint8_t* base = h < 2 ? A + (int64_t)kt * astep : B + (int64_t)kt * bstep;
      __builtin_amdgcn_global_load_lds((const void*)(base + off), (lds_void*)(dst + (i * T_NT + wid * 64) * 16), 16, 0,
                                       0);
    }
  };

  f32x4 acc[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[4][2], bfr[2][2];
  i32x8 af8[4], bf8[2];
  auto read_a = [&](const uint8_t* hb) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (F8) {
        af8[i] = tfrag_f8(hb, wr * 64 + 16 * i);
      } else {
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) af[i][kh] = tfrag_k(hb, wr * 64 + 16 * i, kh);
      }
    }
  };
  auto read_b = [&](const uint8_t* hb) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if constexpr (F8) {
        bf8[j] = tfrag_f8(hb, wc * 32 + 16 * j);
      } else {
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
          bfr[j][kh] = BNL ? tfrag_mn<256>(hb, wc * 32 + 16 * j, kh) : tfrag_k(hb, wc * 32 + 16 * j, kh);
      }
    }
  };
  auto mma = [&](auto qmc, auto qnc) __attribute__((always_inline)) {
    constexpr int qm = decltype(qmc)::value, qn = decltype(qnc)::value, f0 = (qm * 2 + qn) * 8;
    __builtin_amdgcn_s_setprio(1);
    if constexpr (F8) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)  // swapped operands: D = C^T fragment (formats follow operands)
          acc[f0 + i * 2 + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bf8[j], af8[i], acc[f0 + i * 2 + j],
                                                                                  F8B, F8A, 0, 127, 0, 127);
    } else {
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[f0 + i * 2 + j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j][kh], af[i][kh], acc[f0 + i * 2 + j], 0, 0, 0);
    }
#pragma unroll
    for (int f = 0; f < 8; ++f) asm volatile("" ::"v"(acc[f0 + f]));
    __builtin_amdgcn_s_setprio(0);
  };
  auto phase = [&](auto qc, auto shc, const uint8_t* rb, int sbuf, int sd, bool do_stage, int wait)
                   __attribute__((always_inline)) {
    constexpr int q = decltype(qc)::value;
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
    if (do_stage) stage(shc, sbuf, sd);
    if (wait == 6)
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (wait == 0)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    MLT_PPP_SYNC_READS();
    if constexpr (q == 0) mma(PIC<0>{}, PIC<0>{});
    else if constexpr (q == 1) mma(PIC<0>{}, PIC<1>{});
    else if constexpr (q == 2) mma(PIC<1>{}, PIC<1>{});
    else mma(PIC<1>{}, PIC<0>{});
    MLT_PPP_BARRIER();
  };

  float alpha = epi.alpha;
  if (epi.inv_scale_a) alpha *= *epi.inv_scale_a;
  if (epi.inv_scale_b) alpha *= *epi.inv_scale_b;

  // ---- register epilogue of the tile at (m0, n0) ------------------------------------------------
  // accumulator f = (qm * 2 + qn) * 8 + i * 2 + j: lane (g, cl) holds
  // C[m0 + qm*128 + wr*64 + 16 i + cl][n0 + qn*128 + wc*32 + 16 j + 4 g .. +3]
  auto epilogue = [&](const int m0, const int n0) __attribute__((always_inline)) {
    float4 bv[4];  // bias of the lane's 4 column groups (qn, j)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int gn = n0 + (c >> 1) * 128 + wc * 32 + 16 * (c & 1) + 4 * g;
      bv[c] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (epi.bias) {
        if (gn + 4 <= N) {
          bv[c] = *reinterpret_cast<const float4*>(epi.bias + gn);
        } else {
          float tmp[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) tmp[e] = gn + e < N ? epi.bias[gn + e] : 0.f;
          bv[c] = make_float4(tmp[0], tmp[1], tmp[2], tmp[3]);
        }
      }
    }
    auto fr = [&](int f, int& gm, int& gn) __attribute__((always_inline)) {
      const int qd = f >> 3, i = (f >> 1) & 3, j = f & 1;
      gm = m0 + (qd >> 1) * 128 + wr * 64 + 16 * i + cl;
      gn = n0 + (qd & 1) * 128 + wc * 32 + 16 * j + 4 * g;
    };
    const bool interior = m0 + BM <= M && n0 + BN <= N;
    if (EK != PE_GENERIC && interior) {
      // side-operand kinds work in quarter tiles (8 side loads = 16 VGPRs beside the 128 of the
      // accumulators: the kernel sits at the 256-VGPR cap), plain ones in one pass
      constexpr int SC = (EK == PE_RES || EK == PE_DGELU) ? 8 : NF;
#pragma unroll
      for (int hh = 0; hh < NF / SC; ++hh) {  // side loads of the chunk first, then its stores back to back
        ushort4 sd[SC];
        if constexpr (EK == PE_RES || EK == PE_DGELU) {
          const uint16_t* sx = EK == PE_RES ? epi.res : epi.aux;
          const int64_t ldx = EK == PE_RES ? epi.ldres : epi.ldaux;
#pragma unroll
          for (int k = 0; k < SC; ++k) {
            int gm, gn;
            fr(hh * SC + k, gm, gn);
            sd[k] = *reinterpret_cast<const ushort4*>(sx + (int64_t)gm * ldx + gn);
          }
        }
#pragma unroll
        for (int k = 0; k < SC; ++k) {
          const int f = hh * SC + k;
          int gm, gn;
          fr(f, gm, gn);
          const float4 b = bv[((f >> 3) & 1) * 2 + (f & 1)];
          float v[4] = {acc[f][0] * alpha + b.x, acc[f][1] * alpha + b.y, acc[f][2] * alpha + b.z,
                        acc[f][3] * alpha + b.w};
          if constexpr (EK == PE_GELU) {  // keep the (bf16-rounded) pre-activation for the backward
            ushort4 a;
            a.x = f32_to_bf16(v[0]);
            a.y = f32_to_bf16(v[1]);
            a.z = f32_to_bf16(v[2]);
            a.w = f32_to_bf16(v[3]);
            *reinterpret_cast<ushort4*>(const_cast<uint16_t*>(epi.aux) + (int64_t)gm * epi.ldaux + gn) = a;
            v[0] = gelu_f(bf16_to_f32(a.x));
            v[1] = gelu_f(bf16_to_f32(a.y));
            v[2] = gelu_f(bf16_to_f32(a.z));
            v[3] = gelu_f(bf16_to_f32(a.w));
          } else if constexpr (EK == PE_RES) {
            v[0] += bf16_to_f32(sd[k].x);
            v[1] += bf16_to_f32(sd[k].y);
            v[2] += bf16_to_f32(sd[k].z);
            v[3] += bf16_to_f32(sd[k].w);
          } else if constexpr (EK == PE_DGELU) {
            v[0] *= gelu_grad(bf16_to_f32(sd[k].x));
            v[1] *= gelu_grad(bf16_to_f32(sd[k].y));
            v[2] *= gelu_grad(bf16_to_f32(sd[k].z));
            v[3] *= gelu_grad(bf16_to_f32(sd[k].w));
          }
          OutT* cp = C + (int64_t)gm * ldc + gn;
          if constexpr (sizeof(OutT) == 4) {
            *reinterpret_cast<float4*>(cp) = make_float4(v[0], v[1], v[2], v[3]);
          } else {
            ushort4 o;
            o.x = f32_to_bf16(v[0]);
            o.y = f32_to_bf16(v[1]);
            o.z = f32_to_bf16(v[2]);
            o.w = f32_to_bf16(v[3]);
            *reinterpret_cast<ushort4*>(cp) = o;
          }
        }
      }
    } else {
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        int gm, gn;
        fr(f, gm, gn);
        if (gm >= M || gn >= N) continue;
        const float4 b = bv[((f >> 3) & 1) * 2 + (f & 1)];
        float vv[4] = {acc[f][0] * alpha + b.x, acc[f][1] * alpha + b.y, acc[f][2] * alpha + b.z,
                       acc[f][3] * alpha + b.w};
        epilogue_store4<OutT>(C, ldc, epi, gm, gn, N, vv);
      }
    }
#pragma unroll
    for (int f = 0; f < NF; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  // prologue: K-tile 0 -> E (all four halves), 1 -> O (A0, B1, A1; B0 comes in phase 1)
  stage(PIC<0>{}, 0, 0);
  stage(PIC<3>{}, 0, 0);
  stage(PIC<1>{}, 0, 0);
  stage(PIC<2>{}, 0, 0);
  stage(PIC<0>{}, 1, 1);
  stage(PIC<3>{}, 1, 1);
  stage(PIC<1>{}, 1, 1);
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  MLT_PPP_BARRIER();
  const bool late = __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256;  // group 1: wave-uniform branch
  if (late) MLT_PPP_BARRIER();
  const uint8_t* E = smem;
  const uint8_t* O = smem + BUF;
  for (int u = 0; u < U; u += 2) {
    const bool e2 = u + 2 < U, o3 = u + 3 < U;
    phase(PIC<0>{}, PIC<2>{}, E, 1, 1, true, -1);
    phase(PIC<1>{}, PIC<0>{}, E, 0, 2, e2, -1);
    phase(PIC<2>{}, PIC<3>{}, E, 0, 2, e2, -1);
    phase(PIC<3>{}, PIC<1>{}, E, 0, 2, e2, e2 ? 6 : 0);
    phase(PIC<0>{}, PIC<2>{}, O, 0, 2, e2, -1);
    phase(PIC<1>{}, PIC<0>{}, O, 1, 3, o3, -1);
    phase(PIC<2>{}, PIC<3>{}, O, 1, 3, o3, -1);
    phase(PIC<3>{}, PIC<1>{}, O, 1, 3, o3, o3 ? 6 : 0);
    ukt += 2;
    if (ukt == nk) {  // the tile's last K-tile pair is done: epilogue, then the next tile
      epilogue(cm0, cn0);
      ukt = 0;
      ++jt;
      cm0 = nm0;
      cn0 = nn0;
      origin_j(jt + 1, nm0, nn0);
    }
  }
  if (!late) MLT_PPP_BARRIER();  // both groups have now executed the same number of barriers
}
#undef MLT_PPP_SYNC_READS
#undef MLT_PPP_BARRIER

template <bool BNL, typename OutT, int F8A, int F8B, int EK>
static void launch_ek(const uint8_t* A, const uint8_t* B, OutT* C, int M, int N, int K, int64_t lda, int64_t ldb,
                      int64_t ldc, const GemmEpi& e, int group_m, int grid, hipStream_t st) {
  constexpr int SMEM = 2 * 4 * 16384;
  auto kern = gemm_ppp_kernel<BNL, OutT, F8A, F8B, EK>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(grid), dim3(T_NT), SMEM, st, A, B, C, M, N, K, lda, ldb, ldc, e, group_m);
}

template <bool AM, bool BNL, typename OutT, int F8A, int F8B>
void launch_gemm_persist(const uint8_t* A, const uint8_t* B, OutT* C, int M, int N, int K, int64_t lda, int64_t ldb,
                         int64_t ldc, const GemmEpi& e, int group_m, int max_blocks, hipStream_t st) {
  static_assert(!AM, "persistent kernel: A must be k-contiguous");
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  const int grid = tiles < max_blocks ? tiles : max_blocks;
  // branch-free vector epilogue: 8-byte (bf16) / 16-byte (fp32) aligned rows and side operands
  auto al = [](const void* p, int64_t ld, int esz) {
    return p == nullptr || ((((uintptr_t)p) % 16) == 0 && (ld * esz) % 16 == 0);
  };
  const bool vec = N % 4 == 0 && al(C, ldc, (int)sizeof(OutT)) && al(e.res, e.ldres, 2) && al(e.aux, e.ldaux, 2) &&
                   !e.accumulate && (e.bias == nullptr || ((uintptr_t)e.bias) % 16 == 0);
  int ek = PE_GENERIC;
  if (vec && sizeof(OutT) == 4) {  // fp32 outputs (tests, fp32 consumers): plain fast path only
    if (e.mode == 0 && !e.res) ek = PE_PLAIN;
  } else if (vec) {
    if (e.mode == 0 && !e.res) ek = PE_PLAIN;
    else if (e.mode == 1 && !e.res) ek = PE_GELU;
    else if (e.mode == 0 && e.res) ek = PE_RES;
    else if (e.mode == 2 && !e.res) ek = PE_DGELU;
  }
  if (ek == PE_PLAIN) {
    launch_ek<BNL, OutT, F8A, F8B, PE_PLAIN>(A, B, C, M, N, K, lda, ldb, ldc, e, group_m, grid, st);
  } else if (ek == PE_GENERIC) {
    launch_ek<BNL, OutT, F8A, F8B, PE_GENERIC>(A, B, C, M, N, K, lda, ldb, ldc, e, group_m, grid, st);
  } else if constexpr (sizeof(OutT) == 2) {
    if (ek == PE_GELU)
      launch_ek<BNL, OutT, F8A, F8B, PE_GELU>(A, B, C, M, N, K, lda, ldb, ldc, e, group_m, grid, st);
    else if (ek == PE_RES)
      launch_ek<BNL, OutT, F8A, F8B, PE_RES>(A, B, C, M, N, K, lda, ldb, ldc, e, group_m, grid, st);
    else
      launch_ek<BNL, OutT, F8A, F8B, PE_DGELU>(A, B, C, M, N, K, lda, ldb, ldc, e, group_m, grid, st);
  }
}

#define MLT_PERSIST_INST(AMV, BNV, OT, FA, FB)                                                                  \
  template void launch_gemm_persist<AMV, BNV, OT, FA, FB>(const uint8_t*, const uint8_t*, OT*, int, int, int, \
                                                          int64_t, int64_t, int64_t, const GemmEpi&, int, int,   \
                                                          hipStream_t);
#ifndef MLT_PERSIST_FP8
MLT_PERSIST_INST(false, false, uint16_t, -1, -1)
MLT_PERSIST_INST(false, false, float, -1, -1)
MLT_PERSIST_INST(false, true, uint16_t, -1, -1)
MLT_PERSIST_INST(false, true, float, -1, -1)
#else
MLT_PERSIST_INST(false, false, uint16_t, 0, 0)
MLT_PERSIST_INST(false, false, float, 0, 0)
MLT_PERSIST_INST(false, false, uint16_t, 1, 0)
MLT_PERSIST_INST(false, false, float, 1, 0)
MLT_PERSIST_INST(false, false, uint16_t, 0, 1)
MLT_PERSIST_INST(false, false, float, 0, 1)
#endif
#undef MLT_PERSIST_INST

}  // namespace mlt
