// LeNet-5 CIFAR training step (reference src/model.py:7-24, src/trainer.py:180-197) in bf16 on the
// CDNA4 matrix cores: TWO launches per step, whatever the batch.
//
//   KS  lenet_ms<D>  grid B x 1024 threads, one CU per sample, the whole per-sample chain in LDS:
//       [staged / augmented input] -> conv1 (MFMA) + bias + ReLU + maxpool -> conv2 (MFMA) + bias +
//       ReLU + maxpool -> fc1 / fc2 / fc3 (+ReLU, MFMA) -> softmax-CE -> fc dgrad chain (MFMA) ->
//       unpool2 -> conv2 dgrad (MFMA) -> pool1 liveness mask -> conv2 wgrad (MFMA) and conv1 wgrad
//       (MFMA) of the sample -> per-sample weight-gradient slab; + the NEXT step's raw input image
//       gathered (epoch permutation -> dataset row) and staged by an otherwise idle wave, so the
//       next step starts with one round trip instead of ctrl -> perm -> image.
//       The ~250 KB of fc weight fragments a CU fetches per step are the other cost besides the
//       latency chain (a CU's vector memory path moves ~35 B/clk and a wave stalls while its loads
//       queue), so fetches go to waves without work in that phase: waves 8-15 fetch fc1 while 0-7
//       run conv1; from conv2 to the fc1 dgrad the waves form two roles (two branches with the
//       same barrier sequence): 0-7 fetch and run the fc dgrad chain, 8-15 run conv2, the forward
//       chain and the CE.
//   KW  lenet_mw<D>  role-split grid: conv slab sums over the batch (sample order), fc weight
//       gradients over the batch (exact-f32 MFMA tiles, sample-ordered), the fused optimizer update
//       (fp32 masters + bf16 shadow + the per-sample kernel's fragment images), the fixed-order loss
//       / accuracy sums, the step-counter advance.
//
// Why this shape (measured on the fp32 four-kernel step, profiles/pmc/lenet_fp32_b{4,32}_r3.jsonl): every
// kernel of that step sat 55-70 % of its wave cycles in s_waitcnt / barriers, and the step took
// 30.5 us at batch 4 against 32.1 us at batch 32 -- it is a chain of latencies (kernel boundaries,
// dependent global round trips, LDS-barrier phases), not of FLOPs. A CU per sample removes the
// cross-CU hand-offs inside the sample's chain; bf16 MFMA (16x the f32 VALU rate) makes the conv
// phases short enough to run on one CU (an f32 conv1 alone is >= 1.2 us of one CU's FMA issue).
// Mixed precision as BASELINE.json configs 2/3 ("default config bf16"): bf16 operands for the
// conv GEMMs and the fc weights, fp32 accumulation, fp32 activations through the fc chain, fp32
// master weights and optimizer state.
//
// GEMM formulations (v_mfma_f32_16x16x32_bf16; lane l holds A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15],
// C rows 4(l>>4)+r / column l&15):
//   conv1 fwd   M = 196 pooled cells x 2 window rows, N = (out channel, window column), K = (kh, x
//               pair, c4) from the [Y][X][c4] bf16 image (one 16-byte read per fragment); the 2x2
//               pool is in registers (own rows + the partner lane's column, one DPP swap)
//   conv2 fwd   M = 25 cells x 4, N = out channel, K = (tap, ic8) from the [y][x][ic8] p1 image
//   conv2 dgrad M = 196 positions, N = in channel, K = (tap, oc16) from the zero-padded [18][18][oc16]
//               image of the unpooled conv2-output gradient
//   conv2 wgrad M = (kw | ic, kh) taps (+ an all-ones row = bias), N = out channel, K = positions;
//               the A fragment is an 8-wide row window shifted by kw (wave-uniform: v_alignbyte)
//   conv1 wgrad M = (kw | c, kh) taps (+ ones row), N = out channel, K = the 28x32 positions of the
//               unpooled conv1 gradient; split over 3 K-ranges, summed in a fixed order
// All batch reductions (KW) run in sample order: results are bitwise reproducible run to run.
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "mlt_common.h"
#include "mlt_kernels.h"
#include "mlt_optim.h"

namespace mlt {
namespace lm {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

// Workgroup barrier for LDS hand-offs only: drains this wave's LDS (and scalar) operations and
// meets the other waves. Unlike __syncthreads() it never waits for outstanding global loads, so
// prefetches (the fc weights, the next step's image) stay in flight across phases.
__device__ __forceinline__ void lbar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// 8 consecutive bf16 starting KW elements into the 16-element window lo ++ hi
template <int KW>
__device__ __forceinline__ u32x4 fshift(u32x4 lo, u32x4 hi) {
  const unsigned d[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  constexpr int k0 = KW >> 1;
  u32x4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    r[j] = (KW & 1) ? __builtin_amdgcn_alignbyte(d[k0 + j + 1], d[k0 + j], 2) : d[k0 + j];
  return r;
}

// Block-uniform scalar read (s_load through the constant address space: lgkmcnt, not vmcnt, so
// waiting for it never waits for the vector prefetches in flight). Only for data this kernel does
// not write before the read; every write in this file is a vector store.
template <class T>
__device__ __forceinline__ T sload(const T* p) {
  typedef const __attribute__((address_space(4))) T* cptr;
  return *(cptr)(p);
}

__device__ __forceinline__ unsigned pack2(uint16_t lo, uint16_t hi) { return (unsigned)lo | ((unsigned)hi << 16); }

// conv weight B-fragment image (bf16, 13312 entries = 26 KB): [w1f 4 ksteps][w2f 7][w2d 15], each
// [kstep][lane][8]. Slot of a parameter element (inverse of the fragment decode in lenet_ms):
//   conv1 fwd   k = ((kh*3 + i) * 2 + p) * 4 + c, n = 2 oc + dx, with kw = 2 i + p - dx: every
//               weight sits in two columns (output x parity dx = 0 / 1, the pool window's x)
//   conv2 fwd   k = tap * 8 + ic,                       n = oc
//   conv2 dgrad k = ((kh*6 + u) * 16 + oc, n = 2 ic + dx, with kw = u - 1 + dx (two columns per
//               weight, as conv1: the dgrad output's x parity dx is in N)
constexpr int kW1F = 0, kW2F = 4 * 512, kW2D = 11 * 512, kWimg = 26 * 512;
// followed by the fc weights the per-sample kernel cannot read from the row-major shadow with 16-byte
// lanes: every layer TRANSPOSED ([in][out], the backward-data B operand) and fc3 with its rows padded
// to 8 elements; row pitches padded to 8 elements, padding zero. Sized for the largest config.
constexpr int cmax(int a, int b) { return a > b ? a : b; }
constexpr int cmin(int a, int b) { return a < b ? a : b; }
constexpr int kFc1T = kWimg;               // [FLAT][F1]
constexpr int kFc2T = kFc1T + 400 * 120;   // [F1][round8(F2)]
constexpr int kFc3F = kFc2T + 120 * 88;    // [NC][round8(F2)]
constexpr int kFc3T = kFc3F + 10 * 88;     // [F2][round8(NC)]
constexpr int kWimgTot = kFc3T + 84 * 16;
constexpr int round8(int v) { return (v + 7) / 8 * 8; }
__device__ __forceinline__ int w1f_slot(int oc, int c, int kh, int kw, int dx) {
  const int u = kw + dx, qq = kh * 3 + (u >> 1);
  return kW1F + (((qq >> 2) * 64 + (qq & 3) * 16 + 2 * oc + dx) << 3) + ((u & 1) << 2) + c;
}
__device__ __forceinline__ int w2f_slot(int oc, int ic, int tap) {
  return kW2F + (((tap >> 2) * 64 + (tap & 3) * 16 + oc) << 3) + ic;
}
__device__ __forceinline__ int w2d_slot(int oc, int ic, int tap, int dx) {
  const int kh = tap / 5, u = tap - 5 * kh + 1 - dx, pp = kh * 6 + u;
  return kW2D + (((pp >> 1) * 64 + ((((pp & 1) << 1) | (oc >> 3)) * 16) + 2 * ic + dx) << 3) + (oc & 7);
}
// parameter element behind image entry e (or -1: padding), given the flat offsets of w1 / w2
template <int C1, int C2>
__device__ __forceinline__ int64_t wimg_src(int e, int64_t off_w1, int64_t off_w2) {
  const int s = (e & 4095) >> 9;
  if (e < kW2F) {
    const int l = (e >> 3) & 63, j = e & 7, n = l & 15, qq = 4 * (e >> 9) + (l >> 4);
    const int kh = qq / 3, oc = n >> 1, kw = 2 * (qq - 3 * kh) + (j >> 2) - (n & 1), c = j & 3;
    return (qq < 15 && oc < C1 && kw >= 0 && kw < 5 && c < 3) ? off_w1 + ((oc * 3 + c) * 5 + kh) * 5 + kw : -1;
  }
  if (e < kW2D) {
    const int q = e - kW2F, l = (q >> 3) & 63, j = q & 7, oc = l & 15, tap = 4 * (q >> 9) + (l >> 4);
    return (tap < 25 && oc < C2 && j < C1) ? off_w2 + (oc * C1 + j) * 25 + tap : -1;
  }
  const int q = e - kW2D, l = (q >> 3) & 63, j = q & 7, n = l & 15, gg = l >> 4;
  const int pp = 2 * (q >> 9) + (gg >> 1), oc = 8 * (gg & 1) + j, ic = n >> 1, kh = pp / 6;
  const int kw = pp - 6 * kh - 1 + (n & 1);
  (void)s;
  return (pp < 30 && ic < C1 && oc < C2 && kw >= 0 && kw < 5) ? off_w2 + (oc * C1 + ic) * 25 + kh * 5 + kw : -1;
}

template <int C1_, int C2_, int F1_, int F2_, int NC_>
struct Dm {
  static constexpr int C1 = C1_, C2 = C2_, F1 = F1_, F2 = F2_, NC = NC_, FLAT = C2_ * 25;
  static_assert(C1_ <= 8 && C2_ <= 16 && C2_ % 4 == 0 && F1_ % 4 == 0 && F2_ % 4 == 0 && NC_ <= 64, "dims");
  // per-sample weight-gradient slab: [conv1: oc*76 + tap (75 = bias)] [conv2: natural order, then bias]
  static constexpr int S1 = C1 * 76, S2OFF = (S1 + 3) & ~3, S2 = C2 * C1 * 25 + C2;
  static constexpr int SLABN = (S2OFF + S2 + 15) & ~15;
};
using DmDefault = Dm<6, 16, 120, 84, 10>;
using DmTiny = Dm<4, 8, 64, 32, 10>;

constexpr int kT = 1024;        // KS threads (16 waves)
constexpr int XCS = 48;          // [c][Y][X] image row stride (X >= 32 zero: shifted 8-wide windows)
constexpr int P1CS = 32;         // [ic][y][x] pooled-conv1 image row stride (x >= 14 zero)
// LDS row strides chosen against bank conflicts of the MFMA operand reads (64 banks x 4 B; the
// strides of the natural layouts map the rows a fragment gathers onto the same banks):
constexpr int XHS = 48;          // [Y][X][c4] input image: pixels per row (conv1 A, 1.7-way vs 2.4 at 32)
constexpr int P1HS = 24;         // [y][x][ic8] pooled conv1: pixels per row (conv2 A, 1.5-way vs 1.9)
constexpr int DCHS = 19;         // [Y+4][X+4][oc16] padded conv2-output grad: pixels per row (dgrad A, 1-way)
constexpr int DCCS = 24;         // [oc][Y][X] conv2-output grad: row stride (conv2 wgrad B, 1-way)
constexpr int D1S = 28 * 32 + 16;  // [oc][Y][X32] unpooled conv1 grad: channel stride (conv1 wgrad B, 1-way vs 5)
constexpr int kWgT = 256;        // KW threads
constexpr int kP13W = 7;         // conv1 wgrad waves (28 output rows / 4 each)
#ifndef MLT_KC1W
#define MLT_KC1W 8  // (build-time A/B knob)
#endif
constexpr int kC1W = MLT_KC1W;   // conv1 forward waves (the fc1 forward waves 8-15 fetch weights meanwhile)

// ---------------------------------------------------------------------------
// fc layers on the matrix cores: y = W x for ONE sample, its input row x (bf16 in LDS, zero past K
// up to the k-step multiple) broadcast over the 16 A rows; a wave owns a tile of 16 outputs and all
// K steps, its B fragments (W rows, 16 contiguous bytes per lane) in registers. Rows / chunks past
// the matrix re-read its last ones: their products meet zero A columns or land in unstored outputs.
// ---------------------------------------------------------------------------
constexpr int pow2_ge(int v) { return v <= 1 ? 1 : v <= 2 ? 2 : v <= 4 ? 4 : v <= 8 ? 8 : v <= 16 ? 16 : v <= 32 ? 32 : 64; }

template <int KS, int LD, int N, int K>
__device__ __forceinline__ void frag_rows(u32x4 (&f)[KS], const uint16_t* __restrict__ W, int tn) {
  const unsigned lane = threadIdx.x & 63;
  const unsigned row = min(16u * tn + (lane & 15), (unsigned)N - 1);
#pragma unroll
  for (int q = 0; q < KS; ++q) {
    const unsigned col = min(32u * q + 8 * (lane >> 4), (unsigned)((K - 1) / 8 * 8));
    f[q] = *reinterpret_cast<const u32x4*>(W + row * LD + col);
  }
}
// output 16 tn + lane of the tile, valid in lanes 0-15 (all 16 C rows are equal)
template <int KS>
__device__ __forceinline__ float row_dot(const u32x4 (&f)[KS], const uint16_t* x) {
  const int g = (threadIdx.x & 63) >> 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < KS; ++q) acc = mfma(*reinterpret_cast<const u32x4*>(x + 32 * q + 8 * g), f[q], acc);
  return acc[0];
}

// fc1 dgrad B fragment of k-step q for output tile `tile` from the LDS fc1 image (KsLds::F1S layout):
// lane (g, i = 4 qq + p) needs W1[32 q + 8 g + j][16 tile + i], j = 0..7 -- a column of the
// row-major image. Two ds_read_b64_tr_b16 (rows 32q + 8g + qq and + 4, columns 16 tile + 4p .. + 3
// supplied per lane) deliver it transposed. Rows past F1 re-read row F1 - 1 (their A column, the
// fc1 output gradient, is zero there); columns past FLAT re-read the last four (outputs not stored).
// Every lane must execute the reads (EXEC all ones: the gather crosses lanes).
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
template <int F1, int FLAT, int F1S>
__device__ __forceinline__ u32x4 f1t_frag(const uint16_t* img, int tile, int q) {
  const int lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15, qq = i >> 2, p = i & 3;
  const int col = min(16 * tile + 4 * p, FLAT - 4), c = col >> 3, e = col & 7;
  const int r0 = min(32 * q + 8 * g + qq, F1 - 1), r1 = min(32 * q + 8 * g + qq + 4, F1 - 1);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + (r0 * F1S + c + (r0 & 1)) * 8 + e));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + (r1 * F1S + c + (r1 & 1)) * 8 + e));
  return u32x4{(unsigned)(uint16_t)lo[0] | ((unsigned)(uint16_t)lo[1] << 16),
               (unsigned)(uint16_t)lo[2] | ((unsigned)(uint16_t)lo[3] << 16),
               (unsigned)(uint16_t)hi[0] | ((unsigned)(uint16_t)hi[1] << 16),
               (unsigned)(uint16_t)hi[2] | ((unsigned)(uint16_t)hi[3] << 16)};
}

// fc2 dgrad B fragment (as f1t_frag) from the XOR-swizzled fc2 image [F2][16 chunks] (KsLds::F2S)
template <int F2, int F1>
__device__ __forceinline__ u32x4 f2t_frag(const uint16_t* img, int tile, int q) {
  const int lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15, qq = i >> 2, p = i & 3;
  const int col = min(16 * tile + 4 * p, F1 - 4), c = col >> 3, e = col & 7;
  const int r0 = min(32 * q + 8 * g + qq, F2 - 1), r1 = min(32 * q + 8 * g + qq + 4, F2 - 1);
  auto pos = [](int r, int cc) { return r * 16 + (cc ^ (((r & 3) << 2) | ((r >> 2) & 3))); };
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + pos(r0, c) * 8 + e));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + pos(r1, c) * 8 + e));
  return u32x4{(unsigned)(uint16_t)lo[0] | ((unsigned)(uint16_t)lo[1] << 16),
               (unsigned)(uint16_t)lo[2] | ((unsigned)(uint16_t)lo[3] << 16),
               (unsigned)(uint16_t)hi[0] | ((unsigned)(uint16_t)hi[1] << 16),
               (unsigned)(uint16_t)hi[2] | ((unsigned)(uint16_t)hi[3] << 16)};
}

// The fc chain's wave schedule. Fragments (~150 KB per CU and step) are fetched where the issuing
// waves are otherwise idle or light -- the vector memory path of a CU moves them at ~35 B/clk and a
// wave stalls while its loads queue:
//   fc1 fwd  tiles on waves 8-15, fetched at P2 (these waves carry one conv1 tile, the others two)
//   fc2 fwd  tiles on waves 8-13, fetched at P3 (conv2 runs on 0-6); fc3 fwd + softmax-CE on wave 14,
//            fetched during fc2
//   fc3 / fc2 / fc1 dgrad on waves 0-7 (fc1: 3 tiles each, the 25th on wave 15): fetched by those
//   waves while waves 8-15 run the forward
template <class D>
struct Fc {
  static constexpr int T1 = (D::F1 + 15) / 16, K1 = (D::FLAT + 31) / 32, W1F = 16 - T1;  // fc1 fwd
  static_assert(W1F >= 8, "fc1 forward runs on the role-B waves 8-15");
  static constexpr int T2 = (D::F2 + 15) / 16, K2 = (D::F1 + 31) / 32, W2F = 8;           // fc2 fwd
  static constexpr int K3 = (D::F2 + 31) / 32, W3F = 14;                                  // fc3 fwd
  static constexpr int B3T = (D::F2 + 15) / 16, B3K = (D::NC + 31) / 32;                  // fc3 dgrad
  static constexpr int B2T = (D::F1 + 15) / 16, B2K = (D::F2 + 31) / 32;                  // fc2 dgrad
  static constexpr int B1T = (D::FLAT + 15) / 16, B1K = (D::F1 + 31) / 32;                // fc1 dgrad
  static constexpr int B1P = cmin(3, (B1T + 7) / 8);  // fc1 dgrad tiles per wave 0-7 (w + 8 j)
  static constexpr int P2T = round8(D::F2), P3F = round8(D::F2), P3T = round8(D::NC);
  static_assert(D::FLAT % 8 == 0 && D::F1 % 8 == 0 && D::F1 * D::FLAT <= 400 * 120, "fc1 fragments");
  static_assert(T1 <= 8 && T2 <= 6 && D::NC <= 16 && B3T <= 8 && B2T <= 8 && B1T <= 8 * B1P + 1, "fc waves");
  static_assert(D::F1 * P2T <= 120 * 88 && D::NC * P3F <= 10 * 88 && D::F2 * P3T <= 84 * 16, "fc images");
};

template <class D>
struct KsLds {
  using F = Fc<D>;
  static constexpr int SCR = kP13W * 5 * 256;
  // fc1 weight image [F1 rows][F1S 16-byte chunks]: row r holds W1[r][0 .. FLAT) (8 bf16 per chunk)
  // at chunks (r & 1) .. (r & 1) + FLAT/8 - 1 -- the one-chunk shift of odd rows makes the transposed
  // reads of the fc1 dgrad (ds_read_b64_tr_b16: 8 rows x 32 bytes per 32-lane half) conflict-free
  static constexpr int F1S = D::FLAT / 8 + 1;
  // fc2 weight image [F2 rows][16 chunks of 8 bf16]: chunk c of row r at position
  // c ^ ((r & 3) << 2 | (r >> 2) & 3) (256-byte rows: conflict-free transposed reads)
  static constexpr int F2S = 16;
  static_assert(D::F1 <= 8 * F2S, "fc2 image rows");
  alignas(16) uint16_t p1c[D::C1 * 14 * P1CS];       // pooled conv1 [ic][y][x] (zeroed at entry)
  alignas(16) uint16_t xc[3 * 32 * XCS];             // input [c][Y][X48] (X >= 32 zeroed separately)
  // P0 .. P3 the input / conv-forward images; P4c .. P7 the fc2 weight image (written from the fc2
  // forward's register fragments, read transposed by the fc2 dgrad)
  union V {
    struct Fw {
      alignas(16) uint16_t p1h[14 * P1HS * 8];       // pooled conv1 [y][x][ic8] (zeroed at entry)
      alignas(16) uint16_t xh[32 * XHS * 4];         // input [Y][X][c4] (c = 3 zero; X >= 32 never read)
      alignas(16) uint16_t w1f[4 * 64 * 8];          // conv1 B fragments [kstep][lane][8]
      alignas(16) uint16_t w2f[7 * 64 * 8];          // conv2 forward B fragments
      alignas(16) uint8_t raw[3072];                 // this step's raw image (staged or gathered)
    } f;
    alignas(16) uint16_t f2img[D::F2 * F2S * 8];
  } v;
  // bf16 A rows of the fc MFMAs (tails zero to the k-step multiple)
  alignas(16) uint16_t fb16[32 * F::K1];             // flattened pooled conv2 (fc1)
  alignas(16) uint16_t h1b[32 * F::K2];              // fc1 output (fc2)
  alignas(16) uint16_t h2b[32 * F::K3];              // fc2 output (fc3)
  alignas(16) uint16_t dlb[32 * F::B3K];             // logit gradient (fc3 dgrad)
  alignas(16) uint16_t dh2b[32 * F::B2K];            // fc2 output gradient (fc2 dgrad)
  alignas(16) uint16_t dh1b[32 * F::B1K];            // fc1 output gradient (fc1 dgrad)
  alignas(16) float df[D::FLAT];                     // its gradient
  alignas(16) float sh1[D::F1];
  alignas(16) float sh2[D::F2];
  alignas(16) float sdh1[D::F1];
  alignas(16) float sdh2[D::F2];
  alignas(16) float slog[64];
  alignas(16) float sdl[64];
  alignas(16) float f32[D::FLAT];                    // flattened pooled conv2, fp32 (stored for the fc1 wgrad)
  unsigned long long tr[32];                         // LENET_TRACE stamps
  double ce[2];                                      // this sample's (loss / B, hit / B)
  float b1s[16], b2s[16];
  alignas(16) float fb[D::F1 + D::F2 + D::NC];       // fc biases
  uint8_t i1[D::C1 * 196];
  uint8_t i2[D::FLAT];
  // P4a .. P8 the fc1 weight image (written from the fc1 forward's register fragments, read
  // transposed by the fc1 dgrad); P10 .. P13 the backward images, written (and zeroed) in P10
  union U {
    alignas(16) uint16_t f1img[D::F1 * F1S * 8];
    struct Bw {
      alignas(16) uint16_t dch[18 * DCHS * 16];      // unpooled conv2-out grad, padded [Y+4][X+4][oc16]
      alignas(16) uint16_t dcc[16 * 10 * DCCS];      // unpooled conv2-out grad [oc16][Y][X]
      alignas(16) uint16_t d1[D::C1 * D1S];          // unpooled conv1-out grad [oc][Y][X32]
      alignas(16) uint16_t w2d[15 * 64 * 8];         // conv2 dgrad B fragments
      alignas(16) float scr[SCR];                    // conv1 wgrad row-range partials
    } b;
  } u;
};

// RandomCrop(32, pad) + HFlip + ToTensor + Normalize of pixel (Y, X) from a raw HWC uint8 image
// in LDS (src/utils/functions.py:5-12): (u / 255 - mean) / std as one fma per channel
__device__ __forceinline__ void aug_pixel(const uint8_t* img, int Y, int X, int ci, int cj, bool fl, const LeNetAug& A,
                                          float v[3]) {
  const int sx = fl ? 31 - X : X;
  const int r = Y + ci - A.pad, q = sx + cj - A.pad;
  const bool in = (unsigned)r < 32u && (unsigned)q < 32u;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float u = in ? (float)img[(r * 32 + q) * 3 + c] : 0.f;
    v[c] = fmaf(u, A.ascale[c], A.ashift[c]);
  }
}

// h % span of the other kernels' hash (lenet.hip), exactly: the default RandomCrop padding 4 as a
// constant divisor (multiply-high), anything else through two 32-bit remainders -- not the
// generic 64-bit division (~250 instructions on the step's critical path)
__device__ __forceinline__ int hmod(uint64_t h, unsigned span) {
  if (span == 9u) return (int)(h % 9u);
  const unsigned hi = (unsigned)(h >> 32) % span, lo = (unsigned)h % span;
  const unsigned r32 = (0xffffffffu % span + 1u) % span;  // 2^32 mod span
  return (int)((hi * r32 + lo) % span);                    // < span^2 + span: 32 bits (pad < 2^14)
}

__device__ __forceinline__ void aug_params(const LeNetAug& A, int64_t step, int64_t pos, int& ci, int& cj, bool& fl) {
  const uint64_t h = mix64(mix64(A.seed + (uint64_t)step) ^ (uint64_t)pos);
  const unsigned span = 2 * A.pad + 1;
  ci = A.pad ? hmod(h, span) : 0;
  cj = A.pad ? hmod(h >> 20, span) : 0;
  fl = A.flip && ((h >> 40) & 1);
}

__device__ __forceinline__ void pool4(f32x4 a, float bias, float& pv, uint8_t& code) {
  float m = a[0];
  int k = 0;
  if (a[1] > m) { m = a[1]; k = 1; }
  if (a[2] > m) { m = a[2]; k = 2; }
  if (a[3] > m) { m = a[3]; k = 3; }
  m += bias;
  pv = m > 0.f ? m : 0.f;
  code = m > 0.f ? (uint8_t)k : (uint8_t)4;
}

// ---------------------------------------------------------------------------
// KS: the per-sample chain
// ---------------------------------------------------------------------------
template <class D>
// The pointers the first loads need lead the argument list as plain scalars: the file is built with
// kernarg preloading (build.py), so they arrive in SGPRs with the wave instead of behind an s_load
// of the kernarg segment (aggregates are never preloaded).
__global__ __launch_bounds__(kT) void lenet_ms(uint8_t* __restrict__ pstage2, int64_t* __restrict__ pmeta2,
                                               const int64_t* __restrict__ pctrl, const uint16_t* __restrict__ pwimg,
                                               int64_t* __restrict__ pmetaN, int mode, float inv_B, LeNetPtrs P,
                                               LeNetAug A, LeNetOpt O) {
  constexpr int C1 = D::C1, C2 = D::C2, FLAT = D::FLAT, F1 = D::F1, F2 = D::F2, NC = D::NC;
  using S = KsLds<D>;
  static_assert(offsetof(typename S::V::Fw, w2f) == offsetof(typename S::V::Fw, w1f) + 2 * kW2F,
                "forward fragment images must be contiguous");
  static_assert(sizeof(S) <= 160 * 1024, "LDS");
  __shared__ S L;
  // w is wave-uniform: readfirstlane makes the per-wave role branches scalar (uniform) branches,
  // so a role's pending loads never force waits on the other roles' code paths
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, g = lane >> 4, m = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  // LENET_TRACE: s_memtime stamps of block 0 per phase (P.trace: 32 8-byte slots; 100 MHz wall
  // stamps at 14, 15; sub-phase stamps at 16..)
  // (kept in LDS and stored at the end: a global store mid-kernel would make later vmcnt waits
  // wait for its completion too)
  auto stamp = [&](int k) {
    if (!(mode & LENET_TRACE)) return;
    lbar();
    __builtin_amdgcn_sched_barrier(0);
    unsigned long long c, wc;
    asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(c), "=s"(wc)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    if (t == 0) {
      L.tr[k] = c;
      if (k == 0) L.tr[14] = wc;
      if (k == 13) L.tr[15] = wc;
    }
  };
  stamp(0);
  unsigned long long tb0 = 0;
  if (mode & LENET_TRACE) tb0 = __builtin_amdgcn_s_memrealtime();

  // ---- P0: every independent load in flight together ----------------------------------------
  // straight-line and unconditional (ctrl / meta2 / stage2 are host-checked), ctrl first: the
  // only values needed before the others arrive (vmcnt retires in issue order)
  const bool aug = A.data != nullptr;
  const int64_t step = sload(pctrl), sie = sload(pctrl + 1);
  const int64_t mstep = sload(pmeta2 + 4 * b), mpos = sload(pmeta2 + 4 * b + 1), mtgt = sload(pmeta2 + 4 * b + 3);
  uint4 sraw = reinterpret_cast<const uint4*>(pstage2 + (int64_t)b * 3072)[min(t, 191)];
  const bool stage_on = aug && w == 15;  // next-step staging wave (see P2)
  // (vector loads, issued before the bulk: scalar ones would be waited for by every LDS barrier's
  // lgkmcnt(0), and the staging decision they feed is taken in P2, off the critical path)
  longlong2 mN01 = make_longlong2(-1, -1);
  long long mN2 = -1;
  if (stage_on) {
    mN01 = *reinterpret_cast<const longlong2*>(pmetaN + 4 * b);
    mN2 = pmetaN[4 * b + 2];
  }
  float xin[3] = {0.f, 0.f, 0.f};
  if (!aug) {
#pragma unroll
    for (int c = 0; c < 3; ++c) xin[c] = P.x[(int64_t)b * 3072 + c * 1024 + t];
  }
  // conv weight B-fragment images (bf16, packed by the optimizer / lenet_mpack): 24 KB, linear
  // (the forward fragments only: conv2's dgrad fragments follow in P3, off the critical path)
  const uint4* wimg4 = reinterpret_cast<const uint4*>(pwimg);
  constexpr int WIF = kW2D / 8, WID = (kWimg - kW2D) / 8;  // uint4s: forward part, dgrad part
  static_assert(WIF <= kT && WID <= kT, "fragment image staging");
  const uint4 wi0 = wimg4[min(t, WIF - 1)];
  const float b1v = P.b1[min(t, C1 - 1)], b2v = P.b2[min(t, C2 - 1)];
  constexpr int NFB = F1 + F2 + NC;
  const float fbv = t < F1 ? P.b3[t] : (t < F1 + F2 ? P.b4[min(t - F1, F2 - 1)] : P.b5[min(max(t - F1 - F2, 0), NC - 1)]);
  using F1M = typename S::F;
  constexpr int P2T = F1M::P2T, P3F = F1M::P3F, P3T = F1M::P3T;
  u32x4 f1w[F1M::K1];  // fc1 forward B fragments (row-major W rows of the shadow: 16 B per lane)
  // fc weights: issued once this step's image and conv fragments are in LDS (fc1: start of P2; fc2 /
  // fc3: start of P3, where conv1's registers are free), so that their transfer does not delay
  // those. Padding lanes re-read a valid lane's line (coalesced).
  auto load_fc = [&]() {
    if (mode & LENET_PROBE_NOF1W) {
#pragma unroll
      for (int q = 0; q < F1M::K1; ++q) f1w[q] = u32x4{0u, 0u, 0u, 0u};
    } else if (w >= F1M::W1F) {
      frag_rows<F1M::K1, FLAT, F1, FLAT>(f1w, P.shadow + O.off[4], w - F1M::W1F);
    }
  };
  __builtin_amdgcn_sched_barrier(0);  // keep the index math below behind the load issue
  int64_t pos = sie * A.batch_stride + b;
  if (aug && pos >= A.perm_len) pos %= A.perm_len;

  // ---- P1: input images, zero spans, weight fragment images -----------------------------------
  stamp(16);
  const bool hit = aug && mstep == step && mpos == pos;  // block-uniform
  int64_t tgt = 0;
  {
    // zero the pooled-conv1 images p1h, p1c and the X >= 32 columns of xc
    constexpr int ZH = (int)sizeof(L.v.f.p1h) / 16, ZC = (int)sizeof(L.p1c) / 16;
    static_assert(sizeof(L.v.f.p1h) % 16 == 0 && sizeof(L.p1c) % 16 == 0, "zero spans");
    for (int e = t; e < ZH + ZC; e += kT) {
      uint4* z = e < ZH ? reinterpret_cast<uint4*>(L.v.f.p1h) + e : reinterpret_cast<uint4*>(L.p1c) + (e - ZH);
      *z = make_uint4(0u, 0u, 0u, 0u);
    }
    if (t < 3 * 32 * 2) reinterpret_cast<uint4*>(L.xc + (t >> 1) * XCS + 32)[t & 1] = make_uint4(0u, 0u, 0u, 0u);
    if (t < 32 * F1M::K1 - FLAT) L.fb16[FLAT + t] = 0;
    if (t < 32 * F1M::K2 - F1) L.h1b[F1 + t] = 0;
    if (t < 32 * F1M::K3 - F2) L.h2b[F2 + t] = 0;
    if (t < 32 * F1M::B3K - NC) L.dlb[NC + t] = 0;
    if (t < 32 * F1M::B2K - F2) L.dh2b[F2 + t] = 0;
    if (t < 32 * F1M::B1K - F1) L.dh1b[F1 + t] = 0;
    uint4* wl = reinterpret_cast<uint4*>(L.v.f.w1f);  // w1f | w2f | w2d are contiguous
    if (t < WIF) wl[t] = wi0;
    if (t < NFB) L.fb[t] = fbv;
    if (t < 16) {
      L.b1s[t] = t < C1 ? b1v : 0.f;
      L.b2s[t] = t < C2 ? b2v : 0.f;
    }
  }
  const int Y0 = t >> 5, X0 = t & 31;
  uint2 px;
  if (aug) {
    // hit: the previous step staged this sample's raw image (one round trip, issued in P0);
    // miss (first step of an epoch, ...): perm -> image. Either way crop / flip / normalise here.
    // (the LDS write sits inside each branch: a write after the join would wait for the
    // conservative merge of both paths' pending loads -- i.e. for every prefetch in flight)
    if (!hit) {
      int64_t idx = sload(A.perm + pos);
      idx = idx < 0 ? 0 : (idx >= A.n ? A.n - 1 : idx);
      const uint4 graw = reinterpret_cast<const uint4*>(A.data + idx * 3072)[min(t, 191)];
      tgt = sload(P.dtargets + idx);
      if (t < 192) reinterpret_cast<uint4*>(L.v.f.raw)[t] = graw;
    } else {
      tgt = mtgt;
      if (t < 192) reinterpret_cast<uint4*>(L.v.f.raw)[t] = sraw;
    }
    int ci, cj;
    bool fl;
    aug_params(A, step, pos, ci, cj, fl);
    lbar();
    stamp(17);
    float v[3];
    aug_pixel(L.v.f.raw, Y0, X0, ci, cj, fl, A, v);
    px = make_uint2(pack2(f32_to_bf16(v[0]), f32_to_bf16(v[1])), pack2(f32_to_bf16(v[2]), 0));
  } else {
    px = make_uint2(pack2(f32_to_bf16(xin[0]), f32_to_bf16(xin[1])), pack2(f32_to_bf16(xin[2]), 0));
    tgt = sload(P.targets + b);
  }
  reinterpret_cast<uint2*>(L.v.f.xh)[Y0 * XHS + X0] = px;
  L.xc[(0 * 32 + Y0) * XCS + X0] = (uint16_t)(px.x & 0xffff);
  L.xc[(1 * 32 + Y0) * XCS + X0] = (uint16_t)(px.x >> 16);
  L.xc[(2 * 32 + Y0) * XCS + X0] = (uint16_t)(px.y & 0xffff);
  lbar();
  stamp(1);

  load_fc();
  // ---- P2: conv1 (MFMA) + bias + ReLU + maxpool in registers -> p1 images, i1 ------------------
  // M = (pooled cell, window y) rows, N = (out channel, window x) columns, K = (kh, x pair, c4): a
  // lane's accumulators are the window rows of two cells, the partner lane (n ^ 1) holds the other
  // window column. 25 tiles x 4 k-steps on waves 0-7; B fragments (4 x 16 B per lane) read once per wave.
  {
    u32x4 bw[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) bw[s] = *reinterpret_cast<const u32x4*>(L.v.f.w1f + (s * 64 + lane) * 8);
    const int a = m >> 2, r = m & 3, dx = m & 1, oc = m >> 1;
    const float bias = L.b1s[min(oc, 15)];
    // tiles on waves 0 .. kC1W-1 only: the other waves spend this phase issuing the fc1 forward
    // weight fetch (~100 KB, load_fc above), whose queueing would otherwise delay their tiles
    for (int T = w; w < kC1W && T < 25; T += kC1W) {
      const int cell = min(8 * T + 2 * a + (r >> 1), 195);
      const int py = cell / 14, pxx = cell - 14 * py, Y = 2 * py + (r & 1);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int qq = 4 * s + g, kh = qq / 3, i = qq - 3 * kh;
        u32x4 av = *reinterpret_cast<const u32x4*>(L.v.f.xh + ((qq < 15 ? (Y + kh) * XHS + 2 * pxx + 2 * i : 0)) * 4);
        if (qq >= 15) av = u32x4{0u, 0u, 0u, 0u};
        acc = mfma(av, bw[s], acc);
      }
      // rows 4g + r: cell 8T + 2g (r = 0, 1: window y) and 8T + 2g + 1 (r = 2, 3); column (oc, dx)
      float o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        o[k] = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(acc[k]), 0xB1, 0xf, 0xf, false));  // lane ^ 1
      // the dx = 0 lane pools the first cell, the dx = 1 lane the second; window order (y, x)
      const f32x4 win = dx == 0 ? f32x4{acc[0], o[0], acc[1], o[1]} : f32x4{o[2], acc[2], o[3], acc[3]};
      const int cc = 8 * T + 2 * g + dx;
      float pv;
      uint8_t code;
      pool4(win, bias, pv, code);
      if (oc < C1 && cc < 196) {
        const int cy = cc / 14, cx = cc - 14 * cy;
        const uint16_t hv = f32_to_bf16(pv);
        L.v.f.p1h[(cy * P1HS + cx) * 8 + oc] = hv;
        L.p1c[(oc * 14 + cy) * P1CS + cx] = hv;
        L.i1[oc * 196 + cc] = code;
      }
    }
  }
  lbar();
  stamp(2);

  const uint4 wid = wimg4[WIF + min(t, WID - 1)];  // conv2 dgrad fragments (to LDS in P10)

  // ---- P3-P7 as two wave roles (the same barrier sequence in both), then P8 on every wave ---------
  // waves 0-7 fetch the fc3 / fc2 dgrad fragments during conv2 and run that dgrad chain; waves 8-15
  // run conv2, the forward fc chain and the softmax-CE, put their fc1 forward fragments into the
  // LDS fc1 image (read back transposed by the fc1 dgrad: the transposed copy of fc1, ~96 KB per CU
  // and step, is no longer fetched) and do the next-step staging (wave 15). As two branches, each
  // role's register-resident fragments share registers with the other's.
  if (w < 8) {
    // ---- role A: fc3 / fc2 dgrad ----
    u32x4 f3t[F1M::B3K];
    if (w < F1M::B3T) frag_rows<F1M::B3K, P3T, F2, NC>(f3t, pwimg + kFc3T, w);
    lbar();  // P3 (conv2)
    stamp(3);
    lbar();  // P4a (fc1 forward)
    stamp(18);
    lbar();  // P4b (fc2 forward)
    stamp(19);
    lbar();  // P4c (fc3 forward + CE; role B fills the fc1 image)
    stamp(4);
    if (w < F1M::B3T) {  // fc3 dgrad (x the fc2 ReLU mask)
      const int k = 16 * w + m;
      const float v = row_dot(f3t, L.dlb);
      if (g == 0 && k < F2) {
        const float d = L.sh2[k] > 0.f ? v : 0.f;
        L.sdh2[k] = d;
        L.dh2b[k] = f32_to_bf16(d);
      }
    }
    lbar();
    stamp(20);
    if (w < F1M::B2T) {  // fc2 dgrad (x the fc1 ReLU mask), W2 read transposed from the fc2 image
      const int k = 16 * w + m;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < F1M::B2K; ++q)
        acc = mfma(*reinterpret_cast<const u32x4*>(L.dh2b + 32 * q + 8 * g), f2t_frag<F2, F1>(L.v.f2img, w, q), acc);
      const float v = acc[0];
      if (g == 0 && k < F1) {
        const float d = L.sh1[k] > 0.f ? v : 0.f;
        L.sdh1[k] = d;
        L.dh1b[k] = f32_to_bf16(d);
      }
    }
    lbar();
    stamp(21);
  } else {
    // ---- role B: conv2, forward fc chain, softmax-CE, fc1 image, next-step staging ----
    u32x4 f2w[F1M::K2], f3w[F1M::K3];
    if (mode & LENET_PROBE_NOF2) {
#pragma unroll
      for (int q = 0; q < F1M::K2; ++q) f2w[q] = u32x4{0u, 0u, 0u, 0u};
    } else if (w >= F1M::W2F && w < F1M::W2F + F1M::T2) {
      frag_rows<F1M::K2, F1, F2, F1>(f2w, P.shadow + O.off[6], w - F1M::W2F);
    }
    // next-step staging (wave 15, two steps deep so that no load waits on another inside this
    // kernel): metaN[b] = (step, position, perm entry) looked up by the PREVIOUS step for step + 1;
    // when it matches, the raw image of step + 1 is gathered now (stored to stage2 at the end of
    // this role). The perm entry for step + 2 is looked up here and published to metaN. A mismatch
    // (epoch start, new permutation, ...) stages nothing: the next step then gathers its images
    // itself. All vector loads, waited for after the fc chain.
    int64_t pos1 = 0, pos2 = 0, idx1 = 0;
    bool st1 = false;
    int nperm2v = 0;
    long long ntgtv = 0;
    uint4 nraw0 = make_uint4(0u, 0u, 0u, 0u), nraw1 = nraw0, nraw2 = nraw0;
    if (stage_on) {
      pos1 = (sie + 1) * A.batch_stride + b;
      if (pos1 >= A.perm_len) pos1 %= A.perm_len;
      pos2 = (sie + 2) * A.batch_stride + b;
      if (pos2 >= A.perm_len) pos2 %= A.perm_len;
      nperm2v = A.perm[pos2];
      auto rfl64 = [](long long v) {
        return (int64_t)(((uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((int)((uint64_t)v >> 32)) << 32) |
                         (unsigned)__builtin_amdgcn_readfirstlane((int)v));
      };
      const int64_t sN = rfl64(mN01.x), pN = rfl64(mN01.y), iN = rfl64(mN2);
      st1 = sN == step + 1 && pN == pos1 && iN >= 0 && iN < A.n;
      if (st1) {
        idx1 = iN;
        const uint4* src = reinterpret_cast<const uint4*>(A.data + idx1 * 3072);
        nraw0 = src[lane];
        nraw1 = src[lane + 64];
        nraw2 = src[lane + 128];
        ntgtv = P.dtargets[idx1];
      }
    }
    // P3: conv2 (MFMA) + bias + ReLU + maxpool -> f (flatten order oc*25 + cell), i2 (waves 8-14)
    if (w < 15) {
      const int wt = w - 8;
      const int r = 16 * wt + m, cell = min(r >> 2, 24), q = r & 3;
      const int py = cell / 5, pxx = cell - 5 * py, y = 2 * py + (q >> 1), x = 2 * pxx + (q & 1);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 7; ++s) {
        const int tap = 4 * s + g, kh = tap / 5, kw = tap - 5 * kh;
        u32x4 a = *reinterpret_cast<const u32x4*>(L.v.f.p1h + ((tap < 25 ? (y + kh) * P1HS + x + kw : 0)) * 8);
        if (tap >= 25) a = u32x4{0u, 0u, 0u, 0u};
        acc = mfma(a, *reinterpret_cast<const u32x4*>(L.v.f.w2f + (s * 64 + lane) * 8), acc);
      }
      const int cc = 4 * wt + g, oc = m;
      float pv;
      uint8_t code;
      pool4(acc, L.b2s[oc], pv, code);
      if (cc < 25 && oc < C2) {
        const int o = oc * 25 + cc;
        L.fb16[o] = f32_to_bf16(pv);
        L.f32[o] = pv;
        L.i2[o] = code;
      }
    }
    lbar();
    stamp(3);
    if (w >= F1M::W1F) {  // P4a: fc1 forward (the last T1 waves)
      const int r = 16 * (w - F1M::W1F) + m;
      const float v = row_dot(f1w, L.fb16);
      if (g == 0 && r < F1) {
        const float h = fmaxf(v + L.fb[r], 0.f);
        L.sh1[r] = h;
        L.h1b[r] = f32_to_bf16(h);
      }
    }
    lbar();
    stamp(18);
    // the fc1 forward fragments (W1 rows, 16 B per lane) -> the LDS fc1 image; clamped duplicates
    // (rows past F1, chunks past FLAT / 8) are skipped. In phases where the writing wave is idle:
    // P4c for all of them but the fc3 / CE wave, which writes in P5.
    auto put_f1img = [&]() {
      const int row = 16 * (w - F1M::W1F) + m;
      if (row < F1) {
        uint16_t* dst = L.u.f1img + (row * S::F1S + (row & 1)) * 8;
#pragma unroll
        for (int q = 0; q < F1M::K1; ++q)
          if (4 * q + g < FLAT / 8) *reinterpret_cast<u32x4*>(dst + (4 * q + g) * 8) = f1w[q];
      }
    };
    if (w == F1M::W3F) frag_rows<F1M::K3, P3F, NC, F2>(f3w, pwimg + kFc3F, 0);
    if (w >= F1M::W2F && w < F1M::W2F + F1M::T2) {  // P4b: fc2 forward
      const int r = 16 * (w - F1M::W2F) + m;
      const float v = row_dot(f2w, L.h1b);
      if (g == 0 && r < F2) {
        const float h = fmaxf(v + L.fb[F1 + r], 0.f);
        L.sh2[r] = h;
        L.h2b[r] = f32_to_bf16(h);
      }
    }
    lbar();
    stamp(19);
    if (w == F1M::W3F) {  // P4c: fc3 forward + softmax-CE in one wave (the logits are in lanes 0 .. NC-1)
      const float v = row_dot(f3w, L.h2b);
      constexpr int GC = pow2_ge(NC);
      const float z = lane < NC ? v + L.fb[F1 + F2 + lane] : -INFINITY;
      const float mx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(group_reduce_last<GC, true>(z)), GC - 1));
      const float e = lane < NC ? expf(z - mx) : 0.f;
      const float s = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(group_reduce_last<GC>(e)), GC - 1));
      const float lse = mx + logf(s);
      const bool valid = tgt >= 0 && tgt < NC;
      const unsigned long long am_mask = __ballot(lane < NC && z == mx);
      const int am = __ffsll((long long)am_mask) - 1;
      const float zt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(z), valid ? (int)tgt : 0));
      const float loss = valid ? lse - zt : 0.f;
      if (lane < NC) {
        const float dl = valid ? (e / s - (lane == tgt ? 1.f : 0.f)) * inv_B : 0.f;
        L.slog[lane] = z;
        L.sdl[lane] = dl;
        L.dlb[lane] = f32_to_bf16(dl);
      }
      if (lane == 0) {
        L.ce[0] = (double)loss * (double)inv_B;
        L.ce[1] = (am == tgt) ? (double)inv_B : 0.0;
      }
    } else if (w >= F1M::W1F) {
      put_f1img();
    }
    if (w >= F1M::W2F && w < F1M::W2F + F1M::T2) {  // the fc2 forward fragments -> the fc2 image
      const int row = 16 * (w - F1M::W2F) + m;
      if (row < F2) {
#pragma unroll
        for (int q = 0; q < F1M::K2; ++q) {
          const int c = 4 * q + g;
          if (c < F1 / 8)
            *reinterpret_cast<u32x4*>(L.v.f2img + (row * S::F2S + (c ^ (((row & 3) << 2) | ((row >> 2) & 3)))) * 8) = f2w[q];
        }
      }
    }
    lbar();
    stamp(4);
    if (w == F1M::W3F) put_f1img();
    lbar();  // P5 (fc3 dgrad)
    stamp(20);
    if (stage_on) {  // wave 15: publish the next step's raw image + tags
      if (st1) {
        uint4* dst = reinterpret_cast<uint4*>(pstage2 + (int64_t)b * 3072);
        dst[lane] = nraw0;
        dst[lane + 64] = nraw1;
        dst[lane + 128] = nraw2;
      }
      if (lane == 0) {
        if (st1) {
          pmeta2[4 * b] = step + 1;
          pmeta2[4 * b + 1] = pos1;
          pmeta2[4 * b + 2] = idx1;
          pmeta2[4 * b + 3] = ntgtv;
        }
        pmetaN[4 * b] = step + 2;
        pmetaN[4 * b + 1] = pos2;
        pmetaN[4 * b + 2] = nperm2v;
      }
    }
    lbar();  // P6 (fc2 dgrad)
    stamp(21);
  }

  // ---- P8: fc1 dgrad on every wave (tiles w, w + 16) from the LDS fc1 image, read transposed ----
  stamp(22);
  {
    u32x4 ah[F1M::B1K];  // the fc1 output gradient (bf16, zero past F1), broadcast over the A rows
#pragma unroll
    for (int q = 0; q < F1M::B1K; ++q) ah[q] = *reinterpret_cast<const u32x4*>(L.dh1b + 32 * q + 8 * g);
#pragma unroll
    for (int j = 0; j < (F1M::B1T + 15) / 16; ++j) {
      const int tile = w + 16 * j;
      if (tile < F1M::B1T) {  // wave-uniform: every lane runs the transposed reads
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < F1M::B1K; ++q) acc = mfma(ah[q], f1t_frag<F1, FLAT, S::F1S>(L.u.f1img, tile, q), acc);
        const int c = 16 * tile + m;
        if (g == 0 && c < FLAT) L.df[c] = acc[0];
      }
    }
  }
  lbar();
  stamp(5);

  // ---- P10: the backward images (the fc1 image is dead): conv2 dgrad fragments; unpool2 -> the
  //           conv2-output gradient images, all four cells of a pool window written (the value at
  //           the arg max, 0 elsewhere; channels past C2 zero); the zero border of the padded image,
  //           the unread pad columns and the whole conv1-gradient image d1 (written sparsely in P11)
  //           zeroed -- every store to a distinct address, so no barrier inside the phase
  if (t < WID) reinterpret_cast<uint4*>(L.u.b.w2d)[t] = wid;
  if (t < 16 * 25) {
    const int oc = t / 25, cell = t - 25 * oc, py = cell / 5, pxx = cell - 5 * py;
    const int code = oc < C2 ? (int)L.i2[t] : 4;
    const uint16_t v = code < 4 ? f32_to_bf16(L.df[t]) : (uint16_t)0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int Y = 2 * py + (k >> 1), X = 2 * pxx + (k & 1);
      const uint16_t o = k == code ? v : (uint16_t)0;
      L.u.b.dch[((Y + 4) * DCHS + X + 4) * 16 + oc] = o;
      L.u.b.dcc[(oc * 10 + Y) * DCCS + X] = o;
    }
  } else {
    // border of dch: the 18 x DCHS pixels outside [4, 14) x [4, 14), 16 channels = 2 uint4 each
    constexpr int NPIX = 18 * DCHS;
    for (int e = t - 16 * 25; e < 2 * NPIX; e += kT - 16 * 25) {
      const int pix = e >> 1, Y = pix / DCHS, X = pix - DCHS * Y;
      if (Y < 4 || Y >= 14 || X < 4 || X >= 14)
        reinterpret_cast<uint4*>(L.u.b.dch)[2 * pix + (e & 1)] = make_uint4(0u, 0u, 0u, 0u);
    }
  }
  {
    // dcc columns 10 .. DCCS - 1 of its 160 rows (read up to column 15 by the conv2 wgrad)
    static_assert(DCCS == 24, "dcc pad layout");
    for (int e = t; e < 160 * 7; e += kT) {  // 7 u32 = columns 10 .. 23
      const int r = e / 7, k = e - 7 * r;
      reinterpret_cast<unsigned*>(L.u.b.dcc + r * DCCS + 10)[k] = 0u;
    }
    constexpr int D1Q = D::C1 * D1S * 2 / 16;
    static_assert((D::C1 * D1S * 2) % 16 == 0, "d1 zero fill");
    for (int e = t; e < D1Q; e += kT) reinterpret_cast<uint4*>(L.u.b.d1)[e] = make_uint4(0u, 0u, 0u, 0u);
  }
  lbar();
  stamp(6);

  // ---- P11: conv2 dgrad (waves 0-6) -> liveness mask -> unpooled conv1 grad d1 -----------------
  //           conv2 wgrad of the sample (waves 7-15) -> slab
  // dgrad: M = 98 (y, x pair) positions (column-major: conflict-free A reads at DCHS = 19), N =
  // (in channel, x parity), K = (kh, u, oc16) with kw = u - 1 + dx: 7 tiles x 15 k-steps
  float* slab = P.slab1 + (int64_t)b * D::SLABN;
  if (w < 7) {
    const int pidx = min(16 * w + m, 97), Y = pidx % 14, xp = pidx / 14;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 15; ++s) {
      const int pp = 2 * s + (g >> 1), oc0 = 8 * (g & 1), kh = pp / 6, u = pp - 6 * kh;
      u32x4 a = *reinterpret_cast<const u32x4*>(L.u.b.dch + ((pp < 30 ? (Y - kh + 4) * DCHS + 2 * xp + 5 - u : 0)) * 16 + oc0);
      if (pp >= 30) a = u32x4{0u, 0u, 0u, 0u};
      acc = mfma(a, *reinterpret_cast<const u32x4*>(L.u.b.w2d + (s * 64 + lane) * 8), acc);
    }
    const int ic = m >> 1, dx = m & 1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int pr = 16 * w + 4 * g + r;
      if (pr < 98 && ic < C1) {
        const int pc = (pr % 14) * 14 + 2 * (pr / 14) + dx;
        const int code = L.i1[ic * 196 + pc];
        if (code < 4) {
          const int py = pc / 14, pxx = pc - 14 * py;
          L.u.b.d1[ic * D1S + (2 * py + (code >> 1)) * 32 + 2 * pxx + (code & 1)] = f32_to_bf16(acc[r]);
        }
      }
    }
  } else {
    // 10 M-tiles over waves 7-15 (wave 7: two): tile tt = (kw, half); rows (ic, kh) = 16 * half + m;
    // row 31 of tile 1 = ones (bias). Wave 15's staging stores were issued in P10.
    const int t0 = w - 7, t1 = w == 7 ? 2 : w - 6;
    for (int tt0 = t0; tt0 < t1; ++tt0) {
      const int tt = w == 7 && tt0 == 1 ? 9 : tt0;
      // the window shift kw is wave-uniform: one dispatch per tile, then a branch-free unrolled
      // K loop with the shift as a compile-time constant (a switch inside the loop cost a branch
      // and an lgkmcnt(0) wait per step)
      auto tile = [&](auto KWc) __attribute__((always_inline)) {
        constexpr int kw = decltype(KWc)::value;
        const int h = tt & 1, i = 16 * h + m, ic = i / 5, kh = i - 5 * ic;
        const bool valid = ic < C1, ones = tt == 1 && m == 15;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 5; ++s) {
          const int y = 2 * s + (g >> 1), x0 = 8 * (g & 1);
          const u32x4 bq = *reinterpret_cast<const u32x4*>(L.u.b.dcc + (m * 10 + y) * DCCS + x0);
          const uint16_t* rowp = L.p1c + ((valid ? ic : 0) * 14 + y + (valid ? kh : 0)) * P1CS + x0;
          const u32x4 lo = *reinterpret_cast<const u32x4*>(rowp), hi = *reinterpret_cast<const u32x4*>(rowp + 8);
          u32x4 a = fshift<kw>(lo, hi);
          if (!valid) a = ones ? u32x4{0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u} : u32x4{0u, 0u, 0u, 0u};
          acc = mfma(a, bq, acc);
        }
        const int oc = m;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ir = 16 * h + 4 * g + r, icr = ir / 5, khr = ir - 5 * icr;
          if (oc < C2 && icr < C1) slab[D::S2OFF + (oc * C1 + icr) * 25 + khr * 5 + kw] = acc[r];
          if (oc < C2 && tt == 1 && ir == 31) slab[D::S2OFF + C2 * C1 * 25 + oc] = acc[r];
        }
      };
      switch (tt >> 1) {
        case 0: tile(std::integral_constant<int, 0>{}); break;
        case 1: tile(std::integral_constant<int, 1>{}); break;
        case 2: tile(std::integral_constant<int, 2>{}); break;
        case 3: tile(std::integral_constant<int, 3>{}); break;
        default: tile(std::integral_constant<int, 4>{}); break;
      }
    }
  }
  lbar();
  stamp(7);

  // ---- P13: conv1 wgrad (waves 0-6: 4 output rows Y each, all 5 kw tiles) ---------------------
  // One read of the input rows (lo / hi) and of the gradient row feeds the five kw-shifted
  // windows' MFMAs: 84 operand reads in all (450 with one tile per wave); the 7 row-range partials
  // are summed in a fixed order.
  if (w < kP13W) {
    const int c = m / 5, kh = m - 5 * c;
    const bool valid = m < 15;
    const int x0 = 8 * g;
    const uint16_t* xrow = L.xc + ((valid ? c : 0) * 32 + (valid ? kh : 0)) * XCS + x0;
    const uint16_t* drow = L.u.b.d1 + min(m, C1 - 1) * D1S + x0;
    constexpr u32x4 ONES = {0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u};  // bias row (m = 15, kw = 0)
    const u32x4 Z = {0u, 0u, 0u, 0u};
    f32x4 acc[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int yy = 0; yy < 28 / kP13W; ++yy) {
      const int Y = (28 / kP13W) * w + yy;
      u32x4 bq = *reinterpret_cast<const u32x4*>(drow + Y * 32);
      if (m >= C1) bq = Z;
      const u32x4 lo = *reinterpret_cast<const u32x4*>(xrow + Y * XCS), hi = *reinterpret_cast<const u32x4*>(xrow + Y * XCS + 8);
      acc[0] = mfma(valid ? fshift<0>(lo, hi) : (m == 15 ? ONES : Z), bq, acc[0]);
      acc[1] = mfma(valid ? fshift<1>(lo, hi) : Z, bq, acc[1]);
      acc[2] = mfma(valid ? fshift<2>(lo, hi) : Z, bq, acc[2]);
      acc[3] = mfma(valid ? fshift<3>(lo, hi) : Z, bq, acc[3]);
      acc[4] = mfma(valid ? fshift<4>(lo, hi) : Z, bq, acc[4]);
    }
#pragma unroll
    for (int kw = 0; kw < 5; ++kw)
#pragma unroll
      for (int r = 0; r < 4; ++r) L.u.b.scr[((w * 5 + kw) * 16 + 4 * g + r) * 16 + m] = acc[kw][r];
  }
  lbar();
  stamp(23);
  for (int e = t; e < 5 * 256; e += kT) {
    const int kw = e >> 8, i = (e >> 4) & 15, oc = e & 15;
    float v = L.u.b.scr[e];
#pragma unroll
    for (int p = 1; p < kP13W; ++p) v += L.u.b.scr[p * 1280 + e];
    if (oc < C1) {
      if (i < 15) slab[oc * 76 + (i / 5) * 25 + (i % 5) * 5 + kw] = v;
      else if (kw == 0) slab[oc * 76 + 75] = v;
    }
  }
  stamp(24);
  static_assert(F1 <= 128 && F2 <= 128 && NC <= 64, "end-of-kernel store mapping");
  // activations / gradients for the batch reductions of KW (and inspection), all stored here: no
  // load of this kernel is waited for after this point
  for (int e = t; e < FLAT; e += kT) {
    P.p2[(int64_t)b * FLAT + e] = L.f32[e];
    P.dflat[(int64_t)b * FLAT + e] = L.df[e];
  }
  if (t < F1) {
    P.h1[(int64_t)b * F1 + t] = L.sh1[t];
    P.dh1[(int64_t)b * F1 + t] = L.sdh1[t];
  } else if (t >= 128 && t < 128 + F2) {
    P.h2[(int64_t)b * F2 + t - 128] = L.sh2[t - 128];
    P.dh2[(int64_t)b * F2 + t - 128] = L.sdh2[t - 128];
  } else if (t >= 256 && t < 256 + NC) {
    P.logits[(int64_t)b * NC + t - 256] = L.slog[t - 256];
    P.dlogits[(int64_t)b * NC + t - 256] = L.sdl[t - 256];
  } else if (t == 320 && P.cestat) {
    P.cestat[2 * b] = L.ce[0];
    P.cestat[2 * b + 1] = L.ce[1];
  }
  if (aug && t == 0 && P.targets) P.targets[b] = tgt;  // (inspection; nothing downstream reads it)
  // the step's optimizer context for KW (lr from the device table, Adam's t)
  if (b == 0 && t == 0 && P.stepinfo) {
    float lr = O.h.lr;
    if (O.lr_ptr) lr = O.lr_ptr[O.lr_table ? sie : 0];
    P.stepinfo[0] = step;
    P.stepinfo[1] = sie;
    P.stepinfo[2] = (int64_t)__float_as_uint(lr);
  }
  stamp(13);
  if ((mode & LENET_TRACE) && b == 0 && t < 32 && P.trace) reinterpret_cast<unsigned long long*>(P.trace)[t] = L.tr[t];
  if ((mode & LENET_TRACE) && P.trace && b < 200) {  // per-block wall clock: slots 600 + 2 b (+1)
    lbar();
    if (t == 0) {
      reinterpret_cast<unsigned long long*>(P.trace)[600 + 2 * b] = tb0;
      reinterpret_cast<unsigned long long*>(P.trace)[601 + 2 * b] = __builtin_amdgcn_s_memrealtime();
    }
  }
}

// ---------------------------------------------------------------------------
// KW: batch reductions + optimizer
// ---------------------------------------------------------------------------
struct Ctx {
  bool on;
  float lr, t;
};

template <int K>
__device__ __forceinline__ void upd1(const LeNetOpt& O, const Ctx& c, uint16_t* shadow, int64_t i, float g, float p,
                                     float a, float s) {
  O.g[i] = g;
  if (!c.on) return;
  opt_update_k<K>(O.h, c.lr, c.t, p, g, a, s);
  O.p[i] = p;
  if (O.s1) O.s1[i] = a;
  if (O.s2) O.s2[i] = s;
  if (shadow) shadow[i] = f32_to_bf16(p);
}

// Data-parallel exchange inside the batch-reduction kernel (struct XgmiFused, WT ranks; WT = 0: off).
// Every gradient element is produced by exactly one lane of one block, the same lane and block on
// every rank. The lane publishes each of its elements as one 8-byte granule {fp32 value, tag = low
// 32 bits of the block's launch counter} into its rank's granule array (parity p of this launch) with
// a single system-scope store (global_store sc0 sc1: written through, single-copy atomic -- value and
// tag arrive together), then polls the WT - 1 peers' granules of the same elements with system-scope
// loads until every tag matches, and sums in rank order (its own value from registers; the same
// order on every rank: bit-identical replicas) before the update. No flags, no fences, no barriers:
// the data is its own flag, so the exchange costs one store and one (remote) load round trip per
// lane instead of store -> drain -> barrier -> flag -> poll -> barrier -> load. Parity reuse is safe
// as in allreduce.hip: a rank reaches launch s + 2 (parity p again) only after it read every peer's
// launch s + 1 granules, which a peer writes only after its launch s -- including its reads of parity
// p -- retired. W = 1 (loopback) polls its own granules back, so the loopback pays the round trip a
// peer would.
// Failure: the sticky error word (device copy, read once per wave at launch start) stops this rank
// from publishing anything once any launch timed out, so every peer times out too; a lane whose
// poll timed out applies nothing (the job stops with TransportError; resume restores identical
// replicas from the checkpoint).
template <int WT>
struct Xch {
  static constexpr bool on = WT > 0;
  // (plain copies: a dynamically indexed kernel-argument array would be spilled to scratch)
  uint64_t* gr[WT > 0 ? WT : 1];  // this launch's parity half of every rank's granule array
  uint64_t* mine;
  unsigned* err;
  unsigned* derr;
  long long timeout;
  int rank;
  unsigned tag;
  bool dead;      // wave-uniform
  bool withhold;  // fault injection (tests)
  float scale;

  __device__ __forceinline__ void st(int64_t i, float v) const {
    const uint64_t g = (uint64_t)__float_as_uint(v) | ((uint64_t)tag << 32);
    __hip_atomic_store(mine + i, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __device__ __forceinline__ uint64_t ld(int q, int64_t i) const {
    return __hip_atomic_load(gr[q] + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __device__ __forceinline__ void put1(int64_t i, float v) const {
    if (!dead && !withhold) st(i, v);
  }
  __device__ __forceinline__ void put4(int64_t i, float4 v) const {
    if (!dead && !withhold) {
      st(i, v.x);
      st(i + 1, v.y);
      st(i + 2, v.z);
      st(i + 3, v.w);
    }
  }
  static constexpr bool peer(int q, int rank) { return WT == 1 || q != rank; }
  // N consecutive elements at i: every peer's granules, polled until all tags match (false: timed
  // out -- the error words are set), summed in rank order with own[] in this rank's position, scaled;
  // opaque to the compiler so that the optimizer's arithmetic cannot contract with the sum (bitwise
  // equal to all-reduce -> separate update launch)
  template <int N>
  __device__ __forceinline__ bool get(int64_t i, const float* own, float* out) const {
    if (dead) return false;
    uint64_t g[WT][N];
#pragma unroll
    for (int q = 0; q < WT; ++q)
#pragma unroll
      for (int e = 0; e < N; ++e) g[q][e] = peer(q, rank) ? ld(q, i + e) : (uint64_t)tag << 32;
    long long t0 = -1;
    for (;;) {
      bool ready = true;
#pragma unroll
      for (int q = 0; q < WT; ++q)
#pragma unroll
        for (int e = 0; e < N; ++e) ready &= (unsigned)(g[q][e] >> 32) == tag;
      if (ready) break;
      const long long now = wall_clock64();  // 100 MHz constant clock
      if (t0 < 0) {
        t0 = now;
      } else if (now - t0 > timeout) {
        __hip_atomic_fetch_or(derr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return false;
      }
      __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int q = 0; q < WT; ++q)
#pragma unroll
        for (int e = 0; e < N; ++e)
          if (peer(q, rank) && (unsigned)(g[q][e] >> 32) != tag) g[q][e] = ld(q, i + e);
    }
#pragma unroll
    for (int e = 0; e < N; ++e) {
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < WT; ++q) {
        const float v = peer(q, rank) ? __uint_as_float((unsigned)g[q][e]) : own[e];
        s = q == 0 ? v : s + v;
      }
      s *= scale;
      asm volatile("" : "+v"(s));
      out[e] = s;
    }
    return true;
  }
};

template <class D>
__host__ __device__ constexpr int mw_conv_blocks() {
  return (D::S1 + D::S2 + kWgT - 1) / kWgT;
}
// fc weight gradients + update on the matrix cores, exact f32: v_mfma_f32_16x16x4_f32 is a
// k-ordered fma chain, so 8 of them over a 32-sample chunk sum the batch in sample order, exactly as
// a sequential loop would. A wave owns a 16 (inputs c; c == NIN is the bias, fed by a ones column)
// x 16 (outputs j) tile of dW^T: C[c][j] = sum_b X[b][c] dY[b][j]; its lane then holds 4 consecutive
// inputs of one output row -- one float4 of each optimizer buffer.
template <int NIN, int NOUT>
struct FcW {
  static constexpr int CT = (NIN + 1 + 15) / 16, JT = (NOUT + 15) / 16, TILES = CT * JT;
  static_assert(NIN % 4 == 0, "bias row alignment");
};
template <class D>
__host__ __device__ constexpr int mw_fc_waves() {
  return FcW<D::FLAT, D::F1>::TILES + FcW<D::F1, D::F2>::TILES + FcW<D::F2, D::NC>::TILES;
}
template <class D>
__host__ __device__ constexpr int mw_fc_blocks() {
  return (mw_fc_waves<D>() + kWgT / 64 - 1) / (kWgT / 64);
}

template <int NIN, int NOUT, int WT, int K>
__device__ __forceinline__ void fc_wgrad(const Xch<WT>& xc, int tile, int B, const float* __restrict__ dY,
                                         const float* __restrict__ X, const LeNetOpt& O, const Ctx& c, uint16_t* shadow,
                                         int64_t offW, int64_t offb, uint16_t* __restrict__ timg, int tpitch,
                                         uint16_t* __restrict__ fimg = nullptr, int fpitch = 0) {
  using W = FcW<NIN, NOUT>;
  const int ct = tile % W::CT, jt = tile / W::CT;
  const int lane = threadIdx.x & 63, g = lane >> 4, n = lane & 15;
  const int ca = 16 * ct + n, jb = 16 * jt + n;   // this lane's A row (input) / B column (output)
  const int c0 = 16 * ct + 4 * g, j = 16 * jt + n;  // its C rows c0 .. c0 + 3, column j
  const bool jok = j < NOUT, wrow = jok && c0 < NIN, brow = jok && c0 == NIN;
  const int64_t iw = offW + (int64_t)j * NIN + c0, ib = offb + j;
  float4 pw = make_float4(0.f, 0.f, 0.f, 0.f), aw = pw, sw = pw;
  float pb = 0.f, ab = 0.f, sb = 0.f;
  if (c.on && wrow) {  // optimizer state in flight together with the batch loads
    pw = *reinterpret_cast<const float4*>(O.p + iw);
    if (O.s1) aw = *reinterpret_cast<const float4*>(O.s1 + iw);
    if (O.s2) sw = *reinterpret_cast<const float4*>(O.s2 + iw);
  }
  if (c.on && brow) {
    pb = O.p[ib];
    if (O.s1) ab = O.s1[ib];
    if (O.s2) sb = O.s2[ib];
  }
  const int cl = min(ca, NIN - 1), jl = min(jb, NOUT - 1);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int b0 = 0; b0 < B; b0 += 32) {
    float a[8], d[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {  // MFMA u, k = g: sample b0 + 4u + g
      const int bb = min(b0 + 4 * u + g, B - 1);
      a[u] = X[(int64_t)bb * NIN + cl];
      d[u] = dY[(int64_t)bb * NOUT + jl];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool ok = b0 + 4 * u + g < B;
      const float av = ok ? (ca < NIN ? a[u] : (ca == NIN ? 1.f : 0.f)) : 0.f;
      const float dv = ok && jb < NOUT ? d[u] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, dv, acc, 0, 0, 0);
    }
  }
  float4 gv = make_float4(acc[0], acc[1], acc[2], acc[3]);
  float gb = acc[0];
  if constexpr (Xch<WT>::on) {  // data-parallel: this lane's elements summed over the ranks
    if (wrow) {
      xc.put4(iw, gv);
      float o[4] = {gv.x, gv.y, gv.z, gv.w}, r[4];
      if (!xc.template get<4>(iw, o, r)) return;
      gv = make_float4(r[0], r[1], r[2], r[3]);
    }
    if (brow) {
      xc.put1(ib, gb);
      float r;
      if (!xc.template get<1>(ib, &gb, &r)) return;
      gb = r;
    }
  }
  if (wrow) {
    *reinterpret_cast<float4*>(O.g + iw) = gv;
    if (c.on) {
      opt_update_k<K>(O.h, c.lr, c.t, pw.x, gv.x, aw.x, sw.x);
      opt_update_k<K>(O.h, c.lr, c.t, pw.y, gv.y, aw.y, sw.y);
      opt_update_k<K>(O.h, c.lr, c.t, pw.z, gv.z, aw.z, sw.z);
      opt_update_k<K>(O.h, c.lr, c.t, pw.w, gv.w, aw.w, sw.w);
      *reinterpret_cast<float4*>(O.p + iw) = pw;
      if (O.s1) *reinterpret_cast<float4*>(O.s1 + iw) = aw;
      if (O.s2) *reinterpret_cast<float4*>(O.s2 + iw) = sw;
      const uint16_t h0 = f32_to_bf16(pw.x), h1 = f32_to_bf16(pw.y), h2 = f32_to_bf16(pw.z), h3 = f32_to_bf16(pw.w);
      if (shadow) *reinterpret_cast<uint2*>(shadow + iw) = make_uint2(pack2(h0, h1), pack2(h2, h3));
      if (timg) {  // transposed bf16 image [in][out] (the per-sample kernel's dgrad operand)
        timg[(c0 + 0) * tpitch + j] = h0;
        timg[(c0 + 1) * tpitch + j] = h1;
        timg[(c0 + 2) * tpitch + j] = h2;
        timg[(c0 + 3) * tpitch + j] = h3;
      }
      if (fimg)  // row-padded copy [out][round8(in)] (16-byte fragment rows)
        *reinterpret_cast<uint2*>(fimg + j * fpitch + c0) = make_uint2(pack2(h0, h1), pack2(h2, h3));
    }
  }
  if (brow) upd1<K>(O, c, shadow, ib, gb, pb, ab, sb);
}

template <class D, int WT, int K>
__device__ __forceinline__ void mw_body(int mode, const LeNetPtrs& P, const LeNetOpt& O, int B, int64_t* __restrict__ ctrl,
                                        const Xch<WT>& xc) {
  constexpr int C1 = D::C1, C2 = D::C2, F1 = D::F1, F2 = D::F2, NC = D::NC, FLAT = D::FLAT;
  constexpr int NBC = mw_conv_blocks<D>();
  constexpr int NB = mw_fc_blocks<D>(), NW3 = FcW<FLAT, F1>::TILES, NW4 = FcW<F1, F2>::TILES,
                NW5 = FcW<F2, NC>::TILES;
  const int t = threadIdx.x;
  int blk = blockIdx.x;
  // the step's counters / lr as the per-sample kernel saw them (nothing here reads ctrl, which
  // block NBC + fc blocks advances)
  const int64_t step = P.stepinfo[0], sie = P.stepinfo[1];
  Ctx c;
  c.on = (mode & LENET_OPT) != 0;
  c.t = (float)(step + 1);
  c.lr = __uint_as_float((unsigned)P.stepinfo[2]);
  uint16_t* shadow = P.shadow;
  if (blk < NBC) {
    const int e = blk * kWgT + t;
    const bool act = e < D::S1 + D::S2;
    if (!act) return;
    int soff = 0;
    int64_t dst = 0;
    if (!act) {
    } else if (e < D::S1) {
      const int oc = e / 76, tap = e - 76 * oc;
      soff = e;
      dst = tap < 75 ? O.off[0] + oc * 75 + tap : O.off[1] + oc;
    } else {
      const int e2 = e - D::S1;
      soff = D::S2OFF + e2;
      dst = e2 < C2 * C1 * 25 ? O.off[2] + e2 : O.off[3] + (e2 - C2 * C1 * 25);
    }
    float p = 0.f, a = 0.f, s = 0.f;
    if (c.on) {
      p = O.p[dst];
      if (O.s1) a = O.s1[dst];
      if (O.s2) s = O.s2[dst];
    }
    float gsum = 0.f;  // all loads of a 32-sample chunk in flight, summed in sample order
    for (int b0 = 0; b0 < B; b0 += 32) {
      float v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) v[u] = P.slab1[(int64_t)min(b0 + u, B - 1) * D::SLABN + soff];
#pragma unroll
      for (int u = 0; u < 32; ++u) gsum += b0 + u < B ? v[u] : 0.f;
    }
    if constexpr (Xch<WT>::on) {  // data-parallel: summed over the ranks
      if (!act) return;
      xc.put1(dst, gsum);
      float r;
      if (!xc.template get<1>(dst, &gsum, &r)) return;
      gsum = r;
    }
    O.g[dst] = gsum;
    if (c.on) {
      opt_update_k<K>(O.h, c.lr, c.t, p, gsum, a, s);
      O.p[dst] = p;
      if (O.s1) O.s1[dst] = a;
      if (O.s2) O.s2[dst] = s;
      const uint16_t hb = f32_to_bf16(p);
      if (shadow) shadow[dst] = hb;
      if (P.wimg) {  // the per-sample kernel's fragment image of the conv weights
        if (e < D::S1) {
          const int oc = e / 76, tap = e - 76 * oc;
          if (tap < 75) {
            const int c = tap / 25, kh = (tap % 25) / 5, kw = tap % 5;
            P.wimg[w1f_slot(oc, c, kh, kw, 0)] = hb;
            P.wimg[w1f_slot(oc, c, kh, kw, 1)] = hb;
          }
        } else {
          const int e2 = e - D::S1;
          if (e2 < C2 * C1 * 25) {
            const int oc = e2 / (C1 * 25), ic = (e2 / 25) % C1, tap = e2 % 25;
            P.wimg[w2f_slot(oc, ic, tap)] = hb;
            P.wimg[w2d_slot(oc, ic, tap, 0)] = hb;
            P.wimg[w2d_slot(oc, ic, tap, 1)] = hb;
          }
        }
      }
    }
    return;
  }
  blk -= NBC;
  if (blk < NB) {  // one fc weight-gradient tile per wave
    int wv = blk * (kWgT / 64) + (t >> 6);
    wv = __builtin_amdgcn_readfirstlane(wv);
    if (wv < NW3) {
      // (no transposed fc1 image: the per-sample kernel transposes fc1 in LDS)
      fc_wgrad<FLAT, F1, WT, K>(xc, wv, B, P.dh1, P.p2, O, c, shadow, O.off[4], O.off[5], nullptr, F1);
    } else if ((wv -= NW3) < NW4) {
      fc_wgrad<F1, F2, WT, K>(xc, wv, B, P.dh2, P.h1, O, c, shadow, O.off[6], O.off[7], nullptr, Fc<D>::P2T);
    } else if ((wv -= NW4) < NW5) {
      fc_wgrad<F2, NC, WT, K>(xc, wv, B, P.dlogits, P.h2, O, c, shadow, O.off[8], O.off[9],
                       P.wimg ? P.wimg + kFc3T : nullptr, Fc<D>::P3T, P.wimg ? P.wimg + kFc3F : nullptr, Fc<D>::P3F);
    }
  } else {
    // loss / accuracy of the step in sample order (fixed tree): bitwise reproducible epoch stats.
    // One wave, the running totals fetched together with the per-sample values (one round trip).
    if (t >= 64) return;
    double st0 = 0.0, st1 = 0.0;
    if (t == 0) {
      st0 = P.stats[0];
      st1 = P.stats[1];
    }
    double s0 = 0.0, s1 = 0.0;
    for (int i = t; i < B; i += 64) {
      s0 += P.cestat[2 * i];
      s1 += P.cestat[2 * i + 1];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      s0 += __shfl_xor(s0, o, 64);
      s1 += __shfl_xor(s1, o, 64);
    }
    if (t == 0) {
      P.stats[0] = st0 + s0;
      P.stats[1] = st1 + s1;
      if (ctrl) {  // advance the device step counters (next step / lr index / Adam t)
        ctrl[0] = step + 1;
        ctrl[1] = sie + 1;
      }
    }
  }
}

// the optimizer kind, once per block (uniform): each kind's body is contiguous code, so a launch
// runs through one compact instruction footprint instead of all five kinds interleaved per update
template <class D, int WT>
__device__ __forceinline__ void mw_dispatch(int mode, const LeNetPtrs& P, const LeNetOpt& O, int B, int64_t* ctrl,
                                            const Xch<WT>& xc) {
  switch (O.h.kind) {
    case OPT_ADAM: mw_body<D, WT, OPT_ADAM>(mode, P, O, B, ctrl, xc); break;
    case OPT_ADAMW: mw_body<D, WT, OPT_ADAMW>(mode, P, O, B, ctrl, xc); break;
    case OPT_ADAGRAD: mw_body<D, WT, OPT_ADAGRAD>(mode, P, O, B, ctrl, xc); break;
    case OPT_ADAMAX: mw_body<D, WT, OPT_ADAMAX>(mode, P, O, B, ctrl, xc); break;
    default: mw_body<D, WT, OPT_SGD>(mode, P, O, B, ctrl, xc); break;
  }
}

// (the per-block first loads' pointers lead the arguments: preloaded into SGPRs, see lenet_ms)
__device__ __forceinline__ LeNetPtrs with_first(LeNetPtrs P, const float* slab1, const float* p2, const float* dh1,
                                                const float* h1, const float* dh2) {
  P.slab1 = const_cast<float*>(slab1);
  P.p2 = const_cast<float*>(p2);
  P.dh1 = const_cast<float*>(dh1);
  P.h1 = const_cast<float*>(h1);
  P.dh2 = const_cast<float*>(dh2);
  return P;
}
template <class D>
__global__ __launch_bounds__(kWgT) void lenet_mw(const float* __restrict__ pslab1, const float* __restrict__ pp2,
                                                 const float* __restrict__ pdh1, const float* __restrict__ ph1,
                                                 const float* __restrict__ pdh2, int mode, int B, LeNetPtrs P,
                                                 LeNetOpt O, int64_t* __restrict__ ctrl) {
  unsigned long long t0 = 0;
  if (mode & LENET_TRACE) t0 = __builtin_amdgcn_s_memrealtime();
  mw_dispatch<D, 0>(mode, with_first(P, pslab1, pp2, pdh1, ph1, pdh2), O, B, ctrl, Xch<0>{});
  // LENET_TRACE: 100 MHz wall clock per block (start) and per wave (end): P.trace slots 64 + 5 blk (+1 + wave)
  if ((mode & LENET_TRACE) && P.trace && blockIdx.x < 100) {
    unsigned long long* tr = reinterpret_cast<unsigned long long*>(P.trace) + 64 + 5 * blockIdx.x;
    if (threadIdx.x == 0) tr[0] = t0;
    if ((threadIdx.x & 63) == 0) tr[1 + (threadIdx.x >> 6)] = __builtin_amdgcn_s_memrealtime();
  }
}

// the data-parallel batch-reduction kernel: lenet_mw + the xGMI exchange of every block's slice
// (struct Xch) + the update, in one launch (WT = rank count; 1 = loopback)
template <class D, int WT>
__global__ __launch_bounds__(kWgT) void lenet_mwx(const float* __restrict__ pslab1, const float* __restrict__ pp2,
                                                  const float* __restrict__ pdh1, const float* __restrict__ ph1,
                                                  const float* __restrict__ pdh2, int mode, int B, LeNetPtrs P,
                                                  LeNetOpt O, int64_t* __restrict__ ctrl, XgmiFused X) {
  Xch<WT> xc;
  // per-block launch counter: identical on every block and rank; read again only by the next launch
  const uint64_t seq = X.seqs[blockIdx.x] + 1;
  if (threadIdx.x == 0) X.seqs[blockIdx.x] = seq;
  xc.tag = (unsigned)seq;
  const int64_t half = (int64_t)(seq & 1) * X.cap;
  xc.mine = X.gran[0] + half;
#pragma unroll
  for (int q = 0; q < WT; ++q) {
    xc.gr[q] = X.gran[q] + half;
    if (q == X.rank) xc.mine = xc.gr[q];
  }
  xc.err = X.err;
  xc.derr = X.derr;
  xc.timeout = X.timeout;
  xc.rank = X.rank;
  xc.withhold = X.fault == 1 && (int)(blockIdx.x % (2 * WT)) == X.rank;
  // the device copy of the sticky error word (a local read, not a PCIe round trip to the host-mapped
  // word), once per wave: in flight during the batch reduction
  xc.dead = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(X.derr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) != 0u;
  xc.scale = 1.f / (float)WT;
  mw_dispatch<D, WT>(mode, with_first(P, pslab1, pp2, pdh1, ph1, pdh2), O, B, ctrl, xc);
}

// bf16 shadow of the flat parameters + the conv fragment image, from the fp32 masters (start of
// every captured step sequence, and after each data-parallel optimizer launch)
template <class D>
__global__ __launch_bounds__(256) void lenet_mpack(const float* __restrict__ p, int64_t n, uint16_t* __restrict__ shadow,
                                                  uint16_t* __restrict__ wimg, int64_t off_w1, int64_t off_w2,
                                                  int64_t off_w3, int64_t off_w4, int64_t off_w5) {
  using F = Fc<D>;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) shadow[i] = f32_to_bf16(p[i]);
  if (i < kWimg) {
    const int64_t src = wimg_src<D::C1, D::C2>((int)i, off_w1, off_w2);
    wimg[i] = src >= 0 ? f32_to_bf16(p[src]) : (uint16_t)0;
  } else if (i < kFc2T) {  // fc1 transposed: [c][r] = W3[r][c]
    const int e = (int)(i - kFc1T), cc = e / D::F1, r = e - cc * D::F1;
    wimg[i] = cc < D::FLAT ? f32_to_bf16(p[off_w3 + (int64_t)r * D::FLAT + cc]) : (uint16_t)0;
  } else if (i < kFc3F) {  // fc2 transposed [F1][P2T]
    const int e = (int)(i - kFc2T), cc = e / F::P2T, r = e - cc * F::P2T;
    wimg[i] = cc < D::F1 && r < D::F2 ? f32_to_bf16(p[off_w4 + (int64_t)r * D::F1 + cc]) : (uint16_t)0;
  } else if (i < kFc3T) {  // fc3 row-padded [NC][P3F]
    const int e = (int)(i - kFc3F), r = e / F::P3F, cc = e - r * F::P3F;
    wimg[i] = r < D::NC && cc < D::F2 ? f32_to_bf16(p[off_w5 + (int64_t)r * D::F2 + cc]) : (uint16_t)0;
  } else if (i < kWimgTot) {  // fc3 transposed [F2][P3T]
    const int e = (int)(i - kFc3T), cc = e / F::P3T, r = e - cc * F::P3T;
    wimg[i] = cc < D::F2 && r < D::NC ? f32_to_bf16(p[off_w5 + (int64_t)r * D::F2 + cc]) : (uint16_t)0;
  }
}

// Data-parallel step, after the all-reduce of the flat gradient: the optimizer update of every
// element plus everything the per-sample kernel reads (bf16 shadow, conv fragment images, fc
// transposed / padded images) in ONE launch -- the fused single-rank step's update path for
// reduced gradients. `skip` (the transport's sticky error word) vetoes the whole update on this
// rank (all-or-nothing step).
template <class D>
__global__ __launch_bounds__(256) void lenet_mapply(LeNetPtrs P, LeNetOpt O, const unsigned* __restrict__ skip) {
  if (skip && __hip_atomic_load(skip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) return;
  using F = Fc<D>;
  constexpr int C1 = D::C1, F1 = D::F1, F2 = D::F2, FLAT = D::FLAT;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= O.n) return;
  const int64_t step = P.stepinfo[0];
  Ctx c;
  c.on = true;
  c.t = (float)(step + 1);
  c.lr = __uint_as_float((unsigned)P.stepinfo[2]);
  float p = O.p[e], a = O.s1 ? O.s1[e] : 0.f, s = O.s2 ? O.s2[e] : 0.f;
  const float g = O.g[e];
  opt_update(O.h, c.lr, c.t, p, g, a, s);
  O.p[e] = p;
  if (O.s1) O.s1[e] = a;
  if (O.s2) O.s2[e] = s;
  const uint16_t hb = f32_to_bf16(p);
  P.shadow[e] = hb;
  uint16_t* wi = P.wimg;
  if (e >= O.off[0] && e < O.off[0] + D::C1 * 75) {
    const int i = (int)(e - O.off[0]), oc = i / 75, tap = i - 75 * oc, ch = tap / 25, kh = (tap % 25) / 5, kw = tap % 5;
    wi[w1f_slot(oc, ch, kh, kw, 0)] = hb;
    wi[w1f_slot(oc, ch, kh, kw, 1)] = hb;
  } else if (e >= O.off[2] && e < O.off[2] + D::C2 * C1 * 25) {
    const int i = (int)(e - O.off[2]), oc = i / (C1 * 25), ic = (i / 25) % C1, tap = i % 25;
    wi[w2f_slot(oc, ic, tap)] = hb;
    wi[w2d_slot(oc, ic, tap, 0)] = hb;
    wi[w2d_slot(oc, ic, tap, 1)] = hb;
  } else if (e >= O.off[4] && e < O.off[4] + F1 * FLAT) {
    const int i = (int)(e - O.off[4]), r = i / FLAT, cc = i - r * FLAT;
    wi[kFc1T + cc * F1 + r] = hb;
  } else if (e >= O.off[6] && e < O.off[6] + F2 * F1) {
    const int i = (int)(e - O.off[6]), r = i / F1, cc = i - r * F1;
    wi[kFc2T + cc * F::P2T + r] = hb;
  } else if (e >= O.off[8] && e < O.off[8] + D::NC * F2) {
    const int i = (int)(e - O.off[8]), r = i / F2, cc = i - r * F2;
    wi[kFc3F + r * F::P3F + cc] = hb;
    wi[kFc3T + cc * F::P3T + r] = hb;
  }
}

template <class D>
void pack(const LeNetPtrs& P, const LeNetOpt& O, hipStream_t st) {
  const int64_t tot = O.n > kWimgTot ? O.n : kWimgTot;
  hipLaunchKernelGGL(lenet_mpack<D>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, O.p, O.n, P.shadow, P.wimg,
                     O.off[0], O.off[2], O.off[4], O.off[6], O.off[8]);
}

// MLT_LENET_PROBE: timing-probe mode bits OR-ed into the per-sample kernel's mode (profiling only)
static int probe_bits() {
  static const int v = [] {
    const char* e = std::getenv("MLT_LENET_PROBE");
    return e ? std::atoi(e) & (LENET_PROBE_NOF1T | LENET_PROBE_NOF1W | LENET_PROBE_NOF2) : 0;
  }();
  return v;
}

template <class D>
void run(int mode, int B, const LeNetPtrs& P, const LeNetAug& A, const LeNetOpt& O, hipStream_t st) {
  mode |= probe_bits();
  const float inv_B = 1.f / (float)B;
  hipLaunchKernelGGL(lenet_ms<D>, dim3(B), dim3(kT), 0, st, P.stage2, P.meta2, A.ctrl, P.wimg, P.metaN, mode, inv_B, P,
                     A, O);
  const int nblk = mw_conv_blocks<D>() + mw_fc_blocks<D>() + 1;
  hipLaunchKernelGGL(lenet_mw<D>, dim3(nblk), dim3(kWgT), 0, st, P.slab1, P.p2, P.dh1, P.h1, P.dh2, mode, B, P, O,
                     A.ctrl);
}

template <class D>
void run_dp(int mode, int B, const LeNetPtrs& P, const LeNetAug& A, const LeNetOpt& O, const XgmiFused& X,
            hipStream_t st) {
  const int nblk = mw_conv_blocks<D>() + mw_fc_blocks<D>() + 1;
  if (X.G < nblk) throw std::runtime_error("lenet dp step: transport block counters < reduction blocks");
  if (X.cap < O.n) throw std::runtime_error("lenet dp step: transport region smaller than the parameters");
  mode |= probe_bits();
  const float inv_B = 1.f / (float)B;
  hipLaunchKernelGGL(lenet_ms<D>, dim3(B), dim3(kT), 0, st, P.stage2, P.meta2, A.ctrl, P.wimg, P.metaN, mode, inv_B, P,
                     A, O);
  const int m = mode | LENET_OPT;
#define MLT_MWX(WV)                                                                                      \
  case WV:                                                                                               \
    hipLaunchKernelGGL((lenet_mwx<D, WV>), dim3(nblk), dim3(kWgT), 0, st, P.slab1, P.p2, P.dh1, P.h1, P.dh2, m, B, \
                       P, O, A.ctrl, X);                                                                          \
    break;
  switch (X.W) {
    MLT_MWX(1)
    MLT_MWX(2)
    MLT_MWX(3)
    MLT_MWX(4)
    MLT_MWX(5)
    MLT_MWX(6)
    MLT_MWX(7)
    MLT_MWX(8)
    default: throw std::runtime_error("lenet dp step: world size outside 1..8");
  }
#undef MLT_MWX
}

}  // namespace lm

void launch_lenet_mfma_dp(int cfg, int mode, int B, const LeNetPtrs& P, const LeNetAug& A, const LeNetOpt& O,
                          const XgmiFused& X, hipStream_t stream) {
  if (B <= 0) return;
  if (cfg == LENET_TINY)
    lm::run_dp<lm::DmTiny>(mode, B, P, A, O, X, stream);
  else
    lm::run_dp<lm::DmDefault>(mode, B, P, A, O, X, stream);
}

int lenet_mfma_slab_floats(int cfg) { return cfg == LENET_TINY ? lm::DmTiny::SLABN : lm::DmDefault::SLABN; }
int lenet_mfma_wimg_elems() { return lm::kWimgTot; }
int lenet_mfma_kw_blocks(int cfg) {
  return cfg == LENET_TINY ? lm::mw_conv_blocks<lm::DmTiny>() + lm::mw_fc_blocks<lm::DmTiny>() + 1
                           : lm::mw_conv_blocks<lm::DmDefault>() + lm::mw_fc_blocks<lm::DmDefault>() + 1;
}

void launch_lenet_mfma_apply(int cfg, const LeNetPtrs& P, const LeNetOpt& O, const unsigned* skip, hipStream_t stream) {
  if (O.n <= 0) return;
  const dim3 grid((unsigned)((O.n + 255) / 256));
  if (cfg == LENET_TINY)
    hipLaunchKernelGGL(lm::lenet_mapply<lm::DmTiny>, grid, dim3(256), 0, stream, P, O, skip);
  else
    hipLaunchKernelGGL(lm::lenet_mapply<lm::DmDefault>, grid, dim3(256), 0, stream, P, O, skip);
}

void launch_lenet_mfma_pack(int cfg, const LeNetPtrs& P, const LeNetOpt& O, hipStream_t stream) {
  if (cfg == LENET_TINY)
    lm::pack<lm::DmTiny>(P, O, stream);
  else
    lm::pack<lm::DmDefault>(P, O, stream);
}

void launch_lenet_mfma(int cfg, int mode, int B, const LeNetPtrs& P, const LeNetAug& A, const LeNetOpt& O,
                       hipStream_t stream) {
  if (B <= 0) return;
  if (cfg == LENET_TINY)
    lm::run<lm::DmTiny>(mode, B, P, A, O, stream);
  else
    lm::run<lm::DmDefault>(mode, B, P, A, O, stream);
}

}  // namespace mlt
