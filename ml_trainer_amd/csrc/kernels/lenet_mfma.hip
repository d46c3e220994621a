// LeNet-5 CIFAR training step (reference src/model.py:7-24, src/trainer.py:180-197) in bf16 on the
// CDNA4 matrix cores: TWO launches per step, whatever the batch.
//
//   KS  lenet_ms<D>  grid B x 1024 threads, one CU per sample, the whole per-sample chain in LDS:
//       [staged / augmented input] -> conv1 (MFMA) + bias + ReLU + maxpool -> conv2 (MFMA) + bias +
//       ReLU + maxpool -> fc1 / fc2 / fc3 (+ReLU) -> softmax-CE -> fc dgrad chain -> unpool2 ->
//       conv2 dgrad (MFMA) -> pool1 liveness mask -> conv2 wgrad (MFMA) and conv1 wgrad (MFMA) of
//       the sample -> per-sample weight-gradient slab; + the NEXT step's raw input image gathered
//       (epoch permutation -> dataset row) and staged by an otherwise idle wave, so the next step
//       starts with one round trip instead of ctrl -> perm -> image.
//   KW  lenet_mw<D>  role-split grid: conv slab sums over the batch (sample order), fc weight
//       gradients over the batch, the fused optimizer update (fp32 masters + bf16 shadow), the
//       fixed-order loss / accuracy sums, the step-counter advance.
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
// followed by fc1's weight TRANSPOSED ([in][out] bf16, the backward-data B operand: 16 contiguous
// bytes per lane), sized for the largest config
constexpr int kFc1T = kWimg, kWimgTot = kWimg + 400 * 120;
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

// ---------------------------------------------------------------------------
// fc layer with bf16 weights held in registers (4 columns = 8 bytes per slot) for the whole
// kernel: forward row dots (G lanes per row, DPP tree) and backward-data (each lane scales its
// weight fragment by the upstream gradient; row groups summed through LDS in a fixed order).
// ---------------------------------------------------------------------------
constexpr int pow2_ge(int v) { return v <= 1 ? 1 : v <= 2 ? 2 : v <= 4 ? 4 : v <= 8 ? 8 : v <= 16 ? 16 : v <= 32 ? 32 : 64; }

// (opaque to the optimiser: the packed weights stay the register-resident form -- CSE of the
// forward's unpacked values into the backward would double their registers)
__device__ __forceinline__ float4 unpack4(uint2 u) {
  asm volatile("" : "+v"(u.x), "+v"(u.y));
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xffff0000u));
}

template <int NCOLS, int NROWS, int NT>
struct BLinear {
  static constexpr int NV = NCOLS / 4;
  static constexpr int G = pow2_ge(NV);
  static constexpr int PL = (NV + G - 1) / G;
  static constexpr int R = 64 / G;
  static constexpr int NW = NT / 64;
  static constexpr int RPI = NW * R;
  static constexpr int IT = (NROWS + RPI - 1) / RPI;
  static constexpr int SCRATCH = RPI * NCOLS;
  uint2 w[IT][PL];

  __device__ __forceinline__ int row(int it) const {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    return it * RPI + wid * R + lane / G;
  }
  // clamped, unconditional loads: padding rows / columns are never used (forward stores only
  // r < NROWS, v < NV; backward scales padding rows by 0 and stores only v < NV)
  // 32-bit unsigned element offsets (SGPR base + one VGPR offset per load, not a 64-bit address
  // pair per load: all IT * PL loads are in flight at once); clamped only where a row / column
  // group can run past the layer (compile-time per iteration)
  __device__ __forceinline__ void load(const uint16_t* __restrict__ W) {
    const unsigned lane = threadIdx.x & 63, wid = threadIdx.x >> 6, gl = lane % G;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const unsigned r0 = it * RPI + wid * R + lane / G;
      const unsigned r = ((it + 1) * RPI > NROWS) ? min(r0, (unsigned)NROWS - 1) : r0;
#pragma unroll
      for (int i = 0; i < PL; ++i) {
        const unsigned v = ((i + 1) * G > NV) ? min(gl + i * G, (unsigned)NV - 1) : gl + i * G;
        w[it][i] = *reinterpret_cast<const uint2*>(W + (r * NCOLS + 4 * v));
      }
    }
  }
  template <bool RELU>
  __device__ __forceinline__ void fwd(const float* xin, const float* bias, float* out_lds,
                                      float* __restrict__ out_g) const {
    const int gl = (threadIdx.x & 63) % G;
    const float4* x4 = reinterpret_cast<const float4*>(xin);
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < PL; ++i) {
        const int v = gl + i * G;
        if (v < NV) {
          const float4 xv = x4[v], wq = unpack4(w[it][i]);
          acc = fmaf(wq.x, xv.x, acc);
          acc = fmaf(wq.y, xv.y, acc);
          acc = fmaf(wq.z, xv.z, acc);
          acc = fmaf(wq.w, xv.w, acc);
        }
      }
      acc = group_reduce_last<G>(acc);
      const int r = row(it);
      if (gl == G - 1 && r < NROWS) {
        float o = acc + bias[r];
        if (RELU) o = fmaxf(o, 0.f);
        out_lds[r] = o;
        if (out_g) out_g[r] = o;
      }
    }
  }
  // out[k] = mask(k) * sum_r d[r] W[r][k]; scratch >= SCRATCH floats. Ends with a barrier.
  __device__ __forceinline__ void bwd(const float* d, float* scratch, float* out_lds, float* __restrict__ out_g,
                                      const float* mask, uint16_t* out_b16 = nullptr) const {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, gl = lane % G, grp = wid * R + lane / G;
    float dv[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int r = row(it);
      dv[it] = r < NROWS ? d[r] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < PL; ++i) {
      const int v = gl + i * G;
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const float4 wq = unpack4(w[it][i]);
        acc.x = fmaf(dv[it], wq.x, acc.x);
        acc.y = fmaf(dv[it], wq.y, acc.y);
        acc.z = fmaf(dv[it], wq.z, acc.z);
        acc.w = fmaf(dv[it], wq.w, acc.w);
      }
      if (v < NV) reinterpret_cast<float4*>(scratch)[grp * NV + v] = acc;
    }
    lbar();
    for (int k = threadIdx.x; k < NCOLS; k += NT) {
      float sum = 0.f;
#pragma unroll 8
      for (int g = 0; g < RPI; ++g) sum += scratch[g * NCOLS + k];
      if (mask) sum = mask[k] > 0.f ? sum : 0.f;
      out_lds[k] = sum;
      if (out_g) out_g[k] = sum;
      if (out_b16) out_b16[k] = f32_to_bf16(sum);
    }
    lbar();
  }
};

constexpr int cmax(int a, int b) { return a > b ? a : b; }
constexpr int cmin(int a, int b) { return a < b ? a : b; }

// fc1 (FLAT -> F1, 62 % of the model's weights) on the matrix cores, the sample's input row
// broadcast over the 16 A rows. Forward: FNT tiles of 16 outputs, one per wave of the LAST FNT
// waves, all K steps of 32 inputs in that wave; backward-data: BNT tiles of 16 inputs over waves
// 1-15 (wave 0 runs the softmax-CE meanwhile), K steps over the outputs, from the transposed bf16
// image. B fragments live in registers; their ~100 KB per direction are fetched where the
// issuing waves are otherwise idle or light (the vector memory path of a CU moves them at
// ~35 B/clk and a wave stalls while its loads queue): forward at P2 (waves 8-15 carry one conv1
// tile, the others two), backward during the softmax-CE.
template <class D>
struct Fc1 {
  static constexpr int FNT = (D::F1 + 15) / 16, FKS = (D::FLAT + 31) / 32, FW0 = 16 - FNT;
  static constexpr int BNT = (D::FLAT + 15) / 16, BKS = (D::F1 + 31) / 32, BTP = (BNT + 14) / 15;
  static_assert(D::FLAT % 8 == 0 && D::F1 % 8 == 0 && D::F1 * D::FLAT <= 400 * 120 && FNT <= 16, "fc1 fragments");
};

template <class D>
struct KsLds {
  using L2 = BLinear<D::F1, D::F2, kT>;
  using L3 = BLinear<D::F2, D::NC, kT>;
  using F = Fc1<D>;
  static constexpr int SCR = cmax(cmax(L2::SCRATCH, L3::SCRATCH), 3 * 5 * 256);
  // zero-filled at entry (one contiguous span): every image whose padding / untouched cells an
  // MFMA fragment reads
  alignas(16) uint16_t p1h[14 * P1HS * 8];           // pooled conv1 [y][x][ic8]
  alignas(16) uint16_t p1c[D::C1 * 14 * P1CS];       // pooled conv1 [ic][y][x]
  alignas(16) uint16_t dch[18 * DCHS * 16];          // unpooled conv2-out grad, padded [Y+4][X+4][oc16]
  alignas(16) uint16_t dcc[16 * 10 * DCCS];          // unpooled conv2-out grad [oc16][Y][X]
  alignas(16) uint16_t d1[D::C1 * D1S];              // unpooled conv1-out grad [oc][Y][X32]
  // end of the zero span
  alignas(16) uint16_t xh[32 * XHS * 4];             // input [Y][X][c4] (c = 3 zero; X >= 32 never read)
  alignas(16) uint16_t xc[3 * 32 * XCS];             // input [c][Y][X48] (X >= 32 zeroed separately)
  alignas(16) uint16_t w1f[4 * 64 * 8];              // conv1 B fragments [kstep][lane][8]
  alignas(16) uint16_t w2f[7 * 64 * 8];              // conv2 forward B fragments
  alignas(16) uint16_t w2d[15 * 64 * 8];             // conv2 dgrad B fragments
  alignas(16) uint16_t fb16[32 * F::FKS];           // flattened pooled conv2, bf16 (fc1 A row; tail zero)
  alignas(16) uint16_t dh1b[32 * F::BKS];            // fc1 output gradient, bf16 (fc1 dgrad A row; tail zero)
  alignas(16) float df[D::FLAT];                     // its gradient
  alignas(16) float sh1[D::F1];
  alignas(16) float sh2[D::F2];
  alignas(16) float sdh1[D::F1];
  alignas(16) float sdh2[D::F2];
  alignas(16) float slog[64];
  alignas(16) float sdl[64];
  alignas(16) float scr[SCR];                        // fc bwd row-group partials / conv1 wgrad partials
  alignas(16) float f32[D::FLAT];                    // flattened pooled conv2, fp32 (stored for the fc1 wgrad)
  unsigned long long tr[32];                         // LENET_TRACE stamps
  double ce[2];                                      // this sample's (loss / B, hit / B)
  alignas(16) uint8_t raw[3072];                     // this step's raw image (staged or gathered)
  float b1s[16], b2s[16];
  alignas(16) float fb[D::F1 + D::F2 + D::NC];       // fc biases
  uint8_t i1[D::C1 * 196];
  uint8_t i2[D::FLAT];
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
__global__ __launch_bounds__(kT) void lenet_ms(int mode, LeNetPtrs P, LeNetAug A, LeNetOpt O, float inv_B) {
  constexpr int C1 = D::C1, C2 = D::C2, FLAT = D::FLAT, F1 = D::F1, F2 = D::F2, NC = D::NC;
  using S = KsLds<D>;
  static_assert(offsetof(S, w2f) == offsetof(S, w1f) + 2 * kW2F && offsetof(S, w2d) == offsetof(S, w1f) + 2 * kW2D,
                "fragment images must be contiguous");
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

  // ---- P0: every independent load in flight together ----------------------------------------
  // straight-line and unconditional (ctrl / meta2 / stage2 are host-checked), ctrl first: the
  // only values needed before the others arrive (vmcnt retires in issue order)
  const bool aug = A.data != nullptr;
  const int64_t step = sload(A.ctrl), sie = sload(A.ctrl + 1);
  const int64_t mstep = sload(P.meta2 + 4 * b), mpos = sload(P.meta2 + 4 * b + 1), mtgt = sload(P.meta2 + 4 * b + 3);
  uint4 sraw = reinterpret_cast<const uint4*>(P.stage2 + (int64_t)b * 3072)[min(t, 191)];
  const bool stage_on = aug && w == 15;  // next-step staging wave (see P2)
  // (vector loads, issued before the bulk: scalar ones would be waited for by every LDS barrier's
  // lgkmcnt(0), and the staging decision they feed is taken in P2, off the critical path)
  longlong2 mN01 = make_longlong2(-1, -1);
  long long mN2 = -1;
  if (stage_on) {
    mN01 = *reinterpret_cast<const longlong2*>(P.metaN + 4 * b);
    mN2 = P.metaN[4 * b + 2];
  }
  float xin[3] = {0.f, 0.f, 0.f};
  if (!aug) {
#pragma unroll
    for (int c = 0; c < 3; ++c) xin[c] = P.x[(int64_t)b * 3072 + c * 1024 + t];
  }
  // conv weight B-fragment images (bf16, packed by the optimizer / lenet_mpack): 24 KB, linear
  const uint4* wimg4 = reinterpret_cast<const uint4*>(P.wimg);
  constexpr int WI1 = kWimg / 8 - 1024;  // uint4s of the image past the first 1024
  const uint4 wi0 = wimg4[t], wi1 = wimg4[1024 + min(t, WI1 - 1)];
  const float b1v = P.b1[min(t, C1 - 1)], b2v = P.b2[min(t, C2 - 1)];
  constexpr int NFB = F1 + F2 + NC;
  const float fbv = t < F1 ? P.b3[t] : (t < F1 + F2 ? P.b4[min(t - F1, F2 - 1)] : P.b5[min(max(t - F1 - F2, 0), NC - 1)]);
  using F1M = typename S::F;
  u32x4 f1w[F1M::FKS];  // fc1 forward B fragments (row-major W rows of the shadow: 16 B per lane)
  typename S::L2 l2;
  typename S::L3 l3;
  // fc weights: issued once this step's image and conv fragments are in LDS (fc1: start of P2; fc2 /
  // fc3: start of P3, where conv1's registers are free), so that their transfer does not delay
  // those. Padding lanes re-read a valid lane's line (coalesced).
  auto load_fc = [&]() {
    if (w >= F1M::FW0) {
      const unsigned row = min(16u * (w - F1M::FW0) + m, (unsigned)F1 - 1);
#pragma unroll
      for (int q = 0; q < F1M::FKS; ++q) {
        const unsigned col = min(32u * q + 8 * g, (unsigned)FLAT - 8);
        f1w[q] = *reinterpret_cast<const u32x4*>(P.shadow + O.off[4] + row * FLAT + col);
      }
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
    // zero span [p1h .. d1 end) and the X >= 32 columns of xc
    constexpr int ZB = (int)(offsetof(S, xh) - offsetof(S, p1h));
    static_assert(ZB % 16 == 0, "zero span");
    uint4* z = reinterpret_cast<uint4*>(L.p1h);
    for (int e = t; e < ZB / 16; e += kT) z[e] = make_uint4(0u, 0u, 0u, 0u);
    if (t < 3 * 32 * 2) reinterpret_cast<uint4*>(L.xc + (t >> 1) * XCS + 32)[t & 1] = make_uint4(0u, 0u, 0u, 0u);
    if (t < 32 * S::F::FKS - FLAT) L.fb16[FLAT + t] = 0;
    if (t < 32 * S::F::BKS - F1) L.dh1b[F1 + t] = 0;
    uint4* wl = reinterpret_cast<uint4*>(L.w1f);  // w1f | w2f | w2d are contiguous
    wl[t] = wi0;
    if (t < WI1) wl[1024 + t] = wi1;
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
      if (t < 192) reinterpret_cast<uint4*>(L.raw)[t] = graw;
    } else {
      tgt = mtgt;
      if (t < 192) reinterpret_cast<uint4*>(L.raw)[t] = sraw;
    }
    int ci, cj;
    bool fl;
    aug_params(A, step, pos, ci, cj, fl);
    lbar();
    stamp(17);
    float v[3];
    aug_pixel(L.raw, Y0, X0, ci, cj, fl, A, v);
    px = make_uint2(pack2(f32_to_bf16(v[0]), f32_to_bf16(v[1])), pack2(f32_to_bf16(v[2]), 0));
  } else {
    px = make_uint2(pack2(f32_to_bf16(xin[0]), f32_to_bf16(xin[1])), pack2(f32_to_bf16(xin[2]), 0));
    tgt = sload(P.targets + b);
  }
  reinterpret_cast<uint2*>(L.xh)[Y0 * XHS + X0] = px;
  L.xc[(0 * 32 + Y0) * XCS + X0] = (uint16_t)(px.x & 0xffff);
  L.xc[(1 * 32 + Y0) * XCS + X0] = (uint16_t)(px.x >> 16);
  L.xc[(2 * 32 + Y0) * XCS + X0] = (uint16_t)(px.y & 0xffff);
  lbar();
  stamp(1);

  load_fc();
  // ---- P2: conv1 (MFMA) + bias + ReLU + maxpool in registers -> p1 images, i1 ------------------
  // M = (pooled cell, window y) rows, N = (out channel, window x) columns, K = (kh, x pair, c4): a
  // lane's accumulators are the window rows of two cells, the partner lane (n ^ 1) holds the other
  // window column. 25 tiles x 4 k-steps; B fragments (4 x 16 B per lane) read once per wave.
  {
    u32x4 bw[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) bw[s] = *reinterpret_cast<const u32x4*>(L.w1f + (s * 64 + lane) * 8);
    const int a = m >> 2, r = m & 3, dx = m & 1, oc = m >> 1;
    const float bias = L.b1s[min(oc, 15)];
    for (int T = w; T < 25; T += 16) {
      const int cell = min(8 * T + 2 * a + (r >> 1), 195);
      const int py = cell / 14, pxx = cell - 14 * py, Y = 2 * py + (r & 1);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int qq = 4 * s + g, kh = qq / 3, i = qq - 3 * kh;
        u32x4 av = *reinterpret_cast<const u32x4*>(L.xh + ((qq < 15 ? (Y + kh) * XHS + 2 * pxx + 2 * i : 0)) * 4);
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
        L.p1h[(cy * P1HS + cx) * 8 + oc] = hv;
        L.p1c[(oc * 14 + cy) * P1CS + cx] = hv;
        L.i1[oc * 196 + cc] = code;
      }
    }
  }
  lbar();
  stamp(2);

  l2.load(P.shadow + O.off[6]);
  l3.load(P.shadow + O.off[8]);
  // next-step staging (wave 15, two steps deep so that no load waits on another inside this kernel):
  // metaN[b] = (step, position, perm entry) looked up by the PREVIOUS step for step + 1; when it
  // matches, the raw image of step + 1 is gathered now (stored to stage2 in P10). The perm entry
  // for step + 2 is looked up here and published to metaN in P10. A mismatch (epoch start, new
  // permutation, ...) stages nothing: the next step then gathers its images itself. All vector
  // loads, first waited for in P10.
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

  // ---- P3: conv2 (MFMA) + bias + ReLU + maxpool -> f (flatten order oc*25 + cell), i2 ----------
  if (w < 7) {
    const int r = 16 * w + m, cell = min(r >> 2, 24), q = r & 3;
    const int py = cell / 5, pxx = cell - 5 * py, y = 2 * py + (q >> 1), x = 2 * pxx + (q & 1);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 7; ++s) {
      const int tap = 4 * s + g, kh = tap / 5, kw = tap - 5 * kh;
      u32x4 a = *reinterpret_cast<const u32x4*>(L.p1h + ((tap < 25 ? (y + kh) * P1HS + x + kw : 0)) * 8);
      if (tap >= 25) a = u32x4{0u, 0u, 0u, 0u};
      acc = mfma(a, *reinterpret_cast<const u32x4*>(L.w2f + (s * 64 + lane) * 8), acc);
    }
    const int cc = 4 * w + g, oc = m;
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

  // ---- P4-P9: fc1 -> fc2 -> fc3 -> softmax-CE -> fc dgrad chain -------------------------------
  if (w >= F1M::FW0) {
    const int tn = w - F1M::FW0;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < F1M::FKS; ++q) {
      const int col = 32 * q + 8 * g;
      const u32x4 av = *reinterpret_cast<const u32x4*>(L.fb16 + col);
      const bool ok = 16 * tn + m < F1 && col < FLAT;
      acc = mfma(av, ok ? f1w[q] : u32x4{0u, 0u, 0u, 0u}, acc);
    }
    const int r = 16 * tn + m;
    if (g == 0 && r < F1) L.sh1[r] = fmaxf(acc[0] + L.fb[r], 0.f);  // C row 0 (all rows are equal)
  }
  lbar();
  stamp(18);
  l2.template fwd<true>(L.sh1, L.fb + F1, L.sh2, nullptr);
  lbar();
  stamp(19);
  l3.template fwd<false>(L.sh2, L.fb + F1 + F2, L.slog, nullptr);
  lbar();
  stamp(4);
  u32x4 f1t[F1M::BTP][F1M::BKS];  // fc1 backward-data B fragments (waves 1-15), fetched during the CE
  if (w > 0) {
#pragma unroll
    for (int tp = 0; tp < F1M::BTP; ++tp) {
      const unsigned c = min(16u * (w - 1 + 15 * tp) + m, (unsigned)FLAT - 1);
#pragma unroll
      for (int ks = 0; ks < F1M::BKS; ++ks) {
        const unsigned r0 = min(32u * ks + 8 * g, (unsigned)F1 - 8);
        f1t[tp][ks] = *reinterpret_cast<const u32x4*>(P.wimg + kFc1T + c * F1 + r0);
      }
    }
  }
  if (w == 0) {
    constexpr int GC = pow2_ge(NC);
    const float z = lane < NC ? L.slog[lane] : -INFINITY;
    const float mx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(group_reduce_last<GC, true>(z)), GC - 1));
    const float e = lane < NC ? expf(z - mx) : 0.f;
    const float s = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(group_reduce_last<GC>(e)), GC - 1));
    const float lse = mx + logf(s);
    const bool valid = tgt >= 0 && tgt < NC;
    const unsigned long long am_mask = __ballot(lane < NC && z == mx);
    const int am = __ffsll((long long)am_mask) - 1;
    const float loss = valid ? lse - L.slog[valid ? tgt : 0] : 0.f;
    if (lane < NC) {
      const float dl = valid ? (e / s - (lane == tgt ? 1.f : 0.f)) * inv_B : 0.f;
      L.sdl[lane] = dl;
    }
    if (lane == 0) {
      L.ce[0] = (double)loss * (double)inv_B;
      L.ce[1] = (am == tgt) ? (double)inv_B : 0.0;
    }
  }
  lbar();
  stamp(20);
  l3.bwd(L.sdl, L.scr, L.sdh2, nullptr, L.sh2);
  stamp(21);
  l2.bwd(L.sdh2, L.scr, L.sdh1, nullptr, L.sh1, L.dh1b);
  stamp(22);
  // (l2.bwd also wrote the bf16 copy dh1b: fc1's dgrad A row)
#pragma unroll
  for (int tp = 0; tp < F1M::BTP; ++tp) {
    const int tile = w - 1 + 15 * tp;
    if (w > 0 && tile < F1M::BNT) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < F1M::BKS; ++ks) {
        const u32x4 av = *reinterpret_cast<const u32x4*>(L.dh1b + 32 * ks + 8 * g);
        const bool ok = 16 * tile + m < FLAT && 32 * ks + 8 * g < F1;
        acc = mfma(av, ok ? f1t[tp][ks] : u32x4{0u, 0u, 0u, 0u}, acc);
      }
      const int c = 16 * tile + m;
      if (g == 0 && c < FLAT) L.df[c] = acc[0];
    }
  }
  lbar();
  stamp(5);

  // ---- P10: unpool2 -> the conv2-output gradient images (zero except at arg-max cells) ---------
  for (int e = t; e < FLAT; e += kT) {
    const int code = L.i2[e];
    if (code < 4) {
      const int oc = e / 25, cell = e - 25 * oc, py = cell / 5, pxx = cell - 5 * py;
      const int Y = 2 * py + (code >> 1), X = 2 * pxx + (code & 1);
      const uint16_t v = f32_to_bf16(L.df[e]);
      L.dch[((Y + 4) * DCHS + X + 4) * 16 + oc] = v;
      L.dcc[(oc * 10 + Y) * DCCS + X] = v;
    }
  }
  if (stage_on) {  // wave 15 (no unpool work): publish the next step's raw image + tags
    if (st1) {
      uint4* dst = reinterpret_cast<uint4*>(P.stage2 + (int64_t)b * 3072);
      dst[lane] = nraw0;
      dst[lane + 64] = nraw1;
      dst[lane + 128] = nraw2;
    }
    if (lane == 0) {
      if (st1) {
        P.meta2[4 * b] = step + 1;
        P.meta2[4 * b + 1] = pos1;
        P.meta2[4 * b + 2] = idx1;
        P.meta2[4 * b + 3] = ntgtv;
      }
      P.metaN[4 * b] = step + 2;
      P.metaN[4 * b + 1] = pos2;
      P.metaN[4 * b + 2] = nperm2v;
    }
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
      u32x4 a = *reinterpret_cast<const u32x4*>(L.dch + ((pp < 30 ? (Y - kh + 4) * DCHS + 2 * xp + 5 - u : 0)) * 16 + oc0);
      if (pp >= 30) a = u32x4{0u, 0u, 0u, 0u};
      acc = mfma(a, *reinterpret_cast<const u32x4*>(L.w2d + (s * 64 + lane) * 8), acc);
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
          L.d1[ic * D1S + (2 * py + (code >> 1)) * 32 + 2 * pxx + (code & 1)] = f32_to_bf16(acc[r]);
        }
      }
    }
  } else {
    // 10 M-tiles over waves 7-15 (wave 7: two): tile tt = (kw, half); rows (ic, kh) = 16 * half + m;
    // row 31 of tile 1 = ones (bias). Wave 15's staging stores were issued in P10.
    const int t0 = w - 7, t1 = w == 7 ? 2 : w - 6;
    for (int tt0 = t0; tt0 < t1; ++tt0) {
      const int tt = w == 7 && tt0 == 1 ? 9 : tt0;
      const int kw = tt >> 1, h = tt & 1, i = 16 * h + m, ic = i / 5, kh = i - 5 * ic;
      const bool valid = ic < C1, ones = tt == 1 && m == 15;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 5; ++s) {
        const int y = 2 * s + (g >> 1), x0 = 8 * (g & 1);
        const u32x4 bq = *reinterpret_cast<const u32x4*>(L.dcc + (m * 10 + y) * DCCS + x0);
        const uint16_t* rowp = L.p1c + ((valid ? ic : 0) * 14 + y + (valid ? kh : 0)) * P1CS + x0;
        const u32x4 lo = *reinterpret_cast<const u32x4*>(rowp), hi = *reinterpret_cast<const u32x4*>(rowp + 8);
        u32x4 a;
        switch (kw) {
          case 0: a = fshift<0>(lo, hi); break;
          case 1: a = fshift<1>(lo, hi); break;
          case 2: a = fshift<2>(lo, hi); break;
          case 3: a = fshift<3>(lo, hi); break;
          default: a = fshift<4>(lo, hi); break;
        }
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
    }
  }
  lbar();
  stamp(7);

  // ---- P13: conv1 wgrad (waves 0-14: tile kw = w / 3, K range w % 3) ---------------------------
  //           next-step staging (wave 15)
  if (w < 15) {
    const int kw = w / 3, kp = w - 3 * kw, c = m / 5, kh = m - 5 * c;
    const bool valid = m < 15, ones = m == 15 && kw == 0;
    const int ya = 10 * kp, yb = min(ya + 10, 28), x0 = 8 * g;
    const uint16_t* xrow = L.xc + ((valid ? c : 0) * 32 + (valid ? kh : 0)) * XCS + x0;
    const uint16_t* drow = L.d1 + min(m, C1 - 1) * D1S + x0;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int Y = ya; Y < yb; ++Y) {
      u32x4 bq = *reinterpret_cast<const u32x4*>(drow + Y * 32);
      if (m >= C1) bq = u32x4{0u, 0u, 0u, 0u};
      const u32x4 lo = *reinterpret_cast<const u32x4*>(xrow + Y * XCS), hi = *reinterpret_cast<const u32x4*>(xrow + Y * XCS + 8);
      u32x4 a;
      switch (kw) {
        case 0: a = fshift<0>(lo, hi); break;
        case 1: a = fshift<1>(lo, hi); break;
        case 2: a = fshift<2>(lo, hi); break;
        case 3: a = fshift<3>(lo, hi); break;
        default: a = fshift<4>(lo, hi); break;
      }
      if (!valid) a = ones ? u32x4{0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u} : u32x4{0u, 0u, 0u, 0u};
      acc = mfma(a, bq, acc);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) L.scr[((kp * 5 + kw) * 16 + 4 * g + r) * 16 + m] = acc[r];
  }
  lbar();
  for (int e = t; e < 5 * 256; e += kT) {
    const int kw = e >> 8, i = (e >> 4) & 15, oc = e & 15;
    const float v = (L.scr[e] + L.scr[1280 + e]) + L.scr[2560 + e];
    if (oc < C1) {
      if (i < 15) slab[oc * 76 + (i / 5) * 25 + (i % 5) * 5 + kw] = v;
      else if (kw == 0) slab[oc * 76 + 75] = v;
    }
  }
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
}

// ---------------------------------------------------------------------------
// KW: batch reductions + optimizer
// ---------------------------------------------------------------------------
struct Ctx {
  bool on;
  float lr, t;
};

__device__ __forceinline__ void upd1(const LeNetOpt& O, const Ctx& c, uint16_t* shadow, int64_t i, float g, float p,
                                     float a, float s) {
  O.g[i] = g;
  if (!c.on) return;
  opt_update(O.h, c.lr, c.t, p, g, a, s);
  O.p[i] = p;
  if (O.s1) O.s1[i] = a;
  if (O.s2) O.s2[i] = s;
  if (shadow) shadow[i] = f32_to_bf16(p);
}

template <class D>
__host__ __device__ constexpr int mw_conv_blocks() {
  return (D::S1 + D::S2 + kWgT - 1) / kWgT;
}
// fc weight gradients: a block holds kFcItems (row, 4-column) items x kFcQ batch quarters; each
// thread sums its quarter of the batch (all its loads in flight at once: one round trip at batch
// 32), the quarters are combined in a fixed order through LDS
constexpr int kFcQ = 4, kFcItems = kWgT / kFcQ;
template <int NCOLS>
__host__ __device__ constexpr int fc_items(int nrows) {
  return nrows * (NCOLS / 4);
}
template <class D>
__host__ __device__ constexpr int mw_fc_blocks() {
  return (fc_items<D::FLAT>(D::F1) + kFcItems - 1) / kFcItems + (fc_items<D::F1>(D::F2) + kFcItems - 1) / kFcItems +
         (fc_items<D::F2>(D::NC) + kFcItems - 1) / kFcItems;
}

template <int NCOLS>
__device__ __forceinline__ void fc_wgrad(int blk, int nrows, int B, const float* __restrict__ dY,
                                         const float* __restrict__ X, const LeNetOpt& O, const Ctx& c,
                                         uint16_t* shadow, int64_t offW, int64_t offb, float* red,
                                         uint16_t* __restrict__ timg = nullptr) {
  constexpr int NV = NCOLS / 4;
  const int t = threadIdx.x, q = t & (kFcQ - 1);
  const int item = blk * kFcItems + (t >> 2);
  const bool ok = item < nrows * NV;
  const int it = ok ? item : 0, j = it / NV, v = it - j * NV;
  const int64_t iw = offW + 4 * (int64_t)it, ib = offb + j;
  float4 pw = make_float4(0.f, 0.f, 0.f, 0.f), aw = pw, sw = pw;
  float pb = 0.f, ab = 0.f, sb = 0.f;
  if (c.on && q == 0 && ok) {  // optimizer state in flight together with the batch loads
    pw = *reinterpret_cast<const float4*>(O.p + iw);
    if (O.s1) aw = *reinterpret_cast<const float4*>(O.s1 + iw);
    if (O.s2) sw = *reinterpret_cast<const float4*>(O.s2 + iw);
    if (v == 0) {
      pb = O.p[ib];
      if (O.s1) ab = O.s1[ib];
      if (O.s2) sb = O.s2[ib];
    }
  }
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  float bacc = 0.f;
  const float4* x4 = reinterpret_cast<const float4*>(X);
  for (int b0 = 0; b0 < B; b0 += 8 * kFcQ) {  // this thread: samples b0 + 8q .. b0 + 8q + 7
    float d[8];
    float4 xv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int bb = min(b0 + 8 * q + u, B - 1);
      d[u] = dY[(int64_t)bb * nrows + j];
      xv[u] = x4[(int64_t)bb * NV + v];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float du = b0 + 8 * q + u < B ? d[u] : 0.f;
      acc.x = fmaf(du, xv[u].x, acc.x);
      acc.y = fmaf(du, xv[u].y, acc.y);
      acc.z = fmaf(du, xv[u].z, acc.z);
      acc.w = fmaf(du, xv[u].w, acc.w);
      bacc += du;
    }
  }
  float* r = red + 5 * t;
  r[0] = acc.x;
  r[1] = acc.y;
  r[2] = acc.z;
  r[3] = acc.w;
  r[4] = bacc;
  __syncthreads();
  if (q != 0 || !ok) return;
#pragma unroll
  for (int k = 1; k < kFcQ; ++k) {  // fixed order: quarter 0 + 1 + 2 + 3
    acc.x += r[5 * k];
    acc.y += r[5 * k + 1];
    acc.z += r[5 * k + 2];
    acc.w += r[5 * k + 3];
    bacc += r[5 * k + 4];
  }
  *reinterpret_cast<float4*>(O.g + iw) = acc;
  if (c.on) {
    opt_update(O.h, c.lr, c.t, pw.x, acc.x, aw.x, sw.x);
    opt_update(O.h, c.lr, c.t, pw.y, acc.y, aw.y, sw.y);
    opt_update(O.h, c.lr, c.t, pw.z, acc.z, aw.z, sw.z);
    opt_update(O.h, c.lr, c.t, pw.w, acc.w, aw.w, sw.w);
    *reinterpret_cast<float4*>(O.p + iw) = pw;
    if (O.s1) *reinterpret_cast<float4*>(O.s1 + iw) = aw;
    if (O.s2) *reinterpret_cast<float4*>(O.s2 + iw) = sw;
    const uint16_t h0 = f32_to_bf16(pw.x), h1 = f32_to_bf16(pw.y), h2 = f32_to_bf16(pw.z), h3 = f32_to_bf16(pw.w);
    if (shadow) *reinterpret_cast<uint2*>(shadow + iw) = make_uint2(pack2(h0, h1), pack2(h2, h3));
    if (timg) {  // transposed bf16 image [in][out] (the per-sample kernel's fc1 dgrad operand)
      timg[(4 * v + 0) * nrows + j] = h0;
      timg[(4 * v + 1) * nrows + j] = h1;
      timg[(4 * v + 2) * nrows + j] = h2;
      timg[(4 * v + 3) * nrows + j] = h3;
    }
  }
  if (v == 0) upd1(O, c, shadow, ib, bacc, pb, ab, sb);
}

template <class D>
__global__ __launch_bounds__(kWgT) void lenet_mw(int mode, LeNetPtrs P, LeNetOpt O, int B, int64_t* __restrict__ ctrl) {
  constexpr int C1 = D::C1, C2 = D::C2, F1 = D::F1, F2 = D::F2, NC = D::NC, FLAT = D::FLAT;
  constexpr int NBC = mw_conv_blocks<D>();
  constexpr int NB3 = (fc_items<FLAT>(F1) + kFcItems - 1) / kFcItems,
                NB4 = (fc_items<F1>(F2) + kFcItems - 1) / kFcItems, NB5 = (fc_items<F2>(NC) + kFcItems - 1) / kFcItems;
  __shared__ float red[5 * kWgT];
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
    if (e >= D::S1 + D::S2) return;
    int soff;
    int64_t dst;
    if (e < D::S1) {
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
    O.g[dst] = gsum;
    if (c.on) {
      opt_update(O.h, c.lr, c.t, p, gsum, a, s);
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
  if (blk < NB3) {
    fc_wgrad<FLAT>(blk, F1, B, P.dh1, P.p2, O, c, shadow, O.off[4], O.off[5], red, P.wimg ? P.wimg + kFc1T : nullptr);
  } else if ((blk -= NB3) < NB4) {
    fc_wgrad<F1>(blk, F2, B, P.dh2, P.h1, O, c, shadow, O.off[6], O.off[7], red);
  } else if ((blk -= NB4) < NB5) {
    fc_wgrad<F2>(blk, NC, B, P.dlogits, P.h2, O, c, shadow, O.off[8], O.off[9], red);
  } else {
    // loss / accuracy of the step in sample order (fixed tree): bitwise reproducible epoch stats
    double* red2 = reinterpret_cast<double*>(red);
    const int lane = t & 63, wid = t >> 6;
    double s0 = 0.0, s1 = 0.0;
    for (int i = t; i < B; i += kWgT) {
      s0 += P.cestat[2 * i];
      s1 += P.cestat[2 * i + 1];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      s0 += __shfl_xor(s0, o, 64);
      s1 += __shfl_xor(s1, o, 64);
    }
    if (lane == 0) {
      red2[wid] = s0;
      red2[4 + wid] = s1;
    }
    __syncthreads();
    if (t == 0) {
      P.stats[0] += ((red2[0] + red2[1]) + red2[2]) + red2[3];
      P.stats[1] += ((red2[4] + red2[5]) + red2[6]) + red2[7];
      if (ctrl) {  // advance the device step counters (next step / lr index / Adam t)
        ctrl[0] = step + 1;
        ctrl[1] = sie + 1;
      }
    }
  }
}

// bf16 shadow of the flat parameters + the conv fragment image, from the fp32 masters (start of
// every captured step sequence, and after each data-parallel optimizer launch)
template <class D>
__global__ __launch_bounds__(256) void lenet_mpack(const float* __restrict__ p, int64_t n, uint16_t* __restrict__ shadow,
                                                  uint16_t* __restrict__ wimg, int64_t off_w1, int64_t off_w2,
                                                  int64_t off_w3) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) shadow[i] = f32_to_bf16(p[i]);
  if (i < kWimg) {
    const int64_t src = wimg_src<D::C1, D::C2>((int)i, off_w1, off_w2);
    wimg[i] = src >= 0 ? f32_to_bf16(p[src]) : (uint16_t)0;
  } else if (i < kWimgTot) {  // fc1 transposed: [c][r] = W3[r][c]
    const int e = (int)(i - kFc1T), cc = e / D::F1, r = e - cc * D::F1;
    wimg[i] = cc < D::FLAT ? f32_to_bf16(p[off_w3 + (int64_t)r * D::FLAT + cc]) : (uint16_t)0;
  }
}

template <class D>
void pack(const LeNetPtrs& P, const LeNetOpt& O, hipStream_t st) {
  const int64_t tot = O.n > kWimgTot ? O.n : kWimgTot;
  hipLaunchKernelGGL(lenet_mpack<D>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, O.p, O.n, P.shadow, P.wimg,
                     O.off[0], O.off[2], O.off[4]);
}

template <class D>
void run(int mode, int B, const LeNetPtrs& P, const LeNetAug& A, const LeNetOpt& O, hipStream_t st) {
  const float inv_B = 1.f / (float)B;
  hipLaunchKernelGGL(lenet_ms<D>, dim3(B), dim3(kT), 0, st, mode, P, A, O, inv_B);
  const int nblk = mw_conv_blocks<D>() + mw_fc_blocks<D>() + 1;
  hipLaunchKernelGGL(lenet_mw<D>, dim3(nblk), dim3(kWgT), 0, st, mode, P, O, B, A.ctrl);
}

}  // namespace lm

int lenet_mfma_slab_floats(int cfg) { return cfg == LENET_TINY ? lm::DmTiny::SLABN : lm::DmDefault::SLABN; }
int lenet_mfma_wimg_elems() { return lm::kWimgTot; }

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
