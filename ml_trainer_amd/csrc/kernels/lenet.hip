// LeNet-5 CIFAR (reference src/model.py:7-24) forward + backward + optimizer
// for gfx950, as five short kernels designed for one hipGraph-captured step.
//
// Why VALU and not MFMA here: the channel counts (3->6->16) and 5x5 taps map
// onto 16x16 MFMA tiles at <=40% occupancy of the tile, and the whole step is
// ~0.13 GFLOP at batch 32 -- the step is bounded by kernel boundaries (~1.5 us
// each, MI355X_MICROARCH.md "boundary" row) and L2 latency, not by FLOPs.  The
// design therefore minimises launches and keeps every intermediate in LDS:
//
//   K1 conv1_fwd   grid (B, C1)     [augment (RandomCrop+HFlip+Normalize) fused] conv5x5+bias+ReLU+maxpool2
//   K2 conv2_fwd   grid (B, C2/4)   conv5x5+bias+ReLU+maxpool2 -> flatten (c*25+h*5+w, src/model.py:20)
//   K3 fc          grid (B)         fc1/fc2/fc3 (+ReLU) -> softmax-CE + accuracy -> fc dgrad chain
//   K4 conv2_dgrad grid (B, 2*C1)   unpool2 -> conv2 dgrad -> ReLU/unpool1 mask -> the sample's conv1
//                                   wgrad slab (blocks y < C1); the sample's conv2 wgrad slab (y >= C1)
//   K5 wgrad       role-split grid  batch sums of the conv wgrad slabs (sample order), fc1..fc3 wgrad
//                  +bias, fused optimizer update, step counters
//                  (the fused KF path keeps the K5 conv roles: conv1 partials reduced in-launch
//                  by the last-arriving block of each channel)
//
// ReLU+maxpool are fused: pool(relu(c)) = relu(max(c)); the gradient reaches the
// first arg-max of the window only when that max is > 0 (torch's threshold_backward
// zeroes it otherwise), so one uint8 per pooled cell stores the arg-max (0..3) or 4
// for "dead".  The backward never materialises the 4x larger un-pooled gradient.
// All batch reductions run in a fixed order: results are bitwise reproducible.
#include <cstdlib>

#include "mlt_common.h"
#include "mlt_kernels.h"
#include "mlt_optim.h"

namespace mlt {

#ifndef MLT_LENET_TRACE_BUILD
#define MLT_LENET_TRACE_BUILD 0  // 1: the LENET_TRACE phase stamps are compiled in
#endif
// (a runtime-disabled stamp still splits the phase code into basic blocks the scheduler cannot move
// loads across: the bf16 kernel ran 0.6 us per step faster with its stamps compiled out, r6g)
constexpr bool kFp32TraceBuild = MLT_LENET_TRACE_BUILD != 0;

typedef __attribute__((address_space(3))) void lds_void_t;

template <int C1_, int C2_, int F1_, int F2_, int NC_>
struct LeNetDims {
  static constexpr int C1 = C1_, C2 = C2_, F1 = F1_, F2 = F2_, NC = NC_, FLAT = C2_ * 25;
  static_assert(C2_ % 4 == 0 && F1_ % 4 == 0 && F2_ % 4 == 0 && NC_ <= 64, "LeNet dims");
};
using LeNetDefault = LeNetDims<6, 16, 120, 84, 10>;
using LeNetTiny = LeNetDims<4, 8, 64, 32, 10>;

constexpr int kTaps1 = 76;        // conv1 wgrad partial: 75 taps + bias
// floats per (sample, channel) slab: [0, 76) conv1 wgrad partial, [128, 128 + C2*25 + C2) conv2
// wgrad partial (K4 path); 2.5 KB, so no two writers share a cache line
constexpr int kSlabStride = 640;
constexpr int kSlab2Off = 128;
constexpr int kSpb1 = 1;          // samples per conv1-wgrad block (slabs per oc = ceil(B / kSpb1)); 4 measured slower

// ---------------------------------------------------------------------------
// K1: [augment] + conv1 + bias + ReLU + maxpool2x2.  One block per (sample, out-channel).
// ---------------------------------------------------------------------------
template <class D>
__global__ __launch_bounds__(256) void lenet_conv1_fwd(LeNetAug aug, const float* __restrict__ w1,
                                                       const float* __restrict__ b1, float* __restrict__ x,
                                                       float* __restrict__ p1, uint8_t* __restrict__ i1,
                                                       int64_t* __restrict__ targets,
                                                       const int64_t* __restrict__ dtargets,
                                                       const uint8_t* __restrict__ staged,
                                                       const int64_t* __restrict__ staged_meta) {
  const int b = blockIdx.x, oc = blockIdx.y, t = threadIdx.x;
  // input image rows at a 46-float stride: the 14 lanes of a pooled row read 2 px apart, so with
  // a 32-float stride the (up to 5) pooled rows of a wave land on the same banks; 2 * 46 = 28 (mod
  // 64) staggers them (even, so the 8-byte window reads stay aligned)
  constexpr int XR = 46, XC = 32 * XR;
  __shared__ __attribute__((aligned(16))) float xs[3 * XC];
  __shared__ __attribute__((aligned(16))) uint4 rawimg[192];
  // filter + bias first: block-uniform scalar loads that overlap the ctrl -> perm -> image chain
  float wr[75];
#pragma unroll
  for (int i = 0; i < 75; ++i) wr[i] = w1[oc * 75 + i];
  const float bias = b1[oc];
  if (aug.data) {
    // The previous step's K4 staged this step's raw images (stage / stage_meta): ctrl, the tag
    // and the staged image are independent loads issued together -- ONE round trip instead of the
    // ctrl -> perm -> image chain. A tag that does not match the position computed from ctrl
    // (first step of an epoch, a new permutation, ...) falls back to the chain.
    const bool staged_ok = staged != nullptr;
    uint4 sv = make_uint4(0, 0, 0, 0);
    int64_t tag = -1, sidx = 0, stgt = 0;
    if (staged_ok) {
      tag = staged_meta[4 * b];
      sidx = staged_meta[4 * b + 1];
      stgt = staged_meta[4 * b + 2];
      if (t < 192) sv = reinterpret_cast<const uint4*>(staged + (int64_t)b * 3072)[t];
    }
    const int64_t step = aug.ctrl[0], sie = aug.ctrl[1];
    int64_t pos = sie * aug.batch_stride + b;
    if (pos >= aug.perm_len) pos %= aug.perm_len;
    MLT_DCHECK(b < aug.batch_stride && pos < aug.perm_len);
    int64_t idx;
    if (staged_ok && tag == pos) {  // block-uniform branch
      idx = sidx;
      if (t < 192) rawimg[t] = sv;
    } else {
      idx = aug.perm[pos];
      MLT_DCHECK(idx >= 0 && idx < aug.n);  // release builds clamp a bad permutation entry
      idx = idx < 0 ? 0 : (idx >= aug.n ? aug.n - 1 : idx);
      stgt = -1;
      if (t < 192) rawimg[t] = reinterpret_cast<const uint4*>(aug.data + idx * 3072)[t];
    }
    const uint64_t h = mix64(mix64(aug.seed + (uint64_t)step) ^ (uint64_t)pos);
    const int span = 2 * aug.pad + 1;
    const int ci = aug.pad ? (int)(h % span) : 0;
    const int cj = aug.pad ? (int)((h >> 20) % span) : 0;
    const bool fl = aug.flip && ((h >> 40) & 1);
    // the raw 3 KB HWC image (16-byte loads) is cropped / flipped / normalised from LDS
    __syncthreads();
    const uint8_t* img = reinterpret_cast<const uint8_t*>(rawimg);
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      const int e = t + i * 256;
      const int c = e >> 10, y = (e >> 5) & 31, xx = e & 31;
      const int sx = fl ? 31 - xx : xx;
      const int r = y + ci - aug.pad, q = sx + cj - aug.pad;
      const bool in = (unsigned)r < 32u && (unsigned)q < 32u;
      const float u = in ? (float)img[(r * 32 + q) * 3 + c] : 0.f;
      const float v = (u / 255.f - aug.mean[c]) / aug.std[c];
      xs[c * XC + y * XR + xx] = v;
      if (oc == 0) x[(int64_t)b * 3072 + e] = v;
    }
    if (oc == 0 && t == 0 && targets) targets[b] = stgt >= 0 ? stgt : dtargets[idx];
  } else {
    const float4* src = reinterpret_cast<const float4*>(x + (int64_t)b * 3072);
    float4 v[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) v[i] = src[t + i * 256];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int e = 4 * (t + i * 256), c = e >> 10, y = (e >> 5) & 31, xx = e & 31;
      float2* d = reinterpret_cast<float2*>(xs + c * XC + y * XR + xx);
      d[0] = make_float2(v[i].x, v[i].y);
      d[1] = make_float2(v[i].z, v[i].w);
    }
  }
  __syncthreads();
  if (t >= 196) return;
  const int py = t / 14, px = t - py * 14, y0 = 2 * py, x0 = 2 * px;
  float a00 = bias, a01 = bias, a10 = bias, a11 = bias;
#pragma unroll
  for (int ic = 0; ic < 3; ++ic) {
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      float in[6];
#pragma unroll
      for (int q = 0; q < 6; ++q) in[q] = xs[ic * XC + (y0 + r) * XR + x0 + q];
      if (r < 5) {
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) {
          const float wv = wr[ic * 25 + r * 5 + kw];
          a00 = fmaf(wv, in[kw], a00);
          a01 = fmaf(wv, in[kw + 1], a01);
        }
      }
      if (r >= 1) {
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) {
          const float wv = wr[ic * 25 + (r - 1) * 5 + kw];
          a10 = fmaf(wv, in[kw], a10);
          a11 = fmaf(wv, in[kw + 1], a11);
        }
      }
    }
  }
  float m = a00;
  int k = 0;
  if (a01 > m) { m = a01; k = 1; }
  if (a10 > m) { m = a10; k = 2; }
  if (a11 > m) { m = a11; k = 3; }
  const int64_t o = ((int64_t)(b * D::C1 + oc) * 14 + py) * 14 + px;
  MLT_DCHECK(oc < D::C1 && py < 14 && px < 14);
  p1[o] = m > 0.f ? m : 0.f;
  i1[o] = m > 0.f ? (uint8_t)k : (uint8_t)4;
}

// ---------------------------------------------------------------------------
// K2: conv2 + bias + ReLU + maxpool2x2 -> flat [B, C2*25].  Block per (sample, 4 out-channels).
// ---------------------------------------------------------------------------
template <class D>
__global__ __launch_bounds__(128) void lenet_conv2_fwd(const float* __restrict__ p1, const float* __restrict__ w2,
                                                       const float* __restrict__ b2, float* __restrict__ p2,
                                                       uint8_t* __restrict__ i2) {
  constexpr int C1 = D::C1, NP4 = C1 * 49, NW4 = C1 * 25;
  const int b = blockIdx.x, og = blockIdx.y, t = threadIdx.x;
  __shared__ __attribute__((aligned(16))) float ps[C1 * 196];
  __shared__ __attribute__((aligned(16))) float ws[4 * C1 * 25];
  {
    const float4* src = reinterpret_cast<const float4*>(p1 + (int64_t)b * C1 * 196);
    const float4* wsrc = reinterpret_cast<const float4*>(w2 + og * 4 * C1 * 25);
    float4 a[(NP4 + 127) / 128], wv[(NW4 + 127) / 128];
#pragma unroll
    for (int i = 0; i < (NP4 + 127) / 128; ++i)
      if (t + i * 128 < NP4) a[i] = src[t + i * 128];
#pragma unroll
    for (int i = 0; i < (NW4 + 127) / 128; ++i)
      if (t + i * 128 < NW4) wv[i] = wsrc[t + i * 128];
#pragma unroll
    for (int i = 0; i < (NP4 + 127) / 128; ++i)
      if (t + i * 128 < NP4) reinterpret_cast<float4*>(ps)[t + i * 128] = a[i];
#pragma unroll
    for (int i = 0; i < (NW4 + 127) / 128; ++i)
      if (t + i * 128 < NW4) reinterpret_cast<float4*>(ws)[t + i * 128] = wv[i];
  }
  __syncthreads();
  if (t >= 100) return;
  const int ol = t / 25, p = t - ol * 25, py = p / 5, px = p - py * 5, y0 = 2 * py, x0 = 2 * px;
  const int oc = og * 4 + ol;
  const float bias = b2[oc];
  float a00 = bias, a01 = bias, a10 = bias, a11 = bias;
  const float* w = ws + ol * C1 * 25;
#pragma unroll 2
  for (int ic = 0; ic < C1; ++ic) {
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      float in[6];
#pragma unroll
      for (int q = 0; q < 6; ++q) in[q] = ps[ic * 196 + (y0 + r) * 14 + x0 + q];
      if (r < 5) {
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) {
          const float wv = w[ic * 25 + r * 5 + kw];
          a00 = fmaf(wv, in[kw], a00);
          a01 = fmaf(wv, in[kw + 1], a01);
        }
      }
      if (r >= 1) {
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) {
          const float wv = w[ic * 25 + (r - 1) * 5 + kw];
          a10 = fmaf(wv, in[kw], a10);
          a11 = fmaf(wv, in[kw + 1], a11);
        }
      }
    }
  }
  float m = a00;
  int k = 0;
  if (a01 > m) { m = a01; k = 1; }
  if (a10 > m) { m = a10; k = 2; }
  if (a11 > m) { m = a11; k = 3; }
  const int64_t o = (int64_t)b * D::FLAT + oc * 25 + p;
  p2[o] = m > 0.f ? m : 0.f;
  i2[o] = m > 0.f ? (uint8_t)k : (uint8_t)4;
}

// ---------------------------------------------------------------------------
// K3 helpers: a dense layer whose weights stay in registers for the whole
// kernel. Loaded once (all loads issued back to back), used by the forward
// (row dot products, G lanes per row) AND by the backward-data pass (each lane
// multiplies the same register fragment by the upstream gradient; the RPI
// row-groups are then summed through LDS in a fixed order). W is read from
// L2 exactly once per sample instead of twice, and no layer waits on a
// dependent chain of L2 round trips.
// ---------------------------------------------------------------------------
constexpr int pow2_ge(int v) { return v <= 1 ? 1 : v <= 2 ? 2 : v <= 4 ? 4 : v <= 8 ? 8 : v <= 16 ? 16 : v <= 32 ? 32 : 64; }

// IR (< IT) keeps only the first IR row-iterations in registers; rows >= IR*RPI are read from an
// LDS image of W (set `lw`, filled by the caller, e.g. by LDS-DMA) -- for a kernel that cannot
// spare IT*PL*4 registers for the whole layer.
template <int NCOLS, int NROWS, int NT, int IR_ = -1>
struct RegLinear {
  static constexpr int NV = NCOLS / 4;
  static constexpr int G = pow2_ge(NV);
  static constexpr int PL = (NV + G - 1) / G;
  static constexpr int R = 64 / G;
  static constexpr int NW = NT / 64;
  static constexpr int RPI = NW * R;  // row groups (rows per iteration over the block)
  static constexpr int IT = (NROWS + RPI - 1) / RPI;
  static constexpr int IR = IR_ < 0 || IR_ > IT ? IT : IR_;  // register-resident iterations
  static constexpr int LROW0 = IR * RPI;                      // first LDS-resident row
  static constexpr int LDS_FLOATS = NROWS > LROW0 ? (NROWS - LROW0) * NCOLS : 0;
  static constexpr int SCRATCH = RPI * NCOLS;
  float4 w[IR > 0 ? IR : 1][PL];
  float bias[IT];
  const float4* lw = nullptr;  // LDS image [NROWS - LROW0][NV] (float4) of the non-resident rows

  __device__ __forceinline__ int row(int it) const {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    return it * RPI + wid * R + lane / G;
  }
  // weight float4 v of the row this lane handles in iteration `it` (it is a compile-time unrolled index)
  __device__ __forceinline__ float4 wv(int it, int i, int v) const {
    if (it < IR) return w[it < IR ? it : 0][i];
    return lw[(min(row(it), NROWS - 1) - LROW0) * NV + min(v, NV - 1)];  // padding: as load()
  }
  __device__ __forceinline__ void load(const float* __restrict__ W, const float* __restrict__ b) {
    const int gl = (threadIdx.x & 63) % G;
    const float4* w4 = reinterpret_cast<const float4*>(W);
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int r = row(it);
      if (it < IR) {
#pragma unroll
        for (int i = 0; i < PL; ++i) {
          const int v = gl + i * G;
          // clamped, unconditional loads (a guarded load compiles to a branch + vmcnt(0) each): the
          // weights of padding rows / columns are never used (fwd stores only r < NROWS, v < NV;
          // bwd scales padding rows by dv = 0 and stores only v < NV)
          w[it < IR ? it : 0][i] = w4[min(r, NROWS - 1) * NV + min(v, NV - 1)];
        }
      }
      bias[it] = b[min(r, NROWS - 1)];
    }
  }
  template <bool RELU>
  __device__ __forceinline__ void fwd(const float* xin, float* out_lds, float* __restrict__ out_g) const {
    const int gl = (threadIdx.x & 63) % G;
    const float4* x4 = reinterpret_cast<const float4*>(xin);
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < PL; ++i) {
        const int v = gl + i * G;
        if (v < NV) {
          const float4 xv = x4[v], wq = wv(it, i, v);
          acc = fmaf(wq.x, xv.x, acc);
          acc = fmaf(wq.y, xv.y, acc);
          acc = fmaf(wq.z, xv.z, acc);
          acc = fmaf(wq.w, xv.w, acc);
        }
      }
      acc = group_reduce_last<G>(acc);  // DPP tree: valid in the group's last lane
      const int r = row(it);
      if (gl == G - 1 && r < NROWS) {
        float o = acc + bias[it];
        if (RELU) o = fmaxf(o, 0.f);
        out_lds[r] = o;
        if (out_g) out_g[r] = o;
      }
    }
  }
  // out[k] = mask(k) * sum_r d[r] W[r][k]; scratch >= SCRATCH floats. Ends with a barrier.
  __device__ __forceinline__ void bwd(const float* d, float* scratch, float* out_lds, float* __restrict__ out_g,
                                      const float* mask) const {
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
        const float4 wq = wv(it, i, v);
        acc.x = fmaf(dv[it], wq.x, acc.x);
        acc.y = fmaf(dv[it], wq.y, acc.y);
        acc.z = fmaf(dv[it], wq.z, acc.z);
        acc.w = fmaf(dv[it], wq.w, acc.w);
      }
      if (v < NV) reinterpret_cast<float4*>(scratch)[grp * NV + v] = acc;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < NCOLS; k += NT) {
      float sum = 0.f;
#pragma unroll 8
      for (int g = 0; g < RPI; ++g) sum += scratch[g * NCOLS + k];
      if (mask) sum = mask[k] > 0.f ? sum : 0.f;
      if (out_lds) out_lds[k] = sum;
      if (out_g) out_g[k] = sum;
    }
    __syncthreads();
  }
};

constexpr int cmax(int a, int b) { return a > b ? a : b; }

// ---------------------------------------------------------------------------
// K3: fc1 -> fc2 -> fc3 -> CE -> dgrad chain, one 1024-thread block per sample.
// ---------------------------------------------------------------------------
constexpr int kFcThreads = 1024;

// LDS of the fc chain (shared by K3 and the fused per-sample kernel)
template <class D, int NT, int IR1 = -1>
struct FcLds {
  using L1 = RegLinear<D::FLAT, D::F1, NT, IR1>;
  using L2 = RegLinear<D::F1, D::F2, NT>;
  using L3 = RegLinear<D::F2, D::NC, NT>;
  static constexpr int SCR = cmax(L1::SCRATCH, cmax(L2::SCRATCH, L3::SCRATCH));
  alignas(16) float sh1[D::F1];  // RegLinear reads its inputs as float4
  alignas(16) float sh2[D::F2];
  alignas(16) float sdl[64];
  alignas(16) float sdh2[D::F2];
  alignas(16) float sdh1[D::F1];
  alignas(16) float slog[64];
};

// fc1 -> fc2 -> fc3 (fwd, from `f` in LDS) -> softmax-CE -> dgrad chain for sample b, with
// the weights held in registers (l1..l3 loaded by the caller). Writes h1/h2/logits/dlogits/
// dh2/dh1/dflat of sample b to global (K5 reads them); dflat also to `dflat_lds` if given.
// Every path ends with a barrier.
template <class D, int NT, int IR1>
__device__ __forceinline__ void fc_chain(int mode, const LeNetPtrs& P, int b, int64_t tgt_pre, float inv_B,
                                         const typename FcLds<D, NT, IR1>::L1& l1,
                                         const typename FcLds<D, NT, IR1>::L2& l2,
                                         const typename FcLds<D, NT, IR1>::L3& l3, const float* f,
                                         FcLds<D, NT, IR1>& s, float* scratch, float* dflat_lds) {
  constexpr int FLAT = D::FLAT, F1 = D::F1, F2 = D::F2, NC = D::NC;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  float* sh1 = s.sh1;
  float* sh2 = s.sh2;
  float* sdl = s.sdl;
  float* sdh2 = s.sdh2;
  float* sdh1 = s.sdh1;
  float* slog = s.slog;
  if (mode & LENET_FWD) {
    l1.template fwd<true>(f, sh1, P.h1 + (int64_t)b * F1);
    __syncthreads();
    l2.template fwd<true>(sh1, sh2, P.h2 + (int64_t)b * F2);
    __syncthreads();
    l3.template fwd<false>(sh2, slog, P.logits + (int64_t)b * NC);
    __syncthreads();
  } else {
    if (t < F1) sh1[t] = P.h1[(int64_t)b * F1 + t];
    if (t < F2) sh2[t] = P.h2[(int64_t)b * F2 + t];
    if (t < NC) slog[t] = P.logits[(int64_t)b * NC + t];
    __syncthreads();
  }

  if (mode & LENET_CE) {
    if (wid == 0) {
      constexpr int GC = pow2_ge(NC);  // logits live in lanes [0, NC): reduce one DPP group, read its last lane
      const float z = lane < NC ? slog[lane] : -INFINITY;
      const float mx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(group_reduce_last<GC, true>(z)), GC - 1));
      const float e = lane < NC ? expf(z - mx) : 0.f;
      const float s = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(group_reduce_last<GC>(e)), GC - 1));
      const float lse = mx + logf(s);
      const int64_t tgt = tgt_pre;
      const bool valid = tgt >= 0 && tgt < NC;
      const unsigned long long am_mask = __ballot(lane < NC && z == mx);
      const int am = __ffsll((long long)am_mask) - 1;
      const float loss = valid ? lse - slog[valid ? tgt : 0] : 0.f;
      if (lane < NC) {
        const float dl = valid ? (e / s - (lane == tgt ? 1.f : 0.f)) * inv_B : 0.f;
        sdl[lane] = dl;
        if (mode & LENET_BWD) P.dlogits[(int64_t)b * NC + lane] = dl;
      }
      if (lane == 0 && P.stats) {
        if ((mode & LENET_STATS_DEFER) && P.cestat) {  // K4 adds them up in sample order (bitwise reproducible)
          P.cestat[2 * b] = (double)loss * (double)inv_B;
          P.cestat[2 * b + 1] = (am == tgt) ? (double)inv_B : 0.0;
        } else {  // evaluation / fused variant: no K4 follows
          atomicAdd(&P.stats[0], (double)loss * (double)inv_B);
          atomicAdd(&P.stats[1], (am == tgt) ? (double)inv_B : 0.0);
        }
      }
    }
    __syncthreads();
  } else if (mode & LENET_BWD) {
    if (t < NC) sdl[t] = P.dlogits[(int64_t)b * NC + t];
    __syncthreads();
  }

  if (mode & LENET_BWD) {
    l3.bwd(sdl, scratch, sdh2, P.dh2 + (int64_t)b * F2, sh2);
    l2.bwd(sdh2, scratch, sdh1, P.dh1 + (int64_t)b * F1, sh1);
    l1.bwd(sdh1, scratch, dflat_lds, P.dflat + (int64_t)b * FLAT, nullptr);
  }
}

template <class D>
__global__ __launch_bounds__(kFcThreads) void lenet_fc(int mode, LeNetPtrs P, float inv_B) {
  constexpr int FLAT = D::FLAT, NT = kFcThreads;
  using S = FcLds<D, NT>;
  const int b = blockIdx.x, t = threadIdx.x;
  __shared__ __attribute__((aligned(16))) float f[FLAT];
  __shared__ __attribute__((aligned(16))) S s;
  __shared__ __attribute__((aligned(16))) float scratch[S::SCR];

  // the label is needed only by the CE phase, but loading it now keeps it off the dependent chain
  const int64_t tgt_pre = (mode & LENET_CE) ? P.targets[b] : 0;
  typename S::L1 l1;
  typename S::L2 l2;
  typename S::L3 l3;
  l1.load(P.w3, P.b3);  // all weight loads in flight together
  l2.load(P.w4, P.b4);
  l3.load(P.w5, P.b5);
  if (mode & LENET_FWD) {
    const float4* src = reinterpret_cast<const float4*>(P.p2 + (int64_t)b * FLAT);
    if (t < FLAT / 4) reinterpret_cast<float4*>(f)[t] = src[t];
    __syncthreads();
  }
  fc_chain<D, NT, -1>(mode, P, b, tgt_pre, inv_B, l1, l2, l3, f, s, scratch, nullptr);
}

// ---------------------------------------------------------------------------
// weight-gradient helpers shared by K4 (fc roles) and K5
// ---------------------------------------------------------------------------
struct OptCtx {
  bool on;
  float lr, t;
};

// optimizer state of one float4 / scalar, loaded before the gradient is ready so the loads
// overlap the gradient computation instead of adding a dependent round trip after it
struct Opt4 {
  float4 p, a, c;
};
struct Opt1 {
  float p, a, c;
};
__device__ __forceinline__ Opt4 opt_prefetch4(const LeNetOpt& O, const OptCtx& oc, int64_t i) {
  Opt4 r{};
  if (!oc.on) return r;
  r.p = *reinterpret_cast<const float4*>(O.p + i);
  r.a = O.s1 ? *reinterpret_cast<const float4*>(O.s1 + i) : make_float4(0.f, 0.f, 0.f, 0.f);
  r.c = O.s2 ? *reinterpret_cast<const float4*>(O.s2 + i) : make_float4(0.f, 0.f, 0.f, 0.f);
  return r;
}
__device__ __forceinline__ Opt1 opt_prefetch1(const LeNetOpt& O, const OptCtx& oc, int64_t i) {
  Opt1 r{};
  if (!oc.on) return r;
  r.p = O.p[i];
  r.a = O.s1 ? O.s1[i] : 0.f;
  r.c = O.s2 ? O.s2[i] : 0.f;
  return r;
}
__device__ __forceinline__ void apply_pre4(const LeNetOpt& O, const OptCtx& oc, int64_t i, float4 g, Opt4 st) {
  *reinterpret_cast<float4*>(O.g + i) = g;  // keep the gradient visible (inspection / checkpoints)
  if (!oc.on) return;
  opt_update(O.h, oc.lr, oc.t, st.p.x, g.x, st.a.x, st.c.x);
  opt_update(O.h, oc.lr, oc.t, st.p.y, g.y, st.a.y, st.c.y);
  opt_update(O.h, oc.lr, oc.t, st.p.z, g.z, st.a.z, st.c.z);
  opt_update(O.h, oc.lr, oc.t, st.p.w, g.w, st.a.w, st.c.w);
  *reinterpret_cast<float4*>(O.p + i) = st.p;
  if (O.s1) *reinterpret_cast<float4*>(O.s1 + i) = st.a;
  if (O.s2) *reinterpret_cast<float4*>(O.s2 + i) = st.c;
}
__device__ __forceinline__ void apply_pre1(const LeNetOpt& O, const OptCtx& oc, int64_t i, float g, Opt1 st) {
  O.g[i] = g;
  if (!oc.on) return;
  opt_update(O.h, oc.lr, oc.t, st.p, g, st.a, st.c);
  O.p[i] = st.p;
  if (O.s1) O.s1[i] = st.a;
  if (O.s2) O.s2[i] = st.c;
}

template <int NCOLS>
__device__ __forceinline__ void fc_wgrad_block(int blk, int nrows, int B, const float* __restrict__ dY,
                                               const float* __restrict__ X, const LeNetOpt& O, int64_t offW,
                                               int64_t offb, const OptCtx& oc) {
  constexpr int NV = NCOLS / 4;
  const int item = blk * 256 + threadIdx.x;
  if (item >= nrows * NV) return;
  const int j = item / NV, v = item - j * NV;
  const Opt4 pw = opt_prefetch4(O, oc, offW + 4 * (int64_t)item);
  const Opt1 pb = v == 0 ? opt_prefetch1(O, oc, offb + j) : Opt1{};
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  float bacc = 0.f;
  const float4* x4 = reinterpret_cast<const float4*>(X);
#pragma unroll 4
  for (int b0 = 0; b0 < B; b0 += 8) {
    float d[8];
    float4 xv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {  // 16 independent loads in flight
      const int bb = b0 + u;
      const bool ok = bb < B;
      d[u] = ok ? dY[(int64_t)bb * nrows + j] : 0.f;
      xv[u] = ok ? x4[(int64_t)bb * NV + v] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      acc.x = fmaf(d[u], xv[u].x, acc.x);
      acc.y = fmaf(d[u], xv[u].y, acc.y);
      acc.z = fmaf(d[u], xv[u].z, acc.z);
      acc.w = fmaf(d[u], xv[u].w, acc.w);
      bacc += d[u];
    }
  }
  apply_pre4(O, oc, offW + 4 * (int64_t)item, acc, pw);
  if (v == 0) apply_pre1(O, oc, offb + j, bacc, pb);
}

// optimizer context of a weight-gradient launch: step counters / lr read from device memory
// (the last K5 block advances the counters, so every reader in a step sees the same values)
__device__ __forceinline__ OptCtx make_optctx(int mode, const LeNetOpt& O, const int64_t* ctrl) {
  OptCtx oc;
  oc.on = (mode & LENET_OPT) != 0;
  oc.lr = O.h.lr;
  oc.t = 1.f;
  if (oc.on) {
    const int64_t step = ctrl ? ctrl[0] : 0, sie = ctrl ? ctrl[1] : 0;
    oc.t = (float)(step + 1);
    if (O.lr_ptr) oc.lr = O.lr_ptr[O.lr_table ? sie : 0];
  }
  return oc;
}

// the fc weight-gradient roles (+ fused update): block `bf` of NB3 + NB4 + NB5
template <class D>
__device__ __forceinline__ void fc_wgrad_roles(int bf, int B, const LeNetPtrs& P, const LeNetOpt& O,
                                               const OptCtx& oc) {
  constexpr int F1 = D::F1, F2 = D::F2, NC = D::NC, FLAT = D::FLAT;
  constexpr int NB3 = (F1 * (FLAT / 4) + 255) / 256, NB4 = (F2 * (F1 / 4) + 255) / 256,
                NB5 = (NC * (F2 / 4) + 255) / 256;
  if (bf < NB3) {
    fc_wgrad_block<FLAT>(bf, F1, B, P.dh1, P.p2, O, O.off[4], O.off[5], oc);
  } else if ((bf -= NB3) < NB4) {
    fc_wgrad_block<F1>(bf, F2, B, P.dh2, P.h1, O, O.off[6], O.off[7], oc);
  } else if ((bf -= NB4) < NB5) {
    fc_wgrad_block<F2>(bf, NC, B, P.dlogits, P.h2, O, O.off[8], O.off[9], oc);
  }
}
template <class D>
constexpr int fc_wgrad_blocks() {
  return (D::F1 * (D::FLAT / 4) + 255) / 256 + (D::F2 * (D::F1 / 4) + 255) / 256 + (D::NC * (D::F2 / 4) + 255) / 256;
}

// ---------------------------------------------------------------------------
// K4: unpool2 (via arg-max) -> conv2 dgrad -> mask by pool1 arg-max liveness.
// Block (256 = 4 waves) per (sample, input channel); lane = 2x2 output patch of the
// 14x14 map, wave = quarter of the conv2 output channels (reduced through LDS in order).
// ---------------------------------------------------------------------------
//
// WG (the engine / autograd path): the conv weight gradients move here from K5. Everything they
// need per sample is at hand -- the masked conv1-output grad this kernel produces, the dense
// conv2-output grad image `dc` every block rebuilds from dflat, x[b] and p1[b, ic] -- so the grid
// gets a second half: blocks (b, ic) also reduce their sample's conv1 wgrad (oc = ic) after the
// dgrad, blocks (b, C1 + ic) compute the sample's conv2 wgrad for input channel ic instead of a
// dgrad. Both store per-(sample, channel) slabs; K5 only sums B slabs per weight in sample order.
// (The conv wgrads were K5's two longest roles: 11.5 / 9.2 us of a 12.8 us kernel.)
// ---------------------------------------------------------------------------
template <class D, bool WG>
__global__ __launch_bounds__(256) void lenet_conv2_dgrad(const float* __restrict__ dflat,
                                                         const uint8_t* __restrict__ i2,
                                                         const float* __restrict__ w2,
                                                         const uint8_t* __restrict__ i1, float* __restrict__ g1,
                                                         const float* __restrict__ x, const float* __restrict__ p1,
                                                         float* __restrict__ slab, int mode, LeNetPtrs P, LeNetOpt O,
                                                         const int64_t* __restrict__ ctrl, LeNetAug A, int stage_row,
                                                         int stats_row) {
  constexpr int C1 = D::C1, C2 = D::C2, FLAT = D::FLAT, NZ4 = C2 * 81, NS = (FLAT + 255) / 256;
  constexpr int W2N = C2 * 25 + C2;  // conv2 wgrad outputs of one input channel (+ the biases)
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wid = t >> 6;
  if ((int)blockIdx.y == stats_row) {
    // the step's loss / accuracy: per-sample terms (written by the CE) summed in a fixed order --
    // thread partials over a fixed stride, then a fixed xor tree -- so the epoch statistics are
    // bitwise reproducible (a per-sample atomicAdd orders the double sums by arrival). One block,
    // off the critical path (beside the dgrad blocks).
    if (b != 0) return;
    __shared__ double sred[2][4];
    const int B = (int)gridDim.x;
    double s0 = 0.0, s1 = 0.0;
    for (int i = t; i < B; i += 256) {
      s0 += P.cestat[2 * i];
      s1 += P.cestat[2 * i + 1];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      s0 += __shfl_xor(s0, o, 64);
      s1 += __shfl_xor(s1, o, 64);
    }
    if (lane == 0) {
      sred[0][wid] = s0;
      sred[1][wid] = s1;
    }
    __syncthreads();
    if (t == 0) {
      P.stats[0] += ((sred[0][0] + sred[0][1]) + sred[0][2]) + sred[0][3];
      P.stats[1] += ((sred[1][0] + sred[1][1]) + sred[1][2]) + sred[1][3];
    }
    return;
  }
  if ((int)blockIdx.y == stage_row) {
    // next-step input staging (off the step's critical path: runs beside the dgrad blocks).
    // ctrl still holds this step's counters here (K5 advances them after every K4 block is done),
    // so the next step reads position (ctrl[1] + 1) * stride + b -- exactly what its conv1 computes.
    int64_t pos = (A.ctrl[1] + 1) * A.batch_stride + b;
    if (pos >= A.perm_len) pos %= A.perm_len;
    int64_t idx = A.perm[pos];
    idx = idx < 0 ? 0 : (idx >= A.n ? A.n - 1 : idx);
    const int64_t tgt = P.dtargets ? P.dtargets[idx] : 0;
    if (t < 192)
      reinterpret_cast<uint4*>(P.stage + (int64_t)b * 3072)[t] = reinterpret_cast<const uint4*>(A.data + idx * 3072)[t];
    if (t == 0) {
      P.stage_meta[4 * b] = pos;
      P.stage_meta[4 * b + 1] = idx;
      P.stage_meta[4 * b + 2] = tgt;
      P.stage_meta[4 * b + 3] = 0;
    }
    return;
  }
  if (WG && (int)blockIdx.y >= 2 * C1) {  // fc wgrad (+ update) blocks: independent of the dgrad
    const int bf = ((int)blockIdx.y - 2 * C1) * (int)gridDim.x + b;
    if (bf < fc_wgrad_blocks<D>()) fc_wgrad_roles<D>(bf, (int)gridDim.x, P, O, make_optctx(mode, O, ctrl));
    return;
  }
  const bool w2role = WG && (int)blockIdx.y >= C1;
  const int ic = w2role ? (int)blockIdx.y - C1 : (int)blockIdx.y;
  __shared__ __attribute__((aligned(16))) float dc[C2 * 324];  // zero-padded dense conv2-output grad [C2][18][18]
  __shared__ __attribute__((aligned(16))) float4 red[4][64];
  // WG staging: x[b] [3][32][32] | p1[b, ic] rows padded to 16 (aliased: one role each), the
  // conv1-grad cells with their input offsets, the conv2 partials of 3 row groups
  __shared__ __attribute__((aligned(16))) float wx[WG ? 3 * 32 * 37 : 4];
  __shared__ float wg1[WG ? 196 : 1];
  __shared__ int wpos[WG ? 196 : 1];
  __shared__ float wred[WG ? 3 * W2N : 1];
  float4 xv[3];
  float pv[4];
  if constexpr (WG) {  // issued first: in flight across the dgrad / dc build below
    if (!w2role) {
#pragma unroll
      for (int i = 0; i < 3; ++i) xv[i] = reinterpret_cast<const float4*>(x + (int64_t)b * 3072)[t + 256 * i];
    } else if (t < 49) {
      const float* src = p1 + ((int64_t)b * C1 + ic) * 196 + 4 * t;
#pragma unroll
      for (int q = 0; q < 4; ++q) pv[q] = src[q];
    }
  }
  int kk[NS];
  float gg[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    const int e = t + i * 256;
    kk[i] = e < FLAT ? (int)i2[(int64_t)b * FLAT + e] : 4;
    gg[i] = e < FLAT ? dflat[(int64_t)b * FLAT + e] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < (NZ4 + 255) / 256; ++i)
    if (t + i * 256 < NZ4) reinterpret_cast<float4*>(dc)[t + i * 256] = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    const int e = t + i * 256, k = kk[i];
    if (k < 4) {
      const int o = e / 25, p = e - o * 25;
      const int cy = 2 * (p / 5) + (k >> 1), cx = 2 * (p % 5) + (k & 1);
      dc[o * 324 + (cy + 4) * 18 + cx + 4] = gg[i];
    }
  }
  if constexpr (WG) {
    if (w2role) {
      // conv2 wgrad of sample b, input channel ic: thread (oc, kh, row group) slides a 5-wide p1
      // window along x; kh == 0 threads also sum dc (the conv2 bias gradient, stored by ic == 0)
      float* wp = wx;  // [14][16]
      if (t < 49) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int e = 4 * t + q, r = e / 14;
          wp[r * 16 + e - r * 14] = pv[q];
        }
      }
      __syncthreads();
      float a2[5] = {0.f, 0.f, 0.f, 0.f, 0.f}, ab = 0.f;
      const int o2 = t % (C2 * 5), yg = t / (C2 * 5), oc = o2 / 5, kh = o2 - oc * 5;
      if (yg < 3) {
        const int y0 = yg == 0 ? 0 : 1 + 3 * yg, y1 = 4 + 3 * yg;  // rows 0-3, 4-6, 7-9
#pragma unroll 1
        for (int y = y0; y < y1; ++y) {
          const float* dr = dc + oc * 324 + (y + 4) * 18 + 4;
          const float* pr = wp + (y + kh) * 16;
          float win[14];
#pragma unroll
          for (int q = 0; q < 14; ++q) win[q] = pr[q];
#pragma unroll
          for (int xx = 0; xx < 10; ++xx) {
            const float dv = dr[xx];
            ab += dv;
#pragma unroll
            for (int kw = 0; kw < 5; ++kw) a2[kw] = fmaf(dv, win[xx + kw], a2[kw]);
          }
        }
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) wred[yg * W2N + oc * 25 + kh * 5 + kw] = a2[kw];
        if (kh == 0) wred[yg * W2N + C2 * 25 + oc] = ab;
      }
      __syncthreads();
      float* slb = slab + ((int64_t)b * C1 + ic) * kSlabStride + kSlab2Off;
      for (int e = t; e < C2 * 25 + (ic == 0 ? C2 : 0); e += 256)
        slb[e] = (wred[e] + wred[W2N + e]) + wred[2 * W2N + e];
      return;
    }
  }
  __syncthreads();
  float a00 = 0.f, a01 = 0.f, a10 = 0.f, a11 = 0.f;
  if (lane < 49) {
    const int by = lane / 7, bx = lane - by * 7, y0 = 2 * by, x0 = 2 * bx;
    constexpr int OPW = C2 / 4;
#pragma unroll 1
    for (int oo = 0; oo < OPW; ++oo) {
      const int o = wid * OPW + oo;
      const float* w = w2 + (o * C1 + ic) * 25;
      const float* d = dc + o * 324;
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        float in[6];
#pragma unroll
        for (int q = 0; q < 6; ++q) in[q] = d[(y0 + r) * 18 + x0 + q];
        if (r <= 4) {  // output row y0: kh = 4 - r
          const int kh = 4 - r;
#pragma unroll
          for (int kw = 0; kw < 5; ++kw) {
            const float wv = w[kh * 5 + kw];
            a00 = fmaf(wv, in[4 - kw], a00);
            a01 = fmaf(wv, in[5 - kw], a01);
          }
        }
        if (r >= 1) {  // output row y0+1: kh = 5 - r
          const int kh = 5 - r;
#pragma unroll
          for (int kw = 0; kw < 5; ++kw) {
            const float wv = w[kh * 5 + kw];
            a10 = fmaf(wv, in[4 - kw], a10);
            a11 = fmaf(wv, in[5 - kw], a11);
          }
        }
      }
    }
  }
  red[wid][lane] = make_float4(a00, a01, a10, a11);
  __syncthreads();
  if (t < 49) {
    float4 s = red[0][t];
#pragma unroll
    for (int w = 1; w < 4; ++w) {
      const float4 r = red[w][t];
      s.x += r.x;
      s.y += r.y;
      s.z += r.z;
      s.w += r.w;
    }
    const int by = t / 7, bx = t - by * 7, y0 = 2 * by, x0 = 2 * bx;
    const int64_t base = ((int64_t)(b * C1 + ic) * 14 + y0) * 14 + x0;
    const int k00 = i1[base], k01 = i1[base + 1], k10 = i1[base + 14], k11 = i1[base + 15];
    const float v00 = k00 < 4 ? s.x : 0.f, v01 = k01 < 4 ? s.y : 0.f, v10 = k10 < 4 ? s.z : 0.f,
                v11 = k11 < 4 ? s.w : 0.f;
    g1[base] = v00;
    g1[base + 1] = v01;
    g1[base + 14] = v10;
    g1[base + 15] = v11;
    if constexpr (WG) {  // conv1-output grad cell c -> (value, offset of its arg-max in a 32x32 plane)
      const int cells[4] = {y0 * 14 + x0, y0 * 14 + x0 + 1, (y0 + 1) * 14 + x0, (y0 + 1) * 14 + x0 + 1};
      const int ks[4] = {k00, k01, k10, k11};
      const float vs[4] = {v00, v01, v10, v11};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = cells[q], k = ks[q] < 4 ? ks[q] : 0, py = c / 14, px = c - py * 14;
        wg1[c] = vs[q];
        wpos[c] = (2 * py + (k >> 1)) * 37 + 2 * px + (k & 1);  // row stride of the staged x (XR below)
      }
    }
  }
  if constexpr (WG) {
    // conv1 wgrad of sample b, output channel ic: dW1[ic, c, kh, kw] (+ bias) over the 196 pooled
    // cells in 3 slices (lane = tap: the cell's grad / offset are LDS broadcasts). x[b] is staged
    // with a 37-float row stride so the 5 kh rows of a tap window fall in disjoint bank ranges
    // (with 32 they alias every 2 rows: 9-way conflicts).
    constexpr int XR = 37, XC = 32 * XR;  // (wpos above is built with the same 37)
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int e = 4 * (t + 256 * i), c = e >> 10, r = (e >> 5) & 31, col = e & 31;
      float* d = wx + c * XC + r * XR + col;
      d[0] = xv[i].x;
      d[1] = xv[i].y;
      d[2] = xv[i].z;
      d[3] = xv[i].w;
    }
    __syncthreads();
    float acc = 0.f;
    const int tap = t % kTaps1, sl = t / kTaps1;
    if (sl < 3) {
      if (tap < 75) {
        const int c = tap / 25, kh = (tap % 25) / 5, kw = tap % 5;
        const float* xc = wx + c * XC + kh * XR + kw;
#pragma unroll 7
        for (int e = sl; e < 196; e += 3) acc = fmaf(wg1[e], xc[wpos[e]], acc);
      } else {
#pragma unroll 7
        for (int e = sl; e < 196; e += 3) acc += wg1[e];
      }
    }
    float* r1 = reinterpret_cast<float*>(red);
    if (sl < 3) r1[sl * kTaps1 + tap] = acc;
    __syncthreads();
    if (t < kTaps1) slab[((int64_t)b * C1 + ic) * kSlabStride + t] = r1[t] + r1[kTaps1 + t] + r1[2 * kTaps1 + t];
  }
}

// ---------------------------------------------------------------------------
// KF: K1..K4 fused -- the whole per-sample chain in ONE 1024-thread block per sample:
//   [augment] -> conv1+ReLU+pool -> conv2+ReLU+pool -> fc1/fc2/fc3 -> softmax-CE
//   -> fc dgrad chain -> unpool2 -> conv2 dgrad -> pool1 liveness mask.
// Nothing in that chain crosses samples (only the weight-gradient batch sums of K5 do), so the
// four launches -- each a launch boundary plus a global round trip of its inputs -- become one,
// and every intermediate stays in LDS. One CU per sample means the phases must run near the
// CU's VALU rate, so each is register-tiled (a thread owns a row strip: every LDS operand
// read feeds 4-14 FMAs) over row-padded, 16-byte-aligned LDS images read with ds_read_b128,
// and split reductions (input- / output-channel groups, row pairs) are combined across the
// lanes of a quad with DPP (VALU, no LDS round trip) in a fixed order.
//
// The phases follow `mode` (FWD: conv1..fc3 [+CE]; BWD: fc dgrad .. conv2 dgrad, reading the
// forward state from global when FWD is absent), so the autograd path (FWD, then BWD with a
// given dlogits) runs the same arithmetic as the fused engine step. fc1's weights do not fit
// the register budget of 1024 threads beside the conv phases: the first kFusedFc1Regs row
// iterations stay in registers, the rest are LDS-DMA'd (global_load_lds) at entry.
// Writes exactly the tensors K5 reads (x, p1, i1, p2, i2, h1, h2, logits, dlogits, dh2, dh1,
// dflat, g1).
// ---------------------------------------------------------------------------
constexpr int kFusedThreads = 1024;
constexpr int kFusedFc1Regs = 4;  // fc1 row-iterations kept in registers; the rest of W3 is DMA'd to LDS
constexpr int kXs = 36;           // padded row stride (floats) of the input image [3][32][kXs]
constexpr int kP1s = 16;          // padded row stride of the pooled conv1 map [C1][14][kP1s]
constexpr int kDcs = 20;          // padded row stride of the zero-padded conv2-output grad [C2][18][kDcs]

// quad lane exchanges (DPP quad_perm: a VALU operand modifier, no LDS crossbar round trip)
__device__ __forceinline__ float quad_xor1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float quad_xor2(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
}

// max-pool of a 2x2 window (k = 0..3 in row-major window order, first max wins) + ReLU;
// the arg-max code is 4 for a dead cell (as K1/K2)
__device__ __forceinline__ void pool4(float a00, float a01, float a10, float a11, float& pv, uint8_t& iv) {
  float m = a00;
  int k = 0;
  if (a01 > m) { m = a01; k = 1; }
  if (a10 > m) { m = a10; k = 2; }
  if (a11 > m) { m = a11; k = 3; }
  pv = m > 0.f ? m : 0.f;
  iv = m > 0.f ? (uint8_t)k : (uint8_t)4;
}

template <class D>
struct FusedLds {
  using S = FcLds<D, kFusedThreads, kFusedFc1Regs>;
  static constexpr int W3L = S::L1::LDS_FLOATS > 0 ? S::L1::LDS_FLOATS : 4;
  static constexpr int XS = 3 * 32 * kXs;         // padded input image
  static constexpr int U0 = XS + 192 * 4;          // + the raw uint8 image (phases 0-1)
  static constexpr int DC = D::C2 * 18 * kDcs;     // phases 5-6
  static constexpr int U = cmax(U0, cmax(S::SCR, DC));
  alignas(16) float u[U];  // image -> fc dgrad scratch -> dc (phases never overlap; barriers between)
  alignas(16) float p1[D::C1 * 14 * kP1s];
  alignas(16) float f[D::FLAT];
  alignas(16) float df[D::FLAT];
  alignas(16) S s;
  alignas(16) float w3l[W3L];  // fc1 rows >= L1::LROW0, filled by global_load_lds
  float w1[D::C1 * 75], b1[D::C1], w2[D::C2 * D::C1 * 25], b2[D::C2];
  uint8_t i1[D::C1 * 196], i2[D::FLAT];
};

template <class D>
__global__ __launch_bounds__(kFusedThreads) void lenet_sample_fused(int mode, LeNetPtrs P, LeNetAug aug,
                                                                    float inv_B) {
  constexpr int C1 = D::C1, C2 = D::C2, FLAT = D::FLAT, NT = kFusedThreads;
  static_assert(C1 % 2 == 0 && C2 % 4 == 0 && C1 * 98 <= NT && C2 * 20 <= NT && C1 * 56 <= NT,
                "fused LeNet geometry");
  using S = typename FusedLds<D>::S;
  const int b = blockIdx.x, t = threadIdx.x, wid = t >> 6;
  const bool fwd = (mode & LENET_FWD) != 0, bwd = (mode & LENET_BWD) != 0;
  // LENET_FROM_P1 (the default engine path): K1 already ran augment + conv1 for the whole batch;
  // this kernel starts from p1 in global (conv2 -> fc chain -> CE -> fc dgrad) and stops there
  // (K4 does unpool2 / conv2 dgrad / the conv wgrads): K2 + K3 as one launch, with fc1's weights
  // streaming into registers while conv2 computes.
  const bool from_p1 = (mode & LENET_FROM_P1) != 0;
  __shared__ __attribute__((aligned(16))) FusedLds<D> L;
  float* xs = L.u;
  uint4* rawimg = reinterpret_cast<uint4*>(L.u + FusedLds<D>::XS);
  // LENET_TRACE: per-phase cycle stamps of block 0 (phase profiling; K5 is not launched then)
  const bool trace = kFp32TraceBuild && (mode & LENET_TRACE) && b == 0 && t == 0;
  auto stamp = [&](int k) {  // pinned in place: s_memtime can otherwise float across whole phases
    if constexpr (!kFp32TraceBuild) return;
    if (!(mode & LENET_TRACE)) return;
    __builtin_amdgcn_sched_barrier(0);
    unsigned long long c, w;
    asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(c), "=s"(w)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    if (trace) {
      reinterpret_cast<unsigned long long*>(P.slab1)[k] = c;
      if (k == 0 || k == 7) reinterpret_cast<unsigned long long*>(P.slab1)[8 + k / 7] = w;  // 100 MHz
    }
  };
  stamp(0);

  // ---- phase 0: every load in flight together. Independent loads first and branch-free
  // (clamped indices: a guarded load compiles to a branch + vmcnt(0) per element), then the
  // sample-index chain (ctrl -> perm -> image, the longest dependent chain of the kernel), then
  // the LDS-DMA of fc1's LDS-resident rows, which must not sit in front of a chain wait.
  constexpr int NW2 = (C2 * C1 * 25 + NT - 1) / NT;
  static_assert(C1 * 75 <= NT && C1 * 196 <= 2 * NT, "one conv1 filter element / two i1 bytes per thread");
  const float w1r = P.w1[min(t, C1 * 75 - 1)];
  float w2r[NW2];
#pragma unroll
  for (int j = 0; j < NW2; ++j) w2r[j] = P.w2[min(t + j * NT, C2 * C1 * 25 - 1)];
  const float b1r = P.b1[min(t, C1 - 1)], b2r = P.b2[min(t, C2 - 1)];
  typename S::L1 l1;
  typename S::L2 l2;
  typename S::L3 l3;
  l2.load(P.w4, P.b4);
  l3.load(P.w5, P.b5);
  int64_t idx = 0;
  bool fl = false;
  int ci = 0, cj = 0;
  uint4 raw = make_uint4(0u, 0u, 0u, 0u);
  float4 xin = make_float4(0.f, 0.f, 0.f, 0.f);
  uint8_t i1r[2] = {0, 0}, i2r = 0;
  float p1r[2] = {0.f, 0.f};
  if (fwd && from_p1) {
#pragma unroll
    for (int j = 0; j < 2; ++j) p1r[j] = P.p1[(int64_t)b * C1 * 196 + min(t + j * NT, C1 * 196 - 1)];
  } else if (fwd) {
    if (aug.data) {
      const int64_t step = aug.ctrl[0], sie = aug.ctrl[1];
      int64_t pos = sie * aug.batch_stride + b;
      if (pos >= aug.perm_len) pos %= aug.perm_len;
      idx = aug.perm[pos];
      idx = idx < 0 ? 0 : (idx >= aug.n ? aug.n - 1 : idx);
      const uint64_t h = mix64(mix64(aug.seed + (uint64_t)step) ^ (uint64_t)pos);
      const int span = 2 * aug.pad + 1;
      ci = aug.pad ? (int)(h % span) : 0;
      cj = aug.pad ? (int)((h >> 20) % span) : 0;
      fl = aug.flip && ((h >> 40) & 1);
      raw = reinterpret_cast<const uint4*>(aug.data + idx * 3072)[min(t, 191)];
    } else {
      xin = reinterpret_cast<const float4*>(P.x + (int64_t)b * 3072)[min(t, 767)];
    }
  } else if (bwd) {  // backward only: the forward state comes from global
    i1r[0] = P.i1[(int64_t)b * C1 * 196 + min(t, C1 * 196 - 1)];
    i1r[1] = P.i1[(int64_t)b * C1 * 196 + min(t + NT, C1 * 196 - 1)];
    i2r = P.i2[(int64_t)b * FLAT + min(t, FLAT - 1)];
  }
  int64_t tgt_pre = 0;
  if (mode & LENET_CE) tgt_pre = (fwd && aug.data && !from_p1) ? P.dtargets[idx] : P.targets[b];
  if constexpr (S::L1::LDS_FLOATS > 0) {  // fc1 rows beyond the register budget: LDS-DMA, no VGPRs
    constexpr int CH = S::L1::LDS_FLOATS / 4;  // 16-byte chunks
    const float* src = P.w3 + S::L1::LROW0 * FLAT;
#pragma unroll
    for (int i = 0; i < (CH + NT - 1) / NT; ++i) {
      const int e = i * NT + t;
      if (e < CH)
        __builtin_amdgcn_global_load_lds((const void*)(src + 4 * e), (lds_void_t*)(L.w3l + 4 * (i * NT + wid * 64)),
                                         16, 0, 0);
    }
  }
  l1.lw = reinterpret_cast<const float4*>(L.w3l);
  if (t < C1 * 75) L.w1[t] = w1r;
#pragma unroll
  for (int j = 0; j < NW2; ++j)
    if (t + j * NT < C2 * C1 * 25) L.w2[t + j * NT] = w2r[j];
  if (t < C1) L.b1[t] = b1r;
  if (t < C2) L.b2[t] = b2r;
  if (fwd && from_p1) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int e = t + j * NT;
      if (e < C1 * 196) {
        const int ic = e / 196, r = e - ic * 196, y = r / 14;
        L.p1[(ic * 14 + y) * kP1s + r - y * 14] = p1r[j];
      }
    }
  } else if (fwd) {
    if (aug.data) {
      if (t < 192) rawimg[t] = raw;
    } else if (t < 768) {  // [3*32 rows][8 float4] -> padded rows
      *reinterpret_cast<float4*>(xs + (t >> 3) * kXs + (t & 7) * 4) = xin;
    }
  } else if (bwd) {
    if (t < C1 * 196) L.i1[t] = i1r[0];
    if (t + NT < C1 * 196) L.i1[t + NT] = i1r[1];
    if (t < FLAT) L.i2[t] = i2r;
  }
  __syncthreads();

  stamp(1);
  // ---- phase 1: RandomCrop(pad) + HFlip + Normalize from the staged uint8 image
  if (fwd && aug.data && !from_p1) {
    const uint8_t* img = reinterpret_cast<const uint8_t*>(rawimg);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int e = t + i * NT;
      const int c = e >> 10, y = (e >> 5) & 31, xx = e & 31;
      const int sx = fl ? 31 - xx : xx;
      const int r = y + ci - aug.pad, q = sx + cj - aug.pad;
      const bool in = (unsigned)r < 32u && (unsigned)q < 32u;
      const float u = in ? (float)img[(r * 32 + q) * 3 + c] : 0.f;
      const float v = (u / 255.f - aug.mean[c]) / aug.std[c];
      xs[(c * 32 + y) * kXs + xx] = v;  // the raw image is a disjoint part of L.u
      P.x[(int64_t)b * 3072 + e] = v;
    }
    if (t == 0 && P.targets) P.targets[b] = tgt_pre;
    __syncthreads();
  }

  stamp(2);
  // ---- phase 2: conv1 + bias + ReLU + maxpool2. Thread = (oc, pooled row, 2 pooled columns):
  // a 2x4 conv-output strip, input rows read as 2 x b128.
  if (fwd && !from_p1 && t < C1 * 98) {
    const int oc = t / 98, rem = t - oc * 98, py = rem / 7, pxg = rem - py * 7, y0 = 2 * py, x0 = 4 * pxg;
    const float bias = L.b1[oc];
    float acc[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[j][c] = bias;
#pragma unroll
    for (int ic = 0; ic < 3; ++ic) {
      const float* wk = L.w1 + oc * 75 + ic * 25;
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        const float* row = xs + (ic * 32 + y0 + r) * kXs + x0;
        const float4 lo = *reinterpret_cast<const float4*>(row), hi = *reinterpret_cast<const float4*>(row + 4);
        const float in[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int kh = r - j;
          if (kh < 0 || kh > 4) continue;
#pragma unroll
          for (int kw = 0; kw < 5; ++kw) {
            const float wv = wk[kh * 5 + kw];
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[j][c] = fmaf(wv, in[c + kw], acc[j][c]);
          }
        }
      }
    }
    float pv[2];
    uint8_t iv[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) pool4(acc[0][2 * q], acc[0][2 * q + 1], acc[1][2 * q], acc[1][2 * q + 1], pv[q], iv[q]);
    *reinterpret_cast<float2*>(L.p1 + (oc * 14 + py) * kP1s + 2 * pxg) = make_float2(pv[0], pv[1]);
    const int o = oc * 196 + py * 14 + 2 * pxg;
    L.i1[o] = iv[0];
    L.i1[o + 1] = iv[1];
    *reinterpret_cast<float2*>(P.p1 + (int64_t)b * C1 * 196 + o) = make_float2(pv[0], pv[1]);
    P.i1[(int64_t)b * C1 * 196 + o] = iv[0];
    P.i1[(int64_t)b * C1 * 196 + o + 1] = iv[1];
  }
  if (fwd && !from_p1) __syncthreads();

  stamp(3);
  // ---- phase 3: conv2 + bias + ReLU + maxpool2 -> flatten. Quad = (oc, pooled row), lane bit 0 =
  // input-channel half, bit 1 = conv row of the pair; a lane computes a 10-wide conv row over
  // its C1/2 channels; halves summed, then rows pooled, across the quad (DPP).
  // (fc1's register weights are loaded here, not at entry: held through conv1 they spill)
  l1.load(P.w3, P.b3);
  if (fwd && t < C2 * 20) {
    const int icg = t & 1, ry = (t >> 1) & 1, rest = t >> 2, oc = rest / 5, py = rest - oc * 5;
    const int y = 2 * py + ry;
    float acc[10];
#pragma unroll
    for (int c = 0; c < 10; ++c) acc[c] = 0.f;
#pragma unroll
    for (int icc = 0; icc < C1 / 2; ++icc) {
      const int ic = icg * (C1 / 2) + icc;
      const float* wk = L.w2 + (oc * C1 + ic) * 25;
#pragma unroll
      for (int kh = 0; kh < 5; ++kh) {
        const float4* row = reinterpret_cast<const float4*>(L.p1 + (ic * 14 + y + kh) * kP1s);
        const float4 v0 = row[0], v1 = row[1], v2 = row[2], v3 = row[3];
        const float in[16] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w,
                              v2.x, v2.y, v2.z, v2.w, v3.x, v3.y, v3.z, v3.w};
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) {
          const float wv = wk[kh * 5 + kw];
#pragma unroll
          for (int c = 0; c < 10; ++c) acc[c] = fmaf(wv, in[c + kw], acc[c]);
        }
      }
    }
    const float bias = L.b2[oc];
    float s[10];
#pragma unroll
    for (int c = 0; c < 10; ++c) {  // (first half + second half) + bias, identical in both lanes
      const float o = quad_xor1(acc[c]);
      s[c] = (icg ? o + acc[c] : acc[c] + o) + bias;
    }
#pragma unroll
    for (int pc = 0; pc < 5; ++pc) {
      const float n0 = quad_xor2(s[2 * pc]), n1 = quad_xor2(s[2 * pc + 1]);  // the other conv row
      if (t & 3) continue;  // lane (ry 0, icg 0) owns the pooled row
      float pv;
      uint8_t iv;
      pool4(s[2 * pc], s[2 * pc + 1], n0, n1, pv, iv);
      const int o = oc * 25 + py * 5 + pc;
      L.f[o] = pv;
      L.i2[o] = iv;
      P.p2[(int64_t)b * FLAT + o] = pv;
      P.i2[(int64_t)b * FLAT + o] = iv;
    }
  }
  __syncthreads();

  stamp(4);
  // ---- phase 4: fc chain + CE (+ fc dgrad -> dflat); scratch aliases the (dead) image
  fc_chain<D, NT, kFusedFc1Regs>(mode, P, b, tgt_pre, inv_B, l1, l2, l3, L.f, L.s, L.u, L.df);
  if (!bwd || from_p1) return;

  stamp(5);
  // ---- phase 5: unpool2 -> dense zero-padded conv2-output grad (aliases the dead scratch)
  float* dc = L.u;
  for (int e = t; e < C2 * 18 * kDcs; e += NT) {
    const int o = e / (18 * kDcs), r = e - o * (18 * kDcs), cy = r / kDcs - 4, cx = r % kDcs - 4;
    float v = 0.f;
    if ((unsigned)cy < 10u && (unsigned)cx < 10u) {
      const int pp = o * 25 + (cy >> 1) * 5 + (cx >> 1);
      v = L.i2[pp] == (uint8_t)(((cy & 1) << 1) | (cx & 1)) ? L.df[pp] : 0.f;
    }
    dc[e] = v;
  }
  __syncthreads();

  stamp(6);
  // ---- phase 6: conv2 dgrad -> pool1 liveness mask -> g1. Quad = (input channel, output row),
  // lane = quarter of the output channels; a lane computes the 14-wide row over its C2/4
  // channels, the quarters are summed across the quad (DPP, same order in every lane).
  if (t < C1 * 56) {
    const int og = t & 3, rest = t >> 2, ic = rest / 14, y = rest - ic * 14;
    float acc[14];
#pragma unroll
    for (int x = 0; x < 14; ++x) acc[x] = 0.f;
#pragma unroll
    for (int oo = 0; oo < C2 / 4; ++oo) {
      const int o = og * (C2 / 4) + oo;
      const float* wk = L.w2 + (o * C1 + ic) * 25;
#pragma unroll
      for (int r = 0; r < 5; ++r) {  // padded input row y + r pairs with kernel row kh = 4 - r
        const float4* row = reinterpret_cast<const float4*>(dc + (o * 18 + y + r) * kDcs);
        const float4 v0 = row[0], v1 = row[1], v2 = row[2], v3 = row[3], v4 = row[4];
        const float in[20] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w, v2.x, v2.y,
                              v2.z, v2.w, v3.x, v3.y, v3.z, v3.w, v4.x, v4.y, v4.z, v4.w};
        const int kh = 4 - r;
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) {
          const float wv = wk[kh * 5 + kw];
#pragma unroll
          for (int x = 0; x < 14; ++x) acc[x] = fmaf(wv, in[x + 4 - kw], acc[x]);
        }
      }
    }
#pragma unroll
    for (int x = 0; x < 14; ++x) {
      const float s1 = acc[x] + quad_xor1(acc[x]);  // commutative steps: every lane gets the same sum
      acc[x] = s1 + quad_xor2(s1);
    }
    float* g = P.g1 + (int64_t)b * C1 * 196 + ic * 196 + y * 14;
    const uint8_t* m = L.i1 + ic * 196 + y * 14;
#pragma unroll
    for (int x = 0; x < 14; ++x)
      if ((x & 3) == og) g[x] = m[x] < 4 ? acc[x] : 0.f;
  }
  if (kFp32TraceBuild && (mode & LENET_TRACE)) {
    __syncthreads();
    stamp(7);
  }
}

// ---------------------------------------------------------------------------
// K5: all weight gradients (+ the fused optimizer update when single-process),
// role-split over blockIdx.x:
//   [0, ceil(B/4)*C1)       conv1 wgrad partial for (4-sample group, oc) -> slab1[g][oc][76]; the
//                           LAST arriving block of each oc reduces its ceil(B/4) slabs (fixed
//                           order, one round of loads) into the final grad (+ update)
//   [.., + C2*C1)           conv2 wgrad for (oc, ic) over the whole batch (+ bias when ic == 0)
//   [.., + nb3 + nb4 + nb5) fc wgrads (+ bias), one float4 of a weight row per thread
// The last block of the whole launch advances the device step counters.
//
// Cross-workgroup hand-off (cdna_hip_programming.md Guideline 16 R1 / §5 split-K, write-through
// form): slabs are line-disjoint (512 B each) and stored write-through (sc1); every storing
// wave drains (s_waitcnt vmcnt(0)), barrier, then ONE relaxed agent-scope ticket add; the
// block that draws the last ticket reads every slab with sc1 loads. No block ever
// waits on another, so there is no residency requirement and nothing can hang; the
// last arriver resets its counter for the next launch (zeroed once at allocation).
// ---------------------------------------------------------------------------
constexpr int kWgChunk = 32;  // samples staged per LDS pass in the conv2 wgrad role


template <class D>
__global__ __launch_bounds__(256) void lenet_wgrad(int mode, LeNetPtrs P, LeNetOpt O, int B,
                                                   int64_t* __restrict__ ctrl) {
  constexpr int C1 = D::C1, C2 = D::C2, F1 = D::F1, F2 = D::F2, NC = D::NC, FLAT = D::FLAT;
  constexpr int NB3 = (F1 * (FLAT / 4) + 255) / 256, NB4 = (F2 * (F1 / 4) + 255) / 256,
                NB5 = (NC * (F2 / 4) + 255) / 256;
  __shared__ __attribute__((aligned(16))) float lds[kSpb1 * (3072 + 2 * 196) + 3 * kTaps1 + 4 > 8192
                                                        ? kSpb1 * (3072 + 2 * 196) + 3 * kTaps1 + 4
                                                        : 8192];
  const int nA = (B + kSpb1 - 1) / kSpb1 * C1;
  int blk = blockIdx.x;
  const int t = threadIdx.x;
  // The step counters are read by every block here and advanced by the last block of the launch.
  const OptCtx oc = make_optctx(mode, O, ctrl);
  // K4WG: K4 left per-(sample, channel) conv wgrad slabs; the conv roles only reduce them over
  // the batch in sample order (one output per thread) -- the fc roles keep their block ids
  constexpr int NR1 = (C1 * kTaps1 + 255) / 256, NR2 = (C2 * C1 * 25 + C2 + 255) / 256;
  if (mode & LENET_K4WG) {
    if (blk < NR1 + NR2) {
      const bool c1r = blk < NR1;
      const int o = (c1r ? blk : blk - NR1) * 256 + t;
      const int nout = c1r ? C1 * kTaps1 : C2 * C1 * 25 + C2;
      if (o < nout) {
        int64_t src, dst;
        if (c1r) {
          const int ocn = o / kTaps1, tap = o - ocn * kTaps1;
          src = (int64_t)ocn * kSlabStride + tap;
          dst = tap < 75 ? O.off[0] + ocn * 75 + tap : O.off[1] + ocn;
        } else if (o < C2 * C1 * 25) {
          const int ocn = o / (C1 * 25), icn = (o / 25) % C1, tap = o % 25;
          src = (int64_t)icn * kSlabStride + kSlab2Off + ocn * 25 + tap;
          dst = O.off[2] + o;
        } else {
          src = kSlab2Off + C2 * 25 + (o - C2 * C1 * 25);  // ic == 0 slabs hold the bias sums
          dst = O.off[3] + (o - C2 * C1 * 25);
        }
        const Opt1 pst = opt_prefetch1(O, oc, dst);
        const int64_t sstride = (int64_t)C1 * kSlabStride;
        float g = 0.f;  // all 32 loads of a batch chunk in flight (clamped, branch-free), summed in order
        for (int b0 = 0; b0 < B; b0 += 32) {
          float v[32];
#pragma unroll
          for (int u = 0; u < 32; ++u) v[u] = P.slab1[min(b0 + u, B - 1) * sstride + src];
#pragma unroll
          for (int u = 0; u < 32; ++u) g += b0 + u < B ? v[u] : 0.f;
        }
        apply_pre1(O, oc, dst, g, pst);
      }
      blk = -1;  // done: skip the role dispatch below
    } else {
      blk = blk - NR1 - NR2 + nA + C2 * C1;  // fc roles
    }
  }
  // LENET_SKIP_* (profiling only, MLT_LENET_WGRAD_SKIP): drop a role to time the others
  const int role = blk < nA ? 0 : (blk < nA + C2 * C1 ? 1 : 2);
  if (blk < 0 || ((mode >> (9 + role)) & 1)) {
  } else if (blk < nA) {
    // conv1: dW1[oc, ic, kh, kw] partial over kSpb1 samples x 196 pooled cells.
    const int bg = blk / C1, ocn = blk - bg * C1, nbg = (B + kSpb1 - 1) / kSpb1;
    const Opt1 pst = t < kTaps1 ? opt_prefetch1(O, oc, t < 75 ? O.off[0] + ocn * 75 + t : O.off[1] + ocn) : Opt1{};
    float* xs = lds;                                                // [kSpb1][3][32][32]
    float* gs = lds + kSpb1 * 3072;                                 // [kSpb1][196]
    int* pos = reinterpret_cast<int*>(gs + kSpb1 * 196);            // [kSpb1][196] cy*32+cx
    float* red = reinterpret_cast<float*>(pos + kSpb1 * 196);       // [3][76]
    int* flag = reinterpret_cast<int*>(red + 3 * kTaps1);
    float4 xv[kSpb1][3];
    float gv[kSpb1];
    int kv[kSpb1];
#pragma unroll
    for (int j = 0; j < kSpb1; ++j) {  // all loads of the block's samples in flight together
      const int b = bg * kSpb1 + j;
      const bool ok = b < B;
      const float4* src = reinterpret_cast<const float4*>(P.x + (int64_t)(ok ? b : 0) * 3072);
#pragma unroll
      for (int i = 0; i < 3; ++i) xv[j][i] = ok ? src[t + i * 256] : make_float4(0.f, 0.f, 0.f, 0.f);
      gv[j] = 0.f;
      kv[j] = 4;
      if (ok && t < 196) {
        const int64_t o = (int64_t)(b * C1 + ocn) * 196 + t;
        gv[j] = P.g1[o];
        kv[j] = P.i1[o];
      }
    }
#pragma unroll
    for (int j = 0; j < kSpb1; ++j) {
#pragma unroll
      for (int i = 0; i < 3; ++i) reinterpret_cast<float4*>(xs + j * 3072)[t + i * 256] = xv[j][i];
      if (t < 196) {
        const int k = kv[j] < 4 ? kv[j] : 0;
        const int py = t / 14, px = t - py * 14;
        gs[j * 196 + t] = kv[j] < 4 ? gv[j] : 0.f;  // dead cells (and padding samples) add nothing
        pos[j * 196 + t] = (2 * py + (k >> 1)) * 32 + 2 * px + (k & 1);
      }
    }
    __syncthreads();
    if (t < 3 * kTaps1) {
      const int tap = t % kTaps1, s = t / kTaps1;
      float acc = 0.f;
      if (tap < 75) {
        const int ic = tap / 25, kh = (tap % 25) / 5, kw = tap % 5;
#pragma unroll
        for (int j = 0; j < kSpb1; ++j) {
          const float* xc = xs + j * 3072 + ic * 1024 + kh * 32 + kw;
#pragma unroll 8
          for (int c = s; c < 196; c += 3) acc = fmaf(gs[j * 196 + c], xc[pos[j * 196 + c]], acc);
        }
      } else {
#pragma unroll
        for (int j = 0; j < kSpb1; ++j)
#pragma unroll 8
          for (int c = s; c < 196; c += 3) acc += gs[j * 196 + c];
      }
      red[s * kTaps1 + tap] = acc;
    }
    __syncthreads();
    // Write-through (sc1) slab stores: the reducer on any XCD reads them from memory with sc1
    // loads, so neither an agent release nor an acquire fence is needed (Guideline 16, R1).
    if (t < kTaps1)
      __hip_atomic_store(&P.slab1[(int64_t)(bg * C1 + ocn) * kSlabStride + t],
                         red[t] + red[kTaps1 + t] + red[2 * kTaps1 + t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
    __syncthreads();
    if (t == 0) {
      const unsigned prev = __hip_atomic_fetch_add(&P.counters[ocn], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == (unsigned)(nbg - 1);
      if (last) __hip_atomic_store(&P.counters[ocn], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last;
    }
    __syncthreads();
    if (*flag) {
      // reduce the slabs of this oc in a fixed order (bitwise reproducible); sc1 loads only
      if (t < 3 * kTaps1) {
        const int tap = t % kTaps1, s = t / kTaps1;
        float acc = 0.f;
        for (int b0 = s; b0 < nbg; b0 += 3 * 8) {
          float v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int bb = b0 + 3 * u;
            v[u] = bb < nbg ? __hip_atomic_load(&P.slab1[(int64_t)(bb * C1 + ocn) * kSlabStride + tap], __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT)
                            : 0.f;
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) acc += v[u];
        }
        red[s * kTaps1 + tap] = acc;
      }
      __syncthreads();
      if (t < kTaps1) {
        const float g = red[t] + red[kTaps1 + t] + red[2 * kTaps1 + t];
        apply_pre1(O, oc, t < 75 ? O.off[0] + ocn * 75 + t : O.off[1] + ocn, g, pst);
      }
    }
  } else if (blk < nA + C2 * C1) {
    // conv2: dW2[oc, ic, :, :] over the batch, samples staged through LDS in chunks.
    const int b2 = blk - nA;
    const int ocn = b2 / C1, ic = b2 - ocn * C1;
    float* ps = lds;                                   // [CH][196]
    float* gs = lds + kWgChunk * 196;                  // [CH][25]
    int* pos = reinterpret_cast<int*>(gs + kWgChunk * 25);  // [CH][25] bb*196 + cy*14 + cx
    float* red = gs + 2 * kWgChunk * 25;               // [9][26]
    constexpr int NT = 26;                             // 25 taps + bias
    const int tap = t % NT, s = t / NT;                // 9 slices (234 threads)
    const bool owner = t < 25 || (t == 25 && ic == 0);
    const Opt1 pst = owner ? opt_prefetch1(O, oc, t < 25 ? O.off[2] + (ocn * C1 + ic) * 25 + t : O.off[3] + ocn)
                           : Opt1{};
    float acc = 0.f;
    for (int b0 = 0; b0 < B; b0 += kWgChunk) {
      const int nb = (B - b0) < kWgChunk ? (B - b0) : kWgChunk;
      __syncthreads();
      constexpr int NP4 = kWgChunk * 49;
      float4 pv[(NP4 + 255) / 256];
#pragma unroll
      for (int i = 0; i < (NP4 + 255) / 256; ++i) {
        const int e = t + i * 256, bb = e / 49, q = e - bb * 49;
        pv[i] = bb < nb ? reinterpret_cast<const float4*>(P.p1 + ((int64_t)(b0 + bb) * C1 + ic) * 196)[q]
                        : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      constexpr int NG = kWgChunk * 25;
      float gvv[(NG + 255) / 256];
      int kvv[(NG + 255) / 256];
#pragma unroll
      for (int i = 0; i < (NG + 255) / 256; ++i) {
        const int e = t + i * 256, bb = e / 25, q = e - bb * 25;
        const int64_t o = (int64_t)(b0 + bb) * FLAT + ocn * 25 + q;
        const bool ok = bb < nb;
        kvv[i] = ok ? (int)P.i2[o] : 4;
        gvv[i] = ok ? P.dflat[o] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < (NP4 + 255) / 256; ++i)
        if (t + i * 256 < NP4) reinterpret_cast<float4*>(ps)[t + i * 256] = pv[i];
#pragma unroll
      for (int i = 0; i < (NG + 255) / 256; ++i) {
        const int e = t + i * 256;
        if (e < NG) {
          const int bb = e / 25, q = e - bb * 25, k = kvv[i] < 4 ? kvv[i] : 0;
          gs[e] = kvv[i] < 4 ? gvv[i] : 0.f;
          pos[e] = bb * 196 + (2 * (q / 5) + (k >> 1)) * 14 + 2 * (q % 5) + (k & 1);
        }
      }
      __syncthreads();
      if (s < 9) {
        if (tap < 25) {
          const float* pc = ps + (tap / 5) * 14 + tap % 5;
#pragma unroll 8
          for (int e = s; e < nb * 25; e += 9) acc = fmaf(gs[e], pc[pos[e]], acc);
        } else {
#pragma unroll 8
          for (int e = s; e < nb * 25; e += 9) acc += gs[e];
        }
      }
    }
    __syncthreads();
    if (s < 9) red[s * NT + tap] = acc;
    __syncthreads();
    if (t < NT) {
      float v = 0.f;
      for (int i = 0; i < 9; ++i) v += red[i * NT + t];
      if (owner) apply_pre1(O, oc, t < 25 ? O.off[2] + (ocn * C1 + ic) * 25 + t : O.off[3] + ocn, v, pst);
    }
  } else {
    int bf = blk - nA - C2 * C1;
    if (bf < NB3) {
      fc_wgrad_block<FLAT>(bf, F1, B, P.dh1, P.p2, O, O.off[4], O.off[5], oc);
    } else if ((bf -= NB3) < NB4) {
      fc_wgrad_block<F1>(bf, F2, B, P.dh2, P.h1, O, O.off[6], O.off[7], oc);
    } else if ((bf -= NB4) < NB5) {
      fc_wgrad_block<F2>(bf, NC, B, P.dlogits, P.h2, O, O.off[8], O.off[9], oc);
    }
  }
  // launch-wide arrival: the last block advances the step counters (all reads of ctrl above
  // precede each block's own arrival, so no block can observe the increment).
  if (ctrl) {
    __syncthreads();
    if (t == 0) {
      const unsigned prev =
          __hip_atomic_fetch_add(&P.counters[C1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == gridDim.x - 1) {
        ctrl[0] += 1;
        ctrl[1] += 1;
        __hip_atomic_store(&P.counters[C1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Launch variant of the per-sample chain (set_lenet_variant; initial value from MLT_LENET_VARIANT):
//   0 (default)  K1 conv1 -> KF from p1 (conv2 + fc chain) -> K4 -> K5       4 launches
//   1            KF for the whole chain (K1..K4 fused)      -> K5            2 launches
//   2            K1 -> K2 conv2 -> K3 fc chain -> K4 -> K5                  5 launches
// Measured (MI355X, batch 32, bench.py): 0 is fastest -- one CU per sample leaves the fully fused
// KF's conv phases LDS-latency bound (40-44 vs 33 us per step) and 2 pays one more boundary.
// All three run the same arithmetic; tests/test_lenet_native.py checks each against autograd.
static int g_lenet_variant = [] {
  const char* v = getenv("MLT_LENET_VARIANT");
  const int x = v ? atoi(v) : 0;
  return (x >= 0 && x <= 2) ? x : 0;
}();

void set_lenet_variant(int v) { g_lenet_variant = (v >= 0 && v <= 2) ? v : 0; }
int get_lenet_variant() { return g_lenet_variant; }

// non-fused training steps: the CE leaves per-sample stats terms for K4's fixed-order sum
static int kFcDefer(int mode, const LeNetPtrs& P) {
  return ((mode & LENET_CE) && (mode & LENET_BWD) && P.stats && P.cestat) ? LENET_STATS_DEFER : 0;
}

template <class D>
static void run_lenet(int mode, int B, const LeNetPtrs& P, const LeNetAug& A, const LeNetOpt& O, hipStream_t st) {
  if (B <= 0) return;
  const float inv_B = 1.f / (float)B;
  const bool fused = g_lenet_variant == 1 && (mode & (LENET_FWD | LENET_CE | LENET_BWD));
  if (fused) {
    hipLaunchKernelGGL(lenet_sample_fused<D>, dim3(B), dim3(kFusedThreads), 0, st, mode, P, A, inv_B);
  } else {
    const bool c2fc = g_lenet_variant != 2;  // conv2 + fc chain as the per-sample KF launch (from p1)
    if (mode & LENET_FWD) {
      hipLaunchKernelGGL(lenet_conv1_fwd<D>, dim3(B, D::C1), dim3(256), 0, st, A, P.w1, P.b1, P.x, P.p1, P.i1,
                         A.data ? P.targets : nullptr, P.dtargets, A.data ? P.stage : nullptr,
                         A.data ? P.stage_meta : nullptr);
      if (c2fc) {
        hipLaunchKernelGGL(lenet_sample_fused<D>, dim3(B), dim3(kFusedThreads),
                           0, st, mode | LENET_FROM_P1 | kFcDefer(mode, P), P, A, inv_B);
      } else {
        hipLaunchKernelGGL(lenet_conv2_fwd<D>, dim3(B, D::C2 / 4), dim3(128), 0, st, P.p1, P.w2, P.b2, P.p2, P.i2);
        hipLaunchKernelGGL(lenet_fc<D>, dim3(B), dim3(kFcThreads), 0, st, mode | kFcDefer(mode, P), P, inv_B);
      }
    } else if (mode & (LENET_CE | LENET_BWD)) {
      hipLaunchKernelGGL(lenet_fc<D>, dim3(B), dim3(kFcThreads), 0, st, mode | kFcDefer(mode, P), P, inv_B);
    }
    if (mode & LENET_BWD) {
      // K4: dgrad + conv1 wgrad slabs (y < C1), conv2 wgrad slabs (C1 <= y < 2 C1), fc wgrads
      // with their update (y >= 2 C1: fc weights are not read after K3/KF)
      // (+ one row of next-step input staging blocks on the device-dataset path)
      const unsigned k4y = 2 * D::C1 + (fc_wgrad_blocks<D>() + B - 1) / B;
      // (+ one block row summing the deferred per-sample loss / accuracy terms in sample order)
      const bool stage = A.data && A.ctrl && P.stage && P.stage_meta && B <= A.batch_stride;
      const bool defer = kFcDefer(mode, P) != 0;
      const int rows = (int)k4y + (stage ? 1 : 0) + (defer ? 1 : 0);
      hipLaunchKernelGGL((lenet_conv2_dgrad<D, true>), dim3(B, rows), dim3(256), 0, st,
                         P.dflat, P.i2, P.w2, P.i1, P.g1, P.x, P.p1, P.slab1, mode, P, O, A.ctrl, A,
                         stage ? (int)k4y : -1, defer ? rows - 1 : -1);
    }
  }
  if ((mode & LENET_BWD) && !(fused && (mode & LENET_TRACE))) {
    constexpr int NB3 = (D::F1 * (D::FLAT / 4) + 255) / 256, NB4 = (D::F2 * (D::F1 / 4) + 255) / 256,
                  NB5 = (D::NC * (D::F2 / 4) + 255) / 256;
    // non-fused path: K4 already produced the conv wgrad slabs (K4WG); the fused KF does not
    const int k4wg = fused ? 0 : LENET_K4WG;
    constexpr int NR1 = (D::C1 * kTaps1 + 255) / 256, NR2 = (D::C2 * D::C1 * 25 + D::C2 + 255) / 256;
    const int nblk = k4wg ? NR1 + NR2  // K4 ran the fc roles too
                          : (B + kSpb1 - 1) / kSpb1 * D::C1 + D::C2 * D::C1 + NB3 + NB4 + NB5;
#ifdef MLT_DEBUG
    // MLT_LENET_WGRAD_SKIP=<mask> (debug builds, role profiling only): 1 conv1 / 2 conv2 / 4 fc
    // roles return at once -- never compiled into a release build, where it would skip training work
    static const int skip = [] {
      const char* v = getenv("MLT_LENET_WGRAD_SKIP");
      return v ? (atoi(v) & 7) : 0;
    }();
#else
    constexpr int skip = 0;
#endif
    hipLaunchKernelGGL(lenet_wgrad<D>, dim3(nblk), dim3(256), 0, st, mode | (skip << 9) | k4wg, P, O, B, A.ctrl);
  }
}

void launch_lenet(int cfg, int mode, int B, const LeNetPtrs& P, const LeNetAug& A, const LeNetOpt& O,
                  hipStream_t stream) {
  if (cfg == LENET_TINY)
    run_lenet<LeNetTiny>(mode, B, P, A, O, stream);
  else
    run_lenet<LeNetDefault>(mode, B, P, A, O, stream);
}

// ---------------------------------------------------------------------------
// Standalone CIFAR augmentation for the generic device data path.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void cifar_augment_kernel(LeNetAug aug, float* __restrict__ out,
                                                            int64_t* __restrict__ targets_out,
                                                            const int64_t* __restrict__ dtargets) {
  const int b = blockIdx.x, t = threadIdx.x;
  const int64_t step = aug.ctrl ? aug.ctrl[0] : aug.step_host, sie = aug.ctrl ? aug.ctrl[1] : aug.sie_host;
  int64_t pos = sie * aug.batch_stride + b;
  if (pos >= aug.perm_len) pos %= aug.perm_len;
  int64_t idx = aug.perm[pos];
  idx = idx < 0 ? 0 : (idx >= aug.n ? aug.n - 1 : idx);
  const uint64_t h = mix64(mix64(aug.seed + (uint64_t)step) ^ (uint64_t)pos);
  const int span = 2 * aug.pad + 1;
  const int ci = aug.pad ? (int)(h % span) : 0;
  const int cj = aug.pad ? (int)((h >> 20) % span) : 0;
  const bool fl = aug.flip && ((h >> 40) & 1);
  __shared__ __attribute__((aligned(16))) uint4 rawimg[192];
  if (t < 192) rawimg[t] = reinterpret_cast<const uint4*>(aug.data + idx * 3072)[t];
  __syncthreads();
  const uint8_t* img = reinterpret_cast<const uint8_t*>(rawimg);
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const int e = t + i * 256;
    const int c = e >> 10, y = (e >> 5) & 31, xx = e & 31;
    const int sx = fl ? 31 - xx : xx;
    const int r = y + ci - aug.pad, q = sx + cj - aug.pad;
    const bool in = (unsigned)r < 32u && (unsigned)q < 32u;
    const float u = in ? (float)img[(r * 32 + q) * 3 + c] : 0.f;
    out[(int64_t)b * 3072 + e] = (u / 255.f - aug.mean[c]) / aug.std[c];
  }
  if (t == 0 && targets_out) targets_out[b] = dtargets[idx];
}

void launch_cifar_augment(const LeNetAug& A, int B, float* out, int64_t* targets_out, const int64_t* dtargets,
                          hipStream_t stream) {
  if (B <= 0) return;
  hipLaunchKernelGGL(cifar_augment_kernel, dim3(B), dim3(256), 0, stream, A, out, targets_out, dtargets);
}

}  // namespace mlt
