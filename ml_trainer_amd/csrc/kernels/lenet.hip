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
//   K4 conv2_dgrad grid (B, C1)     unpool2 -> conv2 dgrad -> ReLU/unpool1 mask
//   K5 wgrad       role-split grid  conv1/conv2/fc1..fc3 wgrad+bias + fused optimizer update + step counters
//                  (conv1 partials reduced in-launch by the last-arriving block of each channel)
//
// ReLU+maxpool are fused: pool(relu(c)) = relu(max(c)); the gradient reaches the
// first arg-max of the window only when that max is > 0 (torch's threshold_backward
// zeroes it otherwise), so one uint8 per pooled cell stores the arg-max (0..3) or 4
// for "dead".  The backward never materialises the 4x larger un-pooled gradient.
// All batch reductions run in a fixed order: results are bitwise reproducible.
#include "mlt_common.h"
#include "mlt_kernels.h"
#include "mlt_optim.h"

namespace mlt {

template <int C1_, int C2_, int F1_, int F2_, int NC_>
struct LeNetDims {
  static constexpr int C1 = C1_, C2 = C2_, F1 = F1_, F2 = F2_, NC = NC_, FLAT = C2_ * 25;
  static_assert(C2_ % 4 == 0 && F1_ % 4 == 0 && F2_ % 4 == 0 && NC_ <= 64, "LeNet dims");
};
using LeNetDefault = LeNetDims<6, 16, 120, 84, 10>;
using LeNetTiny = LeNetDims<4, 8, 64, 32, 10>;

constexpr int kTaps1 = 76;        // conv1 wgrad partial: 75 taps + bias
constexpr int kSlabStride = 128;  // floats per (sample group, oc) slab: 512 B, so no two writers share a cache line
constexpr int kSpb1 = 1;          // samples per conv1-wgrad block (slabs per oc = ceil(B / kSpb1)); 4 measured slower

// ---------------------------------------------------------------------------
// K1: [augment] + conv1 + bias + ReLU + maxpool2x2.  One block per (sample, out-channel).
// ---------------------------------------------------------------------------
template <class D>
__global__ __launch_bounds__(256) void lenet_conv1_fwd(LeNetAug aug, const float* __restrict__ w1,
                                                       const float* __restrict__ b1, float* __restrict__ x,
                                                       float* __restrict__ p1, uint8_t* __restrict__ i1,
                                                       int64_t* __restrict__ targets,
                                                       const int64_t* __restrict__ dtargets) {
  const int b = blockIdx.x, oc = blockIdx.y, t = threadIdx.x;
  __shared__ __attribute__((aligned(16))) float xs[3 * 1024];
  __shared__ __attribute__((aligned(16))) uint4 rawimg[192];
  // filter + bias first: block-uniform scalar loads that overlap the ctrl -> perm -> image chain
  float wr[75];
#pragma unroll
  for (int i = 0; i < 75; ++i) wr[i] = w1[oc * 75 + i];
  const float bias = b1[oc];
  if (aug.data) {
    const int64_t step = aug.ctrl[0], sie = aug.ctrl[1];
    int64_t pos = sie * aug.batch_stride + b;
    if (pos >= aug.perm_len) pos %= aug.perm_len;
    int64_t idx = aug.perm[pos];
    idx = idx < 0 ? 0 : (idx >= aug.n ? aug.n - 1 : idx);
    const uint64_t h = mix64(mix64(aug.seed + (uint64_t)step) ^ (uint64_t)pos);
    const int span = 2 * aug.pad + 1;
    const int ci = aug.pad ? (int)(h % span) : 0;
    const int cj = aug.pad ? (int)((h >> 20) % span) : 0;
    const bool fl = aug.flip && ((h >> 40) & 1);
    // stage the raw 3 KB HWC image with 16-byte loads, then crop/flip/normalise from LDS
    const uint4* img4 = reinterpret_cast<const uint4*>(aug.data + idx * 3072);
    if (t < 192) rawimg[t] = img4[t];
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
      xs[e] = v;
      if (oc == 0) x[(int64_t)b * 3072 + e] = v;
    }
    if (oc == 0 && t == 0 && targets) targets[b] = dtargets[idx];
  } else {
    const float4* src = reinterpret_cast<const float4*>(x + (int64_t)b * 3072);
    float4 v[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) v[i] = src[t + i * 256];
#pragma unroll
    for (int i = 0; i < 3; ++i) reinterpret_cast<float4*>(xs)[t + i * 256] = v[i];
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
      for (int q = 0; q < 6; ++q) in[q] = xs[ic * 1024 + (y0 + r) * 32 + x0 + q];
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

template <int NCOLS, int NROWS, int NT>
struct RegLinear {
  static constexpr int NV = NCOLS / 4;
  static constexpr int G = pow2_ge(NV);
  static constexpr int PL = (NV + G - 1) / G;
  static constexpr int R = 64 / G;
  static constexpr int NW = NT / 64;
  static constexpr int RPI = NW * R;  // row groups (rows per iteration over the block)
  static constexpr int IT = (NROWS + RPI - 1) / RPI;
  static constexpr int SCRATCH = RPI * NCOLS;
  float4 w[IT][PL];
  float bias[IT];

  __device__ __forceinline__ int row(int it) const {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    return it * RPI + wid * R + lane / G;
  }
  __device__ __forceinline__ void load(const float* __restrict__ W, const float* __restrict__ b) {
    const int gl = (threadIdx.x & 63) % G;
    const float4* w4 = reinterpret_cast<const float4*>(W);
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int r = row(it);
#pragma unroll
      for (int i = 0; i < PL; ++i) {
        const int v = gl + i * G;
        w[it][i] = (r < NROWS && v < NV) ? w4[r * NV + v] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      bias[it] = r < NROWS ? b[r] : 0.f;
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
          const float4 xv = x4[v];
          acc = fmaf(w[it][i].x, xv.x, acc);
          acc = fmaf(w[it][i].y, xv.y, acc);
          acc = fmaf(w[it][i].z, xv.z, acc);
          acc = fmaf(w[it][i].w, xv.w, acc);
        }
      }
      acc = group_sum<G>(acc);
      const int r = row(it);
      if (gl == 0 && r < NROWS) {
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
        acc.x = fmaf(dv[it], w[it][i].x, acc.x);
        acc.y = fmaf(dv[it], w[it][i].y, acc.y);
        acc.z = fmaf(dv[it], w[it][i].z, acc.z);
        acc.w = fmaf(dv[it], w[it][i].w, acc.w);
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

template <class D>
__global__ __launch_bounds__(kFcThreads) void lenet_fc(int mode, LeNetPtrs P, float inv_B) {
  constexpr int FLAT = D::FLAT, F1 = D::F1, F2 = D::F2, NC = D::NC, NT = kFcThreads;
  using L1 = RegLinear<FLAT, F1, NT>;
  using L2 = RegLinear<F1, F2, NT>;
  using L3 = RegLinear<F2, NC, NT>;
  constexpr int SCR = cmax(L1::SCRATCH, cmax(L2::SCRATCH, L3::SCRATCH));
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wid = t >> 6;
  __shared__ __attribute__((aligned(16))) float f[FLAT];
  __shared__ __attribute__((aligned(16))) float sh1[F1];
  __shared__ __attribute__((aligned(16))) float sh2[F2];
  __shared__ __attribute__((aligned(16))) float sdl[64];
  __shared__ __attribute__((aligned(16))) float sdh2[F2];
  __shared__ __attribute__((aligned(16))) float sdh1[F1];
  __shared__ __attribute__((aligned(16))) float slog[64];
  __shared__ __attribute__((aligned(16))) float scratch[SCR];

  // the label is needed only by the CE phase, but loading it now keeps it off the dependent chain
  const int64_t tgt_pre = (mode & LENET_CE) ? P.targets[b] : 0;
  L1 l1;
  L2 l2;
  L3 l3;
  l1.load(P.w3, P.b3);  // all weight loads in flight together
  l2.load(P.w4, P.b4);
  l3.load(P.w5, P.b5);

  if (mode & LENET_FWD) {
    const float4* src = reinterpret_cast<const float4*>(P.p2 + (int64_t)b * FLAT);
    if (t < FLAT / 4) reinterpret_cast<float4*>(f)[t] = src[t];
    __syncthreads();
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
      const float z = lane < NC ? slog[lane] : -INFINITY;
      const float mx = wave_max(z);
      const float e = lane < NC ? expf(z - mx) : 0.f;
      const float s = wave_sum(e);
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
        atomicAdd(&P.stats[0], (double)loss * (double)inv_B);
        atomicAdd(&P.stats[1], (am == tgt) ? (double)inv_B : 0.0);
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
    l1.bwd(sdh1, scratch, nullptr, P.dflat + (int64_t)b * FLAT, nullptr);
  }
}

// ---------------------------------------------------------------------------
// K4: unpool2 (via arg-max) -> conv2 dgrad -> mask by pool1 arg-max liveness.
// Block (256 = 4 waves) per (sample, input channel); lane = 2x2 output patch of the
// 14x14 map, wave = quarter of the conv2 output channels (reduced through LDS in order).
// ---------------------------------------------------------------------------
template <class D>
__global__ __launch_bounds__(256) void lenet_conv2_dgrad(const float* __restrict__ dflat,
                                                         const uint8_t* __restrict__ i2,
                                                         const float* __restrict__ w2,
                                                         const uint8_t* __restrict__ i1, float* __restrict__ g1) {
  constexpr int C1 = D::C1, C2 = D::C2, FLAT = D::FLAT, NZ4 = C2 * 81, NS = (FLAT + 255) / 256;
  const int b = blockIdx.x, ic = blockIdx.y, t = threadIdx.x, lane = t & 63, wid = t >> 6;
  __shared__ __attribute__((aligned(16))) float dc[C2 * 324];  // zero-padded dense conv2-output grad [C2][18][18]
  __shared__ __attribute__((aligned(16))) float4 red[4][64];
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
    g1[base] = i1[base] < 4 ? s.x : 0.f;
    g1[base + 1] = i1[base + 1] < 4 ? s.y : 0.f;
    g1[base + 14] = i1[base + 14] < 4 ? s.z : 0.f;
    g1[base + 15] = i1[base + 15] < 4 ? s.w : 0.f;
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

template <class D>
__global__ __launch_bounds__(256) void lenet_wgrad(int mode, LeNetPtrs P, LeNetOpt O, int B,
                                                   int64_t* __restrict__ ctrl) {
  constexpr int C1 = D::C1, C2 = D::C2, F1 = D::F1, F2 = D::F2, NC = D::NC, FLAT = D::FLAT;
  constexpr int NB3 = (F1 * (FLAT / 4) + 255) / 256, NB4 = (F2 * (F1 / 4) + 255) / 256,
                NB5 = (NC * (F2 / 4) + 255) / 256;
  __shared__ __attribute__((aligned(16))) float lds[kSpb1 * (3072 + 2 * 196) + 3 * kTaps1 + 4 > 8192
                                                        ? kSpb1 * (3072 + 2 * 196) + 3 * kTaps1 + 4
                                                        : 8192];
  const int nA = (B + kSpb1 - 1) / kSpb1 * C1, nblk = nA + C2 * C1 + NB3 + NB4 + NB5;
  int blk = blockIdx.x;
  const int t = threadIdx.x;
  // The step counters are read by every block here and advanced by the last block of the launch.
  OptCtx oc;
  oc.on = (mode & LENET_OPT) != 0;
  oc.lr = O.h.lr;
  oc.t = 1.f;
  if (oc.on) {
    const int64_t step = ctrl ? ctrl[0] : 0, sie = ctrl ? ctrl[1] : 0;
    oc.t = (float)(step + 1);
    if (O.lr_ptr) oc.lr = O.lr_ptr[O.lr_table ? sie : 0];
  }
  if (blk < nA) {
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
      if (prev == (unsigned)(nblk - 1)) {
        ctrl[0] += 1;
        ctrl[1] += 1;
        __hip_atomic_store(&P.counters[C1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// ---------------------------------------------------------------------------
template <class D>
static void run_lenet(int mode, int B, const LeNetPtrs& P, const LeNetAug& A, const LeNetOpt& O, hipStream_t st) {
  if (B <= 0) return;
  const float inv_B = 1.f / (float)B;
  if (mode & LENET_FWD) {
    hipLaunchKernelGGL(lenet_conv1_fwd<D>, dim3(B, D::C1), dim3(256), 0, st, A, P.w1, P.b1, P.x, P.p1, P.i1,
                       A.data ? P.targets : nullptr, P.dtargets);
    hipLaunchKernelGGL(lenet_conv2_fwd<D>, dim3(B, D::C2 / 4), dim3(128), 0, st, P.p1, P.w2, P.b2, P.p2, P.i2);
  }
  if (mode & (LENET_FWD | LENET_CE | LENET_BWD)) {
    hipLaunchKernelGGL(lenet_fc<D>, dim3(B), dim3(kFcThreads), 0, st, mode, P, inv_B);
  }
  if (mode & LENET_BWD) {
    hipLaunchKernelGGL(lenet_conv2_dgrad<D>, dim3(B, D::C1), dim3(256), 0, st, P.dflat, P.i2, P.w2, P.i1, P.g1);
    constexpr int NB3 = (D::F1 * (D::FLAT / 4) + 255) / 256, NB4 = (D::F2 * (D::F1 / 4) + 255) / 256,
                  NB5 = (D::NC * (D::F2 / 4) + 255) / 256;
    const int nblk = (B + kSpb1 - 1) / kSpb1 * D::C1 + D::C2 * D::C1 + NB3 + NB4 + NB5;
    hipLaunchKernelGGL(lenet_wgrad<D>, dim3(nblk), dim3(256), 0, st, mode, P, O, B, A.ctrl);
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
