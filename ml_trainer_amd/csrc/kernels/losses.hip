// Fused softmax-cross-entropy and accuracy for gfx950 (reference criterion
// 'cross_entropy' + metric 'accuracy', src/trainer.py:141-142,164-166).
//
// One wave per row: online max/sum over the class dimension in 64-lane
// chunks, loss and the UNSCALED gradient softmax - onehot written in the same
// pass; accuracy (first arg-max == target) counted in the same kernel when
// requested. Mean reduction follows torch (ignore_index rows excluded from
// both numerator and denominator): sum and count are accumulated with
// atomics, a 1-thread finalize divides, and the backward kernel scales the
// stored gradient by grad_out / n_valid -- no host synchronisation anywhere.
#include "mlt_common.h"
#include "mlt_kernels.h"

namespace mlt {

template <typename T>
__device__ __forceinline__ float ld(const T* p, int64_t i);
template <>
__device__ __forceinline__ float ld<float>(const float* p, int64_t i) { return p[i]; }
template <>
__device__ __forceinline__ float ld<uint16_t>(const uint16_t* p, int64_t i) { return bf16_to_f32(p[i]); }

template <typename T>
__global__ __launch_bounds__(256) void ce_fwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                     int64_t B, int C, float* __restrict__ dl,
                                                     float* __restrict__ acc, float* __restrict__ correct,
                                                     int64_t ignore_index, float label_smoothing) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  __shared__ float red[3][4];
  float loss = 0.f, valid = 0.f, corr = 0.f;
  if (row < B) {
    const T* z = logits + row * C;
    float m = -INFINITY, s = 0.f;
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int c0 = 0; c0 < C; c0 += 64) {
      const int c = c0 + lane;
      const float v = c < C ? ld(z, c) : -INFINITY;
      const float cm = wave_max(v);
      if (cm > best) {  // first arg-max: smallest index holding the running maximum
        const unsigned long long mask = __ballot(v == cm && c < C);
        best = cm;
        bi = c0 + __ffsll((long long)mask) - 1;
      }
      const float nm = fmaxf(m, cm);
      s = s * __expf(m - nm) + wave_sum(c < C ? __expf(v - nm) : 0.f);
      m = nm;
    }
    const float lse = m + __logf(s);
    const int64_t t = tgt[row];
    const bool ok = t != ignore_index && t >= 0 && t < C;
    float zt = 0.f, zsum = 0.f;
    for (int c0 = 0; c0 < C; c0 += 64) {
      const int c = c0 + lane;
      if (c < C) {
        const float v = ld(z, c);
        const float p = __expf(v - lse);
        const float on = (ok && c == t) ? 1.f : 0.f;
        float g = p - (1.f - label_smoothing) * on - label_smoothing / (float)C;
        dl[row * C + c] = ok ? g : 0.f;
        if (c == t) zt = v;
        zsum += v;
      }
    }
    zt = wave_sum(zt);
    zsum = wave_sum(zsum);
    if (ok) {
      loss = (1.f - label_smoothing) * (lse - zt) + label_smoothing * (lse - zsum / (float)C);
      valid = 1.f;
    }
    corr = (bi == t) ? 1.f : 0.f;
  }
  if (lane == 0) {
    red[0][threadIdx.x >> 6] = loss;
    red[1][threadIdx.x >> 6] = valid;
    red[2][threadIdx.x >> 6] = corr;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float a = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    const float b = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    const float c = red[2][0] + red[2][1] + red[2][2] + red[2][3];
    atomicAdd(&acc[0], a);
    atomicAdd(&acc[1], b);
    if (correct) atomicAdd(correct, c / (float)B);
  }
}

__global__ void ce_finalize_kernel(const float* __restrict__ acc, float* __restrict__ loss) {
  loss[0] = acc[0] / fmaxf(acc[1], 1.f);
}

template <typename T>
__global__ __launch_bounds__(256) void ce_bwd_kernel(const float* __restrict__ dl, const float* __restrict__ gout,
                                                     const float* __restrict__ acc, int64_t n, T* __restrict__ out);

template <>
__global__ __launch_bounds__(256) void ce_bwd_kernel<float>(const float* __restrict__ dl,
                                                            const float* __restrict__ gout,
                                                            const float* __restrict__ acc, int64_t n,
                                                            float* __restrict__ out) {
  const float sc = gout[0] / fmaxf(acc[1], 1.f);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = dl[i] * sc;
}

template <>
__global__ __launch_bounds__(256) void ce_bwd_kernel<uint16_t>(const float* __restrict__ dl,
                                                               const float* __restrict__ gout,
                                                               const float* __restrict__ acc, int64_t n,
                                                               uint16_t* __restrict__ out) {
  const float sc = gout[0] / fmaxf(acc[1], 1.f);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = f32_to_bf16(dl[i] * sc);
}

template <typename T>
__global__ __launch_bounds__(256) void accuracy_kernel(const T* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                       int64_t B, int C, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  __shared__ float red[4];
  float corr = 0.f;
  if (row < B) {
    const T* z = logits + row * C;
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int c0 = 0; c0 < C; c0 += 64) {
      const int c = c0 + lane;
      const float v = c < C ? ld(z, c) : -INFINITY;
      const float cm = wave_max(v);
      if (cm > best) {
        const unsigned long long mask = __ballot(v == cm && c < C);
        best = cm;
        bi = c0 + __ffsll((long long)mask) - 1;
      }
    }
    corr = (bi == tgt[row]) ? 1.f : 0.f;
  }
  if (lane == 0) red[threadIdx.x >> 6] = corr;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, (red[0] + red[1] + red[2] + red[3]) / (float)B);
}

void launch_ce_fwd(const void* logits, bool bf16, const int64_t* tgt, int64_t B, int C, float* dl, float* acc,
                   float* correct, float* loss, int64_t ignore_index, float label_smoothing, hipStream_t st) {
  if (B <= 0) return;
  const dim3 grid((unsigned)((B + 3) / 4)), block(256);
  if (bf16)
    hipLaunchKernelGGL(ce_fwd_kernel<uint16_t>, grid, block, 0, st, (const uint16_t*)logits, tgt, B, C, dl, acc,
                       correct, ignore_index, label_smoothing);
  else
    hipLaunchKernelGGL(ce_fwd_kernel<float>, grid, block, 0, st, (const float*)logits, tgt, B, C, dl, acc, correct,
                       ignore_index, label_smoothing);
  hipLaunchKernelGGL(ce_finalize_kernel, dim3(1), dim3(1), 0, st, acc, loss);
}

void launch_ce_bwd(const float* dl, const float* gout, const float* acc, int64_t n, void* out, bool bf16,
                   hipStream_t st) {
  if (n <= 0) return;
  int64_t g = (n + 255) / 256;
  if (g > 2048) g = 2048;
  if (bf16)
    hipLaunchKernelGGL(ce_bwd_kernel<uint16_t>, dim3((unsigned)g), dim3(256), 0, st, dl, gout, acc, n,
                       (uint16_t*)out);
  else
    hipLaunchKernelGGL(ce_bwd_kernel<float>, dim3((unsigned)g), dim3(256), 0, st, dl, gout, acc, n, (float*)out);
}

void launch_accuracy(const void* logits, bool bf16, const int64_t* tgt, int64_t B, int C, float* out,
                     hipStream_t st) {
  if (B <= 0) return;
  const dim3 grid((unsigned)((B + 3) / 4)), block(256);
  if (bf16)
    hipLaunchKernelGGL(accuracy_kernel<uint16_t>, grid, block, 0, st, (const uint16_t*)logits, tgt, B, C, out);
  else
    hipLaunchKernelGGL(accuracy_kernel<float>, grid, block, 0, st, (const float*)logits, tgt, B, C, out);
}


// ---------------------------------------------------------------------------
// Regression / NLL criteria and the mcrmse metric (reference criteria 'l1',
// 'l2', 'neg-loss', custom MSE and metric 'mcrmse', src/trainer.py:143-148,
// 161-163, src/utils/functions.py:15-17).
//
// All reductions are two-pass and fixed-order (per-block partials in global,
// one finalize block sums them in index order): bitwise reproducible, no
// atomics, no host synchronisation. The forward writes the UNSCALED
// elementwise gradient (sign(d) / 2d / -1 at the target) so the backward is a
// single scale by grad_out / n read from device memory.
// ---------------------------------------------------------------------------
constexpr int kRegThreads = 256;
constexpr int kRegMaxBlocks = 1024;

// mode 0: L1 (|p - t|), mode 1: squared error ((p - t)^2)
__global__ __launch_bounds__(kRegThreads) void pointwise_loss_partial_kernel(const float* __restrict__ p,
                                                                             const float* __restrict__ t, int64_t n,
                                                                             int mode, float* __restrict__ g,
                                                                             float* __restrict__ part) {
  __shared__ float red[kRegThreads / 64];
  float s = 0.f;
  const int64_t stride = (int64_t)gridDim.x * kRegThreads;
  for (int64_t i = (int64_t)blockIdx.x * kRegThreads + threadIdx.x; i < n; i += stride) {
    const float d = p[i] - t[i];
    if (mode == 0) {
      s += fabsf(d);
      g[i] = (d > 0.f) ? 1.f : ((d < 0.f) ? -1.f : 0.f);  // torch's sign(0) = 0
    } else {
      s += d * d;
      g[i] = 2.f * d;
    }
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// NLL over log-probabilities [B, C]: per-block partial (sum of -logp[i, t_i], valid count)
__global__ __launch_bounds__(kRegThreads) void nll_partial_kernel(const float* __restrict__ logp,
                                                                  const int64_t* __restrict__ tgt, int64_t B, int C,
                                                                  int64_t ignore_index, float* __restrict__ part) {
  __shared__ float red[kRegThreads / 64];
  float s = 0.f, cnt = 0.f;
  const int64_t stride = (int64_t)gridDim.x * kRegThreads;
  for (int64_t r = (int64_t)blockIdx.x * kRegThreads + threadIdx.x; r < B; r += stride) {
    const int64_t k = tgt[r];
    if (k != ignore_index && k >= 0 && k < C) {
      s -= logp[r * C + k];
      cnt += 1.f;
    }
  }
  s = block_sum(s, red);
  cnt = block_sum(cnt, red);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = s;
    part[2 * blockIdx.x + 1] = cnt;
  }
}

// Sum the `nb` partials (stride `ps`: 1 = value only, 2 = value + count) in index order.
// out[0] = sum / denom, out[1] = denom (denom = n_fixed if > 0, else the summed count).
__global__ __launch_bounds__(kRegThreads) void loss_finalize_kernel(const float* __restrict__ part, int nb, int ps,
                                                                    float n_fixed, float* __restrict__ out) {
  __shared__ float red[kRegThreads / 64];
  float s = 0.f, c = 0.f;
  for (int i = threadIdx.x; i < nb; i += kRegThreads) {
    s += part[i * ps];
    if (ps == 2) c += part[i * ps + 1];
  }
  s = block_sum(s, red);
  c = block_sum(c, red);
  if (threadIdx.x == 0) {
    const float den = n_fixed > 0.f ? n_fixed : c;
    out[0] = s / fmaxf(den, 1.f);  // torch: all-ignored NLL is nan; we return 0 (documented in ops/losses.py)
    out[1] = den;
  }
}

// out = g * grad_out / den   (den = stats[1])
__global__ __launch_bounds__(kRegThreads) void loss_scale_grad_kernel(const float* __restrict__ g,
                                                                      const float* __restrict__ gout,
                                                                      const float* __restrict__ stats, int64_t n,
                                                                      float* __restrict__ out) {
  const float sc = gout[0] / fmaxf(stats[1], 1.f);
  const int64_t stride = (int64_t)gridDim.x * kRegThreads;
  for (int64_t i = (int64_t)blockIdx.x * kRegThreads + threadIdx.x; i < n; i += stride) out[i] = g[i] * sc;
}

// NLL backward: d logp[r, c] = -grad_out / count at c == t_r (valid rows), 0 elsewhere.
__global__ __launch_bounds__(kRegThreads) void nll_bwd_kernel(const int64_t* __restrict__ tgt, int64_t B, int C,
                                                              int64_t ignore_index, const float* __restrict__ gout,
                                                              const float* __restrict__ stats,
                                                              float* __restrict__ out) {
  const float v = -gout[0] / fmaxf(stats[1], 1.f);
  const int64_t n = B * C, stride = (int64_t)gridDim.x * kRegThreads;
  for (int64_t i = (int64_t)blockIdx.x * kRegThreads + threadIdx.x; i < n; i += stride) {
    const int64_t r = i / C, c = i - r * C;
    const int64_t k = tgt[r];
    out[i] = (k == c && k != ignore_index) ? v : 0.f;
  }
}

// mcrmse: column c's mean squared error over the B rows (one block per column, fixed order)
__global__ __launch_bounds__(kRegThreads) void colwise_mse_kernel(const float* __restrict__ p,
                                                                  const float* __restrict__ t, int64_t B, int C,
                                                                  float* __restrict__ col) {
  __shared__ float red[kRegThreads / 64];
  const int c = blockIdx.x;
  float s = 0.f;
  for (int64_t r = threadIdx.x; r < B; r += kRegThreads) {
    const float d = t[r * C + c] - p[r * C + c];
    s += d * d;
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) col[c] = s / (float)B;
}

__global__ __launch_bounds__(kRegThreads) void mcrmse_finalize_kernel(const float* __restrict__ col, int C,
                                                                      float* __restrict__ out) {
  __shared__ float red[kRegThreads / 64];
  float s = 0.f;
  for (int c = threadIdx.x; c < C; c += kRegThreads) s += sqrtf(col[c]);
  s = block_sum(s, red);
  if (threadIdx.x == 0) out[0] = s / (float)C;
}

static int reg_blocks(int64_t n) {
  int64_t b = (n + kRegThreads * 4 - 1) / (kRegThreads * 4);
  if (b < 1) b = 1;
  if (b > kRegMaxBlocks) b = kRegMaxBlocks;
  return (int)b;
}

int loss_partials_needed() { return 2 * kRegMaxBlocks; }

void launch_pointwise_loss_fwd(const float* p, const float* t, int64_t n, int mode, float* g, float* part,
                               float* out, hipStream_t st) {
  const int nb = reg_blocks(n);
  if (n > 0)
    hipLaunchKernelGGL(pointwise_loss_partial_kernel, dim3(nb), dim3(kRegThreads), 0, st, p, t, n, mode, g, part);
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(kRegThreads), 0, st, part, n > 0 ? nb : 0, 1,
                     (float)(n > 0 ? n : 1), out);
}

void launch_nll_fwd(const float* logp, const int64_t* tgt, int64_t B, int C, int64_t ignore_index, float* part,
                    float* out, hipStream_t st) {
  const int nb = reg_blocks(B);
  if (B > 0)
    hipLaunchKernelGGL(nll_partial_kernel, dim3(nb), dim3(kRegThreads), 0, st, logp, tgt, B, C, ignore_index, part);
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(kRegThreads), 0, st, part, B > 0 ? nb : 0, 2, 0.f, out);
}

void launch_loss_scale_grad(const float* g, const float* gout, const float* stats, int64_t n, float* out,
                            hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(loss_scale_grad_kernel, dim3(reg_blocks(n)), dim3(kRegThreads), 0, st, g, gout, stats, n, out);
}

void launch_nll_bwd(const int64_t* tgt, int64_t B, int C, int64_t ignore_index, const float* gout,
                    const float* stats, float* out, hipStream_t st) {
  if (B * C <= 0) return;
  hipLaunchKernelGGL(nll_bwd_kernel, dim3(reg_blocks(B * C)), dim3(kRegThreads), 0, st, tgt, B, C, ignore_index,
                     gout, stats, out);
}

void launch_mcrmse(const float* p, const float* t, int64_t B, int C, float* col, float* out, hipStream_t st) {
  if (C <= 0) return;
  hipLaunchKernelGGL(colwise_mse_kernel, dim3(C), dim3(kRegThreads), 0, st, p, t, B, C, col);
  hipLaunchKernelGGL(mcrmse_finalize_kernel, dim3(1), dim3(kRegThreads), 0, st, col, C, out);
}

}  // namespace mlt
