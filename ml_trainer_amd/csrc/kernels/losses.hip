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

}  // namespace mlt
