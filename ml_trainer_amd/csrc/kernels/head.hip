// Classifier head of the BERT classifier (models/bert.py: pooled = tanh(W_p h_CLS + b_p),
// logits = W_c pooled + b_c; the reference's criterion is softmax-CE, src/trainer.py:141-142).
// The pooler is a plain GEMM with a tanh epilogue (gemm_tile / gemm.hip, epilogue mode 3); the
// classifier has only num_labels (<= 64) outputs, which no MFMA tile fits, so these kernels do
// it on the VALU:
//   head_cls_fwd    one block per sample: num_labels dot products of length h (wave-parallel,
//                   fixed-order reductions) -> logits
//   head_cls_bwd_x  one block per sample: dpre = (dlogits . W_c) * (1 - pooled^2), bf16 -- the
//                   pooler GEMMs' dY
//   head_cls_bwd_w  dW_c = dlogits^T . pooled and db_c = colsum(dlogits), batch summed in sample
//                   order per output (deterministic), written or accumulated into the fp32 grads
#include "mlt_common.h"
#include "mlt_kernels.h"

namespace mlt {

constexpr int kHeadThreads = 256;
constexpr int kHeadMaxLabels = 1024;  // num_labels bound of the backward (bindings check it)

__global__ __launch_bounds__(kHeadThreads) void head_cls_fwd_kernel(const float* __restrict__ pooled, int h,
                                                                     const float* __restrict__ wc,
                                                                     const float* __restrict__ bc, int L,
                                                                     float* __restrict__ logits) {
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wid = t >> 6;
  __shared__ float red[kHeadThreads / 64][64];
  const float* x = pooled + (int64_t)b * h;
  for (int l0 = 0; l0 < L; l0 += 64) {
    const int nl = min(64, L - l0);
    for (int l = 0; l < nl; ++l) {
      float s = 0.f;
      for (int j = t; j < h; j += kHeadThreads) s = fmaf(x[j], wc[(int64_t)(l0 + l) * h + j], s);
      s = wave_sum(s);
      if (lane == 0) red[wid][l] = s;
    }
    __syncthreads();
    if (t < nl) {
      float s = bc ? bc[l0 + t] : 0.f;
      for (int w = 0; w < kHeadThreads / 64; ++w) s += red[w][t];  // fixed order
      logits[(int64_t)b * L + l0 + t] = s;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(kHeadThreads) void head_cls_bwd_x_kernel(const float* __restrict__ dlogits, int L,
                                                                       const float* __restrict__ wc,
                                                                       const float* __restrict__ pooled, int h,
                                                                       uint16_t* __restrict__ dpre) {
  const int b = blockIdx.x, t = threadIdx.x;
  // the sample's whole dlogits row staged once (L <= kHeadMaxLabels, host-checked): the j loop
  // below has a thread-dependent trip count, so it must not contain a barrier
  __shared__ float dl[kHeadMaxLabels];
  for (int l = t; l < L; l += kHeadThreads) dl[l] = dlogits[(int64_t)b * L + l];
  __syncthreads();
  const float* x = pooled + (int64_t)b * h;
  for (int j = t; j < h; j += kHeadThreads) {
    float s = 0.f;
    for (int l = 0; l < L; ++l) s = fmaf(dl[l], wc[(int64_t)l * h + j], s);
    const float y = x[j];
    dpre[(int64_t)b * h + j] = f32_to_bf16(s * (1.f - y * y));
  }
}

// grid: ceil((L * h + L) / 256) blocks; output o < L*h: dW_c[o / h][o % h], else db_c[o - L*h]
__global__ __launch_bounds__(kHeadThreads) void head_cls_bwd_w_kernel(const float* __restrict__ dlogits,
                                                                       const float* __restrict__ pooled, int B,
                                                                       int h, int L, float* __restrict__ dwc,
                                                                       float* __restrict__ dbc, int accumulate) {
  const int64_t o = (int64_t)blockIdx.x * kHeadThreads + threadIdx.x;
  const int64_t nw = (int64_t)L * h;
  if (o >= nw + L) return;
  float s = 0.f;
  if (o < nw) {
    const int l = (int)(o / h), j = (int)(o - (int64_t)l * h);
    for (int b = 0; b < B; ++b) s = fmaf(dlogits[(int64_t)b * L + l], pooled[(int64_t)b * h + j], s);
    dwc[o] = accumulate ? dwc[o] + s : s;
  } else {
    const int l = (int)(o - nw);
    for (int b = 0; b < B; ++b) s += dlogits[(int64_t)b * L + l];
    if (dbc) dbc[l] = accumulate ? dbc[l] + s : s;
  }
}

void launch_head_cls_fwd(const float* pooled, int B, int h, const float* wc, const float* bc, int L, float* logits,
                         hipStream_t st) {
  if (B <= 0) return;
  hipLaunchKernelGGL(head_cls_fwd_kernel, dim3(B), dim3(kHeadThreads), 0, st, pooled, h, wc, bc, L, logits);
}

void launch_head_cls_bwd(const float* dlogits, const float* pooled, const float* wc, int B, int h, int L,
                         uint16_t* dpre, float* dwc, float* dbc, bool accumulate, hipStream_t st) {
  if (B <= 0) return;
  hipLaunchKernelGGL(head_cls_bwd_x_kernel, dim3(B), dim3(kHeadThreads), 0, st, dlogits, L, wc, pooled, h, dpre);
  const int64_t n = (int64_t)L * h + L;
  hipLaunchKernelGGL(head_cls_bwd_w_kernel, dim3((unsigned)((n + kHeadThreads - 1) / kHeadThreads)),
                     dim3(kHeadThreads), 0, st, dlogits, pooled, B, h, L, dwc, dbc, accumulate ? 1 : 0);
}

}  // namespace mlt
