// Fused optimizer math shared by the flat multi-tensor optimizer kernel
// (csrc/kernels/optim.hip) and the LeNet engine's finalize kernel
// (csrc/kernels/lenet.hip).
//
// Semantics follow torch.optim exactly (the reference selects these by name at
// src/trainer.py:123-138): SGD(momentum, dampening, nesterov, weight_decay as L2),
// Adam (L2 weight decay), AdamW (decoupled decay), Adagrad (lr_decay,
// initial_accumulator_value=0), Adamax (infinity norm).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mlt {

enum OptKind : int { OPT_SGD = 0, OPT_ADAM = 1, OPT_ADAMW = 2, OPT_ADAGRAD = 3, OPT_ADAMAX = 4 };

struct OptHyper {
  float lr;            // used when lr_ptr == nullptr
  float momentum;
  float dampening;
  float weight_decay;
  float beta1, beta2, eps;
  float lr_decay;      // adagrad
  float grad_scale;    // multiply incoming grads (e.g. 1/world or 1/loss_scale)
  int nesterov;
  int maximize;
  int kind;
};

// One element update. s1/s2 are the optimizer state slots for this element:
//   SGD: s1 = momentum buffer; Adam/AdamW/Adamax: s1 = exp_avg, s2 = exp_avg_sq / exp_inf;
//   Adagrad: s1 = state_sum.
// `t` is the 1-based step count (after increment), as torch tracks it.
// opt_update_k<K>: the update of one optimizer kind (compile-time): kernels that dispatch the kind
// once at their top keep only that kind's code on their hot path (a compact instruction footprint);
// opt_update: the same arithmetic behind a runtime switch (bitwise identical).
template <int K>
__device__ __forceinline__ void opt_update_k(const OptHyper& h, float lr, float t, float& p, float g, float& s1,
                                             float& s2) {
  g *= h.grad_scale;
  if (h.maximize) g = -g;
  if constexpr (K == OPT_SGD) {
    if (h.weight_decay != 0.f) g = fmaf(h.weight_decay, p, g);
    if (h.momentum != 0.f) {
      // torch initialises the buffer to a clone of d_p on the first step.
      float b = (t <= 1.f) ? g : fmaf(h.momentum, s1, (1.f - h.dampening) * g);
      s1 = b;
      g = h.nesterov ? fmaf(h.momentum, b, g) : b;
    }
    p = fmaf(-lr, g, p);
  } else if constexpr (K == OPT_ADAM || K == OPT_ADAMW) {
    if constexpr (K == OPT_ADAMW) {
      p *= (1.f - lr * h.weight_decay);
    } else {
      if (h.weight_decay != 0.f) g = fmaf(h.weight_decay, p, g);
    }
    s1 = fmaf(h.beta1, s1, (1.f - h.beta1) * g);
    s2 = fmaf(h.beta2, s2, (1.f - h.beta2) * g * g);
    const float bc1 = 1.f - powf(h.beta1, t);
    const float bc2 = 1.f - powf(h.beta2, t);
    const float step_size = lr / bc1;
    const float denom = sqrtf(s2) / sqrtf(bc2) + h.eps;
    p = fmaf(-step_size, s1 / denom, p);
  } else if constexpr (K == OPT_ADAGRAD) {
    if (h.weight_decay != 0.f) g = fmaf(h.weight_decay, p, g);
    const float clr = lr / (1.f + (t - 1.f) * h.lr_decay);
    s1 = fmaf(g, g, s1);
    p = fmaf(-clr, g / (sqrtf(s1) + h.eps), p);
  } else if constexpr (K == OPT_ADAMAX) {
    if (h.weight_decay != 0.f) g = fmaf(h.weight_decay, p, g);
    s1 = fmaf(h.beta1, s1, (1.f - h.beta1) * g);
    s2 = fmaxf(h.beta2 * s2, fabsf(g) + h.eps);
    const float clr = lr / (1.f - powf(h.beta1, t));
    p = fmaf(-clr, s1 / s2, p);
  }
}

__device__ __forceinline__ void opt_update(const OptHyper& h, float lr, float t, float& p, float g, float& s1,
                                           float& s2) {
  switch (h.kind) {
    case OPT_SGD: opt_update_k<OPT_SGD>(h, lr, t, p, g, s1, s2); break;
    case OPT_ADAM: opt_update_k<OPT_ADAM>(h, lr, t, p, g, s1, s2); break;
    case OPT_ADAMW: opt_update_k<OPT_ADAMW>(h, lr, t, p, g, s1, s2); break;
    case OPT_ADAGRAD: opt_update_k<OPT_ADAGRAD>(h, lr, t, p, g, s1, s2); break;
    case OPT_ADAMAX: opt_update_k<OPT_ADAMAX>(h, lr, t, p, g, s1, s2); break;
    default: break;
  }
}

}  // namespace mlt
