// Shared pieces of the bf16 GEMM kernels (gemm.hip: 128x128 general kernel,
// gemm_tile.hip: 256-wide global_load_lds kernels with split-K): epilogue parameters and
// the fused 4-column epilogue store.
#pragma once
#include "mlt_common.h"

namespace mlt {

struct GemmEpi {
  const float* bias;     // [N] or nullptr
  const uint16_t* aux;   // GELU: pre-activation output (written); DGELU: pre-activation input (read)
  const uint16_t* res;   // residual [M,N] bf16 (added) or nullptr
  int64_t ldaux, ldres;
  float alpha;
  int mode;              // 0 none, 1 gelu (writes aux), 2 dgelu (reads aux)
  int accumulate;        // C += result (fp32 output only)
  const float* inv_scale_a = nullptr;  // fp8: device-side 1/scale of A and B (multiplied into alpha)
  const float* inv_scale_b = nullptr;
};

// erf(z) by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below the bf16 output's ulp):
// one v_rcp, one v_exp, five FMAs instead of the library erff; `ez2` returns e^{-z^2}, which
// the GELU derivative reuses as its Gaussian density term.
__device__ __forceinline__ float erf_fast(float z, float& ez2) {
  const float a = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.f));
  const float poly =
      t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f), 0.254829592f);
  ez2 = __builtin_amdgcn_exp2f(-a * a * 1.4426950408889634f);
  return copysignf(fmaf(-poly, ez2, 1.f), z);
}
__device__ __forceinline__ float gelu_f(float x) {
  float e;
  return 0.5f * x * (1.f + erf_fast(x * 0.70710678118654752f, e));
}
__device__ __forceinline__ float gelu_grad(float x) {
  float e;  // e = exp(-x^2 / 2)
  const float cdf = 0.5f * (1.f + erf_fast(x * 0.70710678118654752f, e));
  return fmaf(x, 0.3989422804014327f * e, cdf);
}

// Apply the epilogue to 4 consecutive columns gn..gn+3 of row gm (values already scaled by
// alpha and biased) and store them. Columns >= N are skipped.
template <typename OutT>
__device__ __forceinline__ void epilogue_store4(OutT* __restrict__ C, int64_t ldc, const GemmEpi& epi, int gm,
                                                int gn, int N, float (&vv)[4]) {
  const bool full = gn + 4 <= N;
  if (epi.mode == 1) {  // GELU: keep the pre-activation for the backward pass
    uint16_t* aux = const_cast<uint16_t*>(epi.aux) + (int64_t)gm * epi.ldaux + gn;
    if (full && (((uintptr_t)aux) & 7) == 0) {
      ushort4 o;
      o.x = f32_to_bf16(vv[0]);
      o.y = f32_to_bf16(vv[1]);
      o.z = f32_to_bf16(vv[2]);
      o.w = f32_to_bf16(vv[3]);
      *reinterpret_cast<ushort4*>(aux) = o;
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (gn + q < N) aux[q] = f32_to_bf16(vv[q]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) vv[q] = gelu_f(bf16_to_f32(f32_to_bf16(vv[q])));
  } else if (epi.mode == 2) {
    const uint16_t* aux = epi.aux + (int64_t)gm * epi.ldaux + gn;
    if (full && (((uintptr_t)aux) & 7) == 0) {
      const ushort4 a = *reinterpret_cast<const ushort4*>(aux);
      vv[0] *= gelu_grad(bf16_to_f32(a.x));
      vv[1] *= gelu_grad(bf16_to_f32(a.y));
      vv[2] *= gelu_grad(bf16_to_f32(a.z));
      vv[3] *= gelu_grad(bf16_to_f32(a.w));
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (gn + q < N) vv[q] *= gelu_grad(bf16_to_f32(aux[q]));
    }
  }
  if (epi.res) {
    const uint16_t* rp = epi.res + (int64_t)gm * epi.ldres + gn;
    if (full && (((uintptr_t)rp) & 7) == 0) {
      const ushort4 a = *reinterpret_cast<const ushort4*>(rp);
      vv[0] += bf16_to_f32(a.x);
      vv[1] += bf16_to_f32(a.y);
      vv[2] += bf16_to_f32(a.z);
      vv[3] += bf16_to_f32(a.w);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (gn + q < N) vv[q] += bf16_to_f32(rp[q]);
    }
  }
  OutT* cp = C + (int64_t)gm * ldc + gn;
  if constexpr (sizeof(OutT) == 4) {
    float* fp = reinterpret_cast<float*>(cp);
    if (full && (((uintptr_t)fp) & 15) == 0) {
      float4 o = make_float4(vv[0], vv[1], vv[2], vv[3]);
      if (epi.accumulate) {
        const float4 old = *reinterpret_cast<float4*>(fp);
        o.x += old.x;
        o.y += old.y;
        o.z += old.z;
        o.w += old.w;
      }
      *reinterpret_cast<float4*>(fp) = o;
    } else {
      for (int q = 0; q < 4; ++q)
        if (gn + q < N) fp[q] = epi.accumulate ? fp[q] + vv[q] : vv[q];
    }
  } else {
    uint16_t* hp = reinterpret_cast<uint16_t*>(cp);
    if (full && (((uintptr_t)hp) & 7) == 0) {
      ushort4 o;
      o.x = f32_to_bf16(vv[0]);
      o.y = f32_to_bf16(vv[1]);
      o.z = f32_to_bf16(vv[2]);
      o.w = f32_to_bf16(vv[3]);
      *reinterpret_cast<ushort4*>(hp) = o;
    } else {
      for (int q = 0; q < 4; ++q)
        if (gn + q < N) hp[q] = f32_to_bf16(vv[q]);
    }
  }
}

}  // namespace mlt
