// Shared pieces of the bf16 GEMM kernels (gemm.hip: 128x128 general kernel,
// gemm_tile.hip: 256-wide global_load_lds kernels with split-K): epilogue parameters and
// the fused 4-column epilogue store.
#pragma once
#include <type_traits>

#include "mlt_common.h"

namespace mlt {

struct GemmEpi {
  const float* bias;     // [N] or nullptr
  const uint16_t* aux;   // GELU: pre-activation output (written); DGELU: pre-activation input (read)
  const uint16_t* res;   // residual [M,N] bf16 (added) or nullptr
  int64_t ldaux, ldres;
  float alpha;
  int mode;              // 0 none, 1 gelu (writes aux), 2 dgelu (reads aux), 3 tanh
  int accumulate;        // C += result (fp32 output only)
  const float* inv_scale_a = nullptr;  // fp8: device-side 1/scale of A and B (multiplied into alpha)
  const float* inv_scale_b = nullptr;
  // quantising ("q8") epilogue -- gemm_pp_kernel with OutT = uint8_t: C is the fp8 output [M,N];
  // the kernel also writes C^T, records amax of the (unscaled) output and optionally the column
  // partial sums (bias gradient of a dGELU output) -- the consumer GEMM's operands straight from
  // the producer, no bf16 round trip through HBM
  uint8_t* qt = nullptr;           // fp8 C^T [N, M], row stride ldqt
  int64_t ldqt = 0;
  const float* q_scale = nullptr;  // quantisation scale (device)
  float* q_amax = nullptr;         // kAmaxSlots amax slots of the output
  float* q_colpart = nullptr;      // [M / 64, N] fp32 column partial sums, or nullptr (also the bf16
                                   // pp kernel's dGELU epilogue: fused bias gradient)
  int q_fmt = 0;                   // 0 e4m3, 1 e5m2
};

// GELU and its derivative. Every epilogue evaluates them at bf16 points (the GELU input is the
// bf16-rounded pre-activation it also saves; the dGELU epilogue reads that bf16 tensor back), so
// they come from exact tables indexed by the bf16 bits (mlt_gelu_table.inc, scripts/gen_gelu_table.py):
// gelu_f / gelu_grad / gelu_pair_g from global memory, gelu_tab2 from an LDS copy (4-wave and
// quantising epilogues) -- one multiply by the same entry, so every path produces the same bits.
//
// The two-wide A&S 7.1.26 erf below is the build-switch alternative of the 4-wave and quantising
// epilogues (-DMLT_W4_GELU_TAB=0 / -DMLT_Q8_GELU_TAB=0, kept for their A/Bs): every
// non-transcendental step one v_pk_fma_f32 / v_pk_mul_f32 for two elements (~11 + 2
// transcendentals per element). q = Phi(-|x|) = 0.5 erfc(|x| / sqrt 2) = 0.5 poly(t) e^{-x^2/2}
// (the 0.5 and 1/sqrt 2 folded into the constants), then
//   gelu(x)  = x Phi(x) = relu(x) - |x| q
//   gelu'(x) = Phi(x) + x phi(x),  Phi(x) = 0.5 + copysign(0.5 - q, x),  phi(x) = e^{-x^2/2} / sqrt(2 pi)
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
// packed round-to-nearest-even f32 x 2 -> bf16 x 2 (one v_cvt_pk_bf16_f32), element 0 in the low half
__device__ __forceinline__ uint32_t cvt_pk_bf16(f32x2 v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}
__device__ __forceinline__ f32x2 unpack_bf16x2(uint32_t u) {
  return f32x2{__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
}
#include "mlt_gelu_table.inc"
// q = Phi(-|x|) of N pairs, step by step across the pairs (N independent chains in source order:
// a dependent packed op right behind its producer costs an s_nop on gfx950); also |x| and
// e^{-x^2/2}
template <int N>
__device__ __forceinline__ void phi_tail2(const f32x2 (&x)[N], f32x2 (&ax)[N], f32x2 (&e)[N], f32x2 (&q)[N]) {
  f32x2 t[N], h[N], arg[N];
#pragma unroll
  for (int i = 0; i < N; ++i) ax[i] = f32x2{fabsf(x[i].x), fabsf(x[i].y)};
#pragma unroll
  for (int i = 0; i < N; ++i) t[i] = pk_fma(ax[i], f32x2(0.3275911f * 0.70710678118654752f), f32x2(1.f));
#pragma unroll
  for (int i = 0; i < N; ++i) t[i] = f32x2{__builtin_amdgcn_rcpf(t[i].x), __builtin_amdgcn_rcpf(t[i].y)};
#pragma unroll
  for (int i = 0; i < N; ++i) arg[i] = x[i] * f32x2(-0.5f * 1.4426950408889634f);
#pragma unroll
  for (int i = 0; i < N; ++i) h[i] = pk_fma(t[i], f32x2(0.5f * 1.061405429f), f32x2(0.5f * -1.453152027f));
#pragma unroll
  for (int i = 0; i < N; ++i) arg[i] = arg[i] * x[i];
#pragma unroll
  for (int i = 0; i < N; ++i) h[i] = pk_fma(t[i], h[i], f32x2(0.5f * 1.421413741f));
#pragma unroll
  for (int i = 0; i < N; ++i) e[i] = f32x2{__builtin_amdgcn_exp2f(arg[i].x), __builtin_amdgcn_exp2f(arg[i].y)};
#pragma unroll
  for (int i = 0; i < N; ++i) h[i] = pk_fma(t[i], h[i], f32x2(0.5f * -0.284496736f));
#pragma unroll
  for (int i = 0; i < N; ++i) h[i] = pk_fma(t[i], h[i], f32x2(0.5f * 0.254829592f));
#pragma unroll
  for (int i = 0; i < N; ++i) h[i] = t[i] * h[i];
#pragma unroll
  for (int i = 0; i < N; ++i) q[i] = h[i] * e[i];
}
template <int N>
__device__ __forceinline__ void gelu2(f32x2 (&x)[N]) {
  f32x2 ax[N], e[N], q[N];
  phi_tail2<N>(x, ax, e, q);
#pragma unroll
  for (int i = 0; i < N; ++i) x[i] = pk_fma(-ax[i], q[i], (x[i] + ax[i]) * f32x2(0.5f));  // relu = (x + |x|) / 2
}
template <int N>
__device__ __forceinline__ void gelu_grad2(f32x2 (&x)[N]) {
  f32x2 ax[N], e[N], q[N];
  phi_tail2<N>(x, ax, e, q);
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const f32x2 r = f32x2(0.5f) - q[i];  // in [0, 0.5]: its sign bit is free for x's
    q[i] = f32x2(0.5f) + f32x2{copysignf(r.x, x[i].x), copysignf(r.y, x[i].y)};
  }
#pragma unroll
  for (int i = 0; i < N; ++i) x[i] = pk_fma(x[i] * f32x2(0.3989422804014327f), e[i], q[i]);
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
  } else if (epi.mode == 3) {  // tanh (BERT pooler)
#pragma unroll
    for (int q = 0; q < 4; ++q) vv[q] = tanhf(vv[q]);
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


// ---- prefetched epilogue side operands --------------------------------------------------------
// A tile's epilogue stores IT float4 groups per lane per pass. When the runtime epilogue mode needs
// a side operand (the dGELU pre-activation, a residual, or the fp32 accumulate target), loading it
// next to each store costs one dependent HBM round trip per group (hipcc waits vmcnt(0) at every use
// inside the mode branches). Instead the whole pass's side operands are loaded up front -- before
// the pass's accumulator -> LDS round trip, so that latency is hidden behind it -- and consumed from
// registers. kind: 0 = no side operand (plain epilogue_store4), 1 = one bf16 operand (aux in mode 2
// XOR res), 2 = fp32 accumulate target; -1 = combination / alignment without a fast path.
struct EpiSide {
  const uint16_t* x = nullptr;
  int64_t ldx = 0;
  int kind = 0;
};

template <typename OutT>
__device__ __forceinline__ EpiSide epi_side(const GemmEpi& epi, const OutT* C, int64_t ldc, int N, bool ext) {
  EpiSide s;
  if (ext) return s;
  const bool dg = epi.mode == 2, rs = epi.res != nullptr;
  if (dg && rs) {
    s.kind = -1;
  } else if (dg || rs) {
    s.x = dg ? epi.aux : epi.res;
    s.ldx = dg ? epi.ldaux : epi.ldres;
    s.kind = 1;
  }
  if (sizeof(OutT) == 4 && epi.accumulate) s.kind = s.kind == 0 ? 2 : -1;
  if (s.kind > 0) {
    const bool ok = N % 4 == 0 && ldc % 4 == 0 && (((uintptr_t)C) & 15) == 0 &&
                    (s.kind != 1 || (s.ldx % 4 == 0 && (((uintptr_t)s.x) & 7) == 0));
    if (!ok) s.kind = -1;
  }
  return s;
}

// One epilogue pass of EIT float4 groups per lane with a side operand, for a tile that lies wholly
// inside C (no range checks, no divergent branches: hipcc then counts the waits instead of
// draining vmcnt at every group). The first H groups' operands are loaded before `stage()` (the
// accumulator -> LDS round trip, barriers included); each later load re-fills the slot just
// consumed. H = EIT for the 2-VGPR bf16 operands; HF for the 4-VGPR fp32 accumulate target, which
// would otherwise spill kernels already at 256 VGPRs. `rc(it, gm, gn, off)` gives group it's
// output coordinates and its float offset in the staged LDS image.
enum { EPI_RES = 1, EPI_DGELU = 2, EPI_ACC = 3 };

// CS: also accumulate the lane's final values per column into csum[0..3] (the pass's 4 columns
// of a lane are fixed: column partial sums for a fused bias gradient).
template <int KIND, typename OutT, int EIT, int HF, bool CS = false, class RC, class STAGE>
__device__ __forceinline__ void epi_pass_side(OutT* __restrict__ C, int64_t ldc, const EpiSide& s, const float* cs,
                                              RC rc, STAGE stage, float* __restrict__ csum = nullptr) {
  constexpr int H = KIND == EPI_ACC ? HF : (EIT >= 8 ? EIT / 2 : EIT);
  using X = std::conditional_t<KIND == EPI_ACC, float4, ushort4>;
  X x[H];
  auto load = [&](int k, int it) __attribute__((always_inline)) {
    int gm, gn, off;
    rc(it, gm, gn, off);
    if constexpr (KIND == EPI_ACC)
      x[k] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(C) + (int64_t)gm * ldc + gn);
    else
      x[k] = *reinterpret_cast<const ushort4*>(s.x + (int64_t)gm * s.ldx + gn);
  };
#pragma unroll
  for (int it = 0; it < H; ++it) load(it, it);
  stage();
#pragma unroll
  for (int it = 0; it < EIT; ++it) {
    int gm, gn, off;
    rc(it, gm, gn, off);
    const int k = it % H;
    const float4 v = *reinterpret_cast<const float4*>(cs + off);
    float vv[4] = {v.x, v.y, v.z, v.w};
    OutT* cp = C + (int64_t)gm * ldc + gn;
    if constexpr (KIND == EPI_ACC) {
      const float4 o = x[k];
      *reinterpret_cast<float4*>(cp) = make_float4(vv[0] + o.x, vv[1] + o.y, vv[2] + o.z, vv[3] + o.w);
    } else {
      const ushort4 a = x[k];
      const float xv[4] = {bf16_to_f32(a.x), bf16_to_f32(a.y), bf16_to_f32(a.z), bf16_to_f32(a.w)};
#pragma unroll
      for (int q = 0; q < 4; ++q) vv[q] = KIND == EPI_DGELU ? vv[q] * gelu_grad(xv[q]) : vv[q] + xv[q];
      if constexpr (CS) {
#pragma unroll
        for (int q = 0; q < 4; ++q) csum[q] += vv[q];
      }
      if constexpr (sizeof(OutT) == 4) {
        *reinterpret_cast<float4*>(cp) = make_float4(vv[0], vv[1], vv[2], vv[3]);
      } else {
        ushort4 o;
        o.x = f32_to_bf16(vv[0]);
        o.y = f32_to_bf16(vv[1]);
        o.z = f32_to_bf16(vv[2]);
        o.w = f32_to_bf16(vv[3]);
        *reinterpret_cast<ushort4*>(cp) = o;
      }
    }
    if (it + H < EIT) load(k, it + H);
  }
}

// which side-operand pass a tile takes (0 = the general epilogue)
template <typename OutT>
__device__ __forceinline__ int epi_side_kind(const EpiSide& s, const GemmEpi& epi, bool interior) {
  if (s.kind <= 0 || !interior) return 0;
  if (s.kind == 1) return epi.mode == 2 ? EPI_DGELU : EPI_RES;
  return sizeof(OutT) == 4 ? EPI_ACC : 0;
}

// 16-byte-store epilogue pass for bf16 outputs without a side operand (plain / GELU + saved
// pre-activation / tanh) of a tile wholly inside C: each lane takes 8 consecutive columns of the
// staged fp32 image (two float4 LDS reads) and writes them with ONE 16-byte store (two for GELU:
// pre-activation + output). The epilogue's store tail is issue-bound (MI355X_MICROARCH.md: store
// tail; cdna_hip_programming.md T21), so half the store instructions of the 8-byte-per-group
// path. `rc8(it, gm, gn, off)` gives group it's output coordinates / image offset (off % 4 == 0).
__device__ __forceinline__ bool epi_store8_ok(const GemmEpi& epi, const void* C, int64_t ldc, int N, bool interior,
                                              bool ext) {
  if (ext || !interior || epi.res || epi.accumulate || epi.mode == 2 || N % 8 || ldc % 8 ||
      (((uintptr_t)C) & 15))
    return false;
  return epi.mode != 1 || (epi.ldaux % 8 == 0 && (((uintptr_t)epi.aux) & 15) == 0);
}

__device__ __forceinline__ uint4 pack_bf16x8(const float (&v)[8]) {
  return make_uint4(cvt_pk_bf16(f32x2{v[0], v[1]}), cvt_pk_bf16(f32x2{v[2], v[3]}), cvt_pk_bf16(f32x2{v[4], v[5]}),
                    cvt_pk_bf16(f32x2{v[6], v[7]}));
}

template <int MODE, int EIT8, class RC8>
__device__ __forceinline__ void epi_store8_loop(uint16_t* __restrict__ C, int64_t ldc, const GemmEpi& epi,
                                                const float* cs, RC8 rc8) {
#pragma unroll 4
  for (int it = 0; it < EIT8; ++it) {
    int gm, gn, off;
    rc8(it, gm, gn, off);
    const float4 a = *reinterpret_cast<const float4*>(cs + off);
    const float4 b = *reinterpret_cast<const float4*>(cs + off + 4);
    float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    if constexpr (MODE == 1) {
      const uint4 pre = pack_bf16x8(v);
      *reinterpret_cast<uint4*>(const_cast<uint16_t*>(epi.aux) + (int64_t)gm * epi.ldaux + gn) = pre;
      const f32x2 x2[4] = {gelu_pair_g(pre.x), gelu_pair_g(pre.y), gelu_pair_g(pre.z), gelu_pair_g(pre.w)};
#pragma unroll
      for (int q = 0; q < 4; ++q) v[2 * q] = x2[q].x, v[2 * q + 1] = x2[q].y;
    } else if constexpr (MODE == 3) {
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = tanhf(v[q]);
    }
    *reinterpret_cast<uint4*>(C + (int64_t)gm * ldc + gn) = pack_bf16x8(v);
  }
}

template <int EIT8, class RC8>
__device__ __forceinline__ void epi_store8(uint16_t* __restrict__ C, int64_t ldc, const GemmEpi& epi, const float* cs,
                                           RC8 rc8) {
  if (epi.mode == 1)
    epi_store8_loop<1, EIT8>(C, ldc, epi, cs, rc8);
  else if (epi.mode == 3)
    epi_store8_loop<3, EIT8>(C, ldc, epi, cs, rc8);
  else
    epi_store8_loop<0, EIT8>(C, ldc, epi, cs, rc8);
}

}  // namespace mlt
