"""Generate the exact GELU / GELU' lookup tables of the 4-wave GEMM's epilogues
(csrc/include/mlt_gelu_table.inc, included by mlt_gemm.h: EVERY GELU / GELU' GEMM epilogue -- the
4-wave kernel's and the quantising epilogue's from an LDS copy, the scalar / split-K / general paths
from global memory -- multiplies by the same table entry, so they all produce the same bits).

Why a table: the GELU epilogue's input is the bf16-ROUNDED pre-activation (the value it also saves
for the backward), and the dGELU epilogue reads that same bf16 tensor, so the function is only ever
evaluated at bf16 points. The A&S 7.1.26 erf (mlt_gemm.h gelu2 / gelu_grad2) costs ~11 packed f32
ops + 4 transcendentals per element pair and makes these epilogues VALU-bound (819 / 831 TF vs
1,090 for the plain epilogue at 256 K tokens, profiles/r4/gemm_epi_262k_final.jsonl). A table
indexed by the bf16 bits is exact (float64 erf rounded once to f32) and costs ~8 16-bit-packed
integer ops + 2 LDS reads + 1 packed multiply per pair.

Layout (one table per function, 5,892 f32 = 23,568 B, copied to LDS once per workgroup):
  entry j = s * (NR + 2) + i   s = the bf16 sign bit
    i = 0            |x| < 2^-20          multiplier 0.5        (x Phi(x) = x/2 + O(x^2): < 1e-12)
    i = 1 .. NR      bf16 magnitude bits LO + i - 1, i.e. |x| in [2^-20, 8) (23 binades x 128)
    i = NR + 1       |x| >= 8, inf, nan   multiplier 1 (x > 0) / 0 (x < 0)
  GELU table: Phi(x)  (gelu(x) = x * T[j], one multiply);  GELU' table: Phi(x) + x phi(x).
The device index is min(sat_sub(bits & 0x7fff, LO - 1), NR + 1) + s (NR + 2), on both halves of a
bf16 pair at once (v_pk_sub_u16 clamp / v_pk_min_u16 / v_pk_mad_u16).

Usage: python scripts/gen_gelu_table.py  (rewrites the .inc: tables + the device lookups)
"""
import math
import os
import struct

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "ml_trainer_amd", "csrc", "include", "mlt_gelu_table.inc")

E_LO, E_HI = 107, 130            # bf16 biased exponents covered: [2^-20, 2^3)
LO = E_LO << 7                   # first covered magnitude bit pattern
NR = (E_HI - E_LO) << 7          # covered magnitudes per sign
PER_SIGN = NR + 2
ENTRIES = 2 * PER_SIGN


def bf16_value(bits: int) -> float:
    return struct.unpack("<f", struct.pack("<I", bits << 16))[0]


def f32_bits(v: float) -> int:
    return struct.unpack("<I", struct.pack("<f", v))[0]


def phi_cdf(x: float) -> float:
    return 0.5 * math.erfc(-x / math.sqrt(2.0))


def gelu_grad(x: float) -> float:
    return phi_cdf(x) + x * math.exp(-0.5 * x * x) / math.sqrt(2.0 * math.pi)


def table(fn):
    out = []
    for s in (0, 1):
        out.append(0.5)  # |x| < 2^-20
        for i in range(1, NR + 1):
            x = bf16_value((s << 15) | (LO + i - 1))
            out.append(fn(x))
        out.append(0.0 if s else 1.0)  # |x| >= 8
    assert len(out) == ENTRIES
    return out


DEVICE_HELPERS = r"""
constexpr int kGeluTabBytes = MLT_GELU_TAB_ENTRIES * 4;
// workgroup copy of one table (grad: GELU' instead of Phi) into LDS at dst (16-byte aligned)
__device__ __forceinline__ void gelu_tab_load(uint8_t* dst, bool grad, int nthreads) {
  const uint4* src = reinterpret_cast<const uint4*>(grad ? kGeluGradTab : kGeluPhiTab);
  for (int i = threadIdx.x; i < kGeluTabBytes / 16; i += nthreads) reinterpret_cast<uint4*>(dst)[i] = src[i];
}
// table multipliers of a bf16 pair (element 0 in the low half): index = min(sat(|bits| - (LO - 1)),
// NR + 1) + sign (NR + 2), both halves at once in 16-bit packed integer ops, then one LDS read each
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu_tab2(uint32_t u2, const uint8_t* tab) {
  const u16x2 u = __builtin_bit_cast(u16x2, u2);
  const u16x2 sg = u >> (u16x2)15;
  u16x2 i = __builtin_elementwise_sub_sat(u & (u16x2)0x7fff, (u16x2)(MLT_GELU_TAB_LO - 1));
  i = __builtin_elementwise_min(i, (u16x2)(MLT_GELU_TAB_NR + 1));
  i = i * (u16x2)4 + sg * (u16x2)(4 * (MLT_GELU_TAB_NR + 2));
  const uint32_t w = __builtin_bit_cast(uint32_t, i);
  return f32x2{*reinterpret_cast<const float*>(tab + (w & 0xffffu)), *reinterpret_cast<const float*>(tab + (w >> 16))};
}
// the same index for one bf16 (bits b), and the scalar / two-wide lookups from global memory (the
// general, persistent and split-K-reduce epilogues: L1/L2-resident table, no LDS copy)
__device__ __forceinline__ uint32_t gelu_tab_index(uint32_t b) {
  const uint32_t m = b & 0x7fffu;
  const uint32_t i = m > MLT_GELU_TAB_LO - 1 ? min(m - (MLT_GELU_TAB_LO - 1), (uint32_t)MLT_GELU_TAB_NR + 1) : 0u;
  return i + (b >> 15) * (MLT_GELU_TAB_NR + 2);
}
// GELU(x) and GELU'(x) of a bf16 value x (the low 16 bits of its f32 pattern are zero)
__device__ __forceinline__ float gelu_f(float x) {
  return x * __uint_as_float(kGeluPhiTab[gelu_tab_index(__float_as_uint(x) >> 16)]);
}
__device__ __forceinline__ float gelu_grad(float x) {
  return __uint_as_float(kGeluGradTab[gelu_tab_index(__float_as_uint(x) >> 16)]);
}
// GELU of a packed bf16 pair (element 0 in the low half), from global memory
__device__ __forceinline__ f32x2 gelu_pair_g(uint32_t u2) {
  const f32x2 x = unpack_bf16x2(u2);
  return x * f32x2{__uint_as_float(kGeluPhiTab[gelu_tab_index(u2 & 0xffffu)]),
                   __uint_as_float(kGeluPhiTab[gelu_tab_index(u2 >> 16)])};
}"""


def main():
    lines = ["// generated by scripts/gen_gelu_table.py -- do not edit",
             f"// exact GELU multiplier Phi(x) and GELU'(x) at every bf16 x (layout: see the generator)",
             f"#define MLT_GELU_TAB_LO {LO}",
             f"#define MLT_GELU_TAB_NR {NR}",
             f"#define MLT_GELU_TAB_ENTRIES {ENTRIES}"]
    for name, fn in (("kGeluPhiTab", phi_cdf), ("kGeluGradTab", gelu_grad)):
        vals = [f32_bits(v) for v in table(fn)]
        # static: every kernel file that includes the tables gets its own copy (no host-side
        # duplicate of the __device__ symbol's shadow at link time)
        lines.append(f"static __device__ __attribute__((aligned(16))) const unsigned {name}[{ENTRIES}] = {{")
        for k in range(0, ENTRIES, 8):
            lines.append("    " + ", ".join(f"0x{v:08x}u" for v in vals[k:k + 8]) + ",")
        lines.append("};")
    lines += DEVICE_HELPERS.splitlines()
    with open(OUT, "w") as f:
        f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
