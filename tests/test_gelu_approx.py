"""CPU check of the two-wide A&S GELU / GELU' formula (mlt_gemm.h: phi_tail2 / gelu2 / gelu_grad2), the
build-switch alternative of the 4-wave and quantising epilogues (-DMLT_W4_GELU_TAB=0 /
-DMLT_Q8_GELU_TAB=0); the default epilogues use the exact tables (tests/test_gelu_table.py).

The device code evaluates erf by Abramowitz & Stegun 7.1.26 with the 0.5 and 1/sqrt(2) folded
into the constants:
    q = Phi(-|x|) = t * h(t) * exp2(-x^2 log2(e) / 2),  t = 1 / (1 + p |x| / sqrt 2)
    gelu(x)  = fma(-|x|, q, (x + |x|) / 2)
    gelu'(x) = fma(x / sqrt(2 pi), e^{-x^2/2}, 0.5 + copysign(0.5 - q, x))
This test replays that sequence in float32 numpy (exact division / exp2 standing in for v_rcp /
v_exp, which are within 1 ulp) and bounds its error against the exact erf GELU, so a change of a
constant or of the sequence in the header has a reference to fail against.
"""
import math
from pathlib import Path

import numpy as np
from scipy.special import erf

HDR = Path(__file__).resolve().parents[1] / "ml_trainer_amd" / "csrc" / "include" / "mlt_gemm.h"


def _device_gelu(x):
    f = np.float32
    ax = np.abs(x)
    t = f(1) / (ax * f(0.3275911 * 0.70710678118654752) + f(1))
    h = t * f(0.5 * 1.061405429) + f(0.5 * -1.453152027)
    h = t * h + f(0.5 * 1.421413741)
    h = t * h + f(0.5 * -0.284496736)
    h = t * h + f(0.5 * 0.254829592)
    e = np.exp2((x * f(-0.5 * 1.4426950408889634)) * x).astype(np.float32)
    q = (t * h) * e
    gelu = -ax * q + (x + ax) * f(0.5)
    grad = (x * f(0.3989422804014327)) * e + (f(0.5) + np.copysign(f(0.5) - q, x))
    return gelu.astype(np.float32), grad.astype(np.float32)


def test_gelu_formula_matches_exact_erf_gelu():
    x = np.linspace(-12.0, 12.0, 480001, dtype=np.float32)
    g, gp = _device_gelu(x)
    xd = x.astype(np.float64)
    cdf = 0.5 * (1.0 + erf(xd / math.sqrt(2.0)))
    g_ref = xd * cdf
    gp_ref = cdf + xd * np.exp(-0.5 * xd * xd) / math.sqrt(2.0 * math.pi)
    assert np.max(np.abs(g - g_ref)) < 1e-6
    assert np.max(np.abs(gp - gp_ref)) < 1e-6
    # far below a bf16 ulp wherever the output is representable at bf16 precision
    big = np.abs(g_ref) > 1e-2
    assert np.max(np.abs(g - g_ref)[big] / np.abs(g_ref[big])) < 2 ** -12
    # the tails: gelu(-12) ~ -2e-32 (no NaN / inf from the exp2 underflow), gelu(12) = 12, gelu' -> 0 / 1
    assert abs(g[0]) < 1e-30 and g[-1] == np.float32(12.0)
    assert abs(gp[0]) < 1e-29 and gp[-1] == 1.0
    assert np.all(np.isfinite(g)) and np.all(np.isfinite(gp))


def test_header_carries_the_tested_constants():
    src = HDR.read_text()
    for c in ("0.3275911f", "1.061405429f", "-1.453152027f", "1.421413741f", "-0.284496736f", "0.254829592f",
              "0.3989422804014327f", "1.4426950408889634f"):
        assert src.count(c) >= 1, c  # the two-wide form (the scalar paths use the exact tables)
    assert "pk_fma(-ax[i], q[i], (x[i] + ax[i]) * f32x2(0.5f))" in src
