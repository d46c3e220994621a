"""CPU checks of the GEMM epilogues' table GELU (csrc/include/mlt_gelu_table.inc: gelu_tab2 from LDS in
the 4-wave / quantising epilogues, gelu_f / gelu_grad / gelu_pair_g from global memory elsewhere):
the committed include is exactly the generator's output, and the device index sequence (16-bit
packed saturating subtract / min / sign offset), replayed in numpy over EVERY bf16 bit pattern,
gives GELU and GELU' within 1e-6 absolute of the float64 erf forms."""
import importlib.util
import math
import os
import re

import numpy as np
from scipy.special import erfc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "ml_trainer_amd", "csrc", "include", "mlt_gelu_table.inc")


def _gen():
    spec = importlib.util.spec_from_file_location("gen_gelu_table", os.path.join(ROOT, "scripts", "gen_gelu_table.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _tables():
    src = open(INC).read()
    out = {}
    for name in ("kGeluPhiTab", "kGeluGradTab"):
        body = re.search(name + r"\[\d+\] = \{(.*?)\};", src, re.S).group(1)
        words = np.array([int(w, 16) for w in re.findall(r"0x([0-9a-f]{8})u", body)], dtype=np.uint32)
        out[name] = words.view(np.float32)
    return out


def _device_index(bits: np.ndarray, lo: int, nr: int) -> np.ndarray:
    """gelu_tab2's index arithmetic on uint16 lanes (byte offset / 4)."""
    u = bits.astype(np.int64)
    sg = u >> 15
    i = np.maximum((u & 0x7FFF) - (lo - 1), 0)  # v_pk_sub_u16 with clamp
    i = np.minimum(i, nr + 1)                   # v_pk_min_u16
    return i + sg * (nr + 2)


def test_committed_include_matches_generator(tmp_path, monkeypatch):
    g = _gen()
    out = tmp_path / "gelu_table.inc"
    monkeypatch.setattr(g, "OUT", str(out))
    g.main()
    assert out.read_text() == open(INC).read(), "re-run scripts/gen_gelu_table.py"


def test_table_gelu_matches_erf_at_every_bf16_point():
    g = _gen()
    tabs = _tables()
    bits = np.arange(1 << 16, dtype=np.uint32)
    x = (bits << 16).view(np.float32)
    fin = np.isfinite(x)
    bits, x = bits[fin], x[fin]
    idx = _device_index(bits, g.LO, g.NR)
    assert idx.max() < g.ENTRIES and 4 * idx.max() < (1 << 16)  # byte offsets fit the 16-bit lanes
    gelu = (x * tabs["kGeluPhiTab"][idx]).astype(np.float32)
    grad = tabs["kGeluGradTab"][idx]
    xd = x.astype(np.float64)
    cdf = 0.5 * erfc(-xd / math.sqrt(2.0))  # no cancellation in the negative tail
    g_ref = xd * cdf
    gp_ref = cdf + xd * np.exp(-0.5 * xd * xd) / math.sqrt(2.0 * math.pi)
    assert np.max(np.abs(gelu - g_ref)) < 1e-6
    assert np.max(np.abs(grad - gp_ref)) < 1e-6
    # inside the table range (2^-20 <= |x| < 8) the multiplier is the correctly rounded f32 value:
    # relative error of the product at the f32 rounding level
    inr = (np.abs(x) >= 2.0 ** -20) & (np.abs(x) < 8.0)
    assert np.max(np.abs(gelu - g_ref)[inr] / np.abs(g_ref[inr])) < 2 ** -22
    # the covered range and the sentinels
    assert tabs["kGeluPhiTab"][0] == 0.5 and tabs["kGeluGradTab"][0] == 0.5
    assert tabs["kGeluPhiTab"][g.NR + 1] == 1.0 and tabs["kGeluPhiTab"][g.ENTRIES - 1] == 0.0
    assert gelu[x == 12.0][0] == 12.0 and gelu[x == -12.0][0] == 0.0


def test_kernels_use_the_generated_layout():
    inc = open(INC).read()
    # the packed (LDS) index and the scalar (global) index are the same function of the bits
    assert "__builtin_elementwise_sub_sat(u & (u16x2)0x7fff, (u16x2)(MLT_GELU_TAB_LO - 1))" in inc
    assert "__builtin_elementwise_min(i, (u16x2)(MLT_GELU_TAB_NR + 1))" in inc
    assert "sg * (u16x2)(4 * (MLT_GELU_TAB_NR + 2))" in inc
    assert "m > MLT_GELU_TAB_LO - 1 ? min(m - (MLT_GELU_TAB_LO - 1), (uint32_t)MLT_GELU_TAB_NR + 1) : 0u" in inc
    assert "i + (b >> 15) * (MLT_GELU_TAB_NR + 2)" in inc
    hdr = open(os.path.join(ROOT, "ml_trainer_amd", "csrc", "include", "mlt_gemm.h")).read()
    assert '#include "mlt_gelu_table.inc"' in hdr
    w4 = open(os.path.join(ROOT, "ml_trainer_amd", "csrc", "kernels", "gemm_w4.hip")).read()
    pp = open(os.path.join(ROOT, "ml_trainer_amd", "csrc", "kernels", "gemm_tile.hip")).read()
    assert "gelu_tab2(a[q2], smem + kW4Smem)" in w4 and "gelu_tab2(sw4[q2], smem + kW4Smem)" in w4
    assert "gelu_tab2(pr[4 * hh + q], tab)" in pp and "gelu_tab2(w[4 * hh + q], tab)" in pp
