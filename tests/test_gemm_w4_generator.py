"""The committed main loops of the 4-wave GEMM (csrc/kernels/gemm_w4_loop.inc) are exactly what
scripts/gen_gemm_w4.py emits, and the schedule keeps its structural invariants (CPU only)."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gen():
    spec = importlib.util.spec_from_file_location("gen_gemm_w4", os.path.join(ROOT, "scripts", "gen_gemm_w4.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_committed_include_matches_generator(tmp_path, monkeypatch):
    g = _gen()
    out = tmp_path / "gemm_w4_loop.inc"
    monkeypatch.setattr(g, "OUT", str(out))
    g.main()
    committed = open(os.path.join(ROOT, "ml_trainer_amd", "csrc", "kernels", "gemm_w4_loop.inc")).read()
    assert out.read_text() == committed, "re-run scripts/gen_gemm_w4.py"


def test_schedule_invariants():
    g = _gen()
    for name, lines, per_tile in (("tn", g.build(), 128), ("bn", g.build(bn=True), 128),
                                  ("anbn", g.build(bn=True, an=True), 128), ("f8", g.build_f8(), 64)):
        mf = [l for l in lines if "v_mfma" in l]
        assert len(mf) % per_tile == 0, name
        # one barrier per K-tile (+ the prologue's), never an s_waitcnt vmcnt(0) outside the barriers
        bars = sum(1 for l in lines if l == "s_barrier")
        assert bars == len(mf) // per_tile + 1, (name, bars)
        # the first K-tile starts from C = 0 and nothing zeroes the accumulators
        assert not any(l.startswith("v_accvgpr_write") for l in lines), name
        assert mf[0].endswith(", 0") or " 0, v192" in mf[0], name
        # every LDS-DMA piece is preceded by its M0 write
        for i, l in enumerate(lines):
            if l.startswith("global_load_lds"):
                assert lines[i - 1].startswith("s_add_u32 m0"), (name, i)
        # scalar instructions: a fixed whitelist (moves / arithmetic / compare / branch / waits /
        # barrier / nop): all memory writes of the generated code are vector instructions
        allowed = ("s_mov_b32", "s_mov_b64", "s_add_u32", "s_addc_u32", "s_sub_u32", "s_cmp_eq_u32",
                   "s_cmp_lg_u32", "s_cbranch_scc1", "s_waitcnt", "s_barrier", "s_nop")
        for l in lines:
            if l.startswith("s_"):
                assert l.split()[0] in allowed, (name, l)
