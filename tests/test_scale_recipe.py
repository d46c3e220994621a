"""The node recipe (scripts/scale_curve.sh) covers every BASELINE.json DDP config."""
import os
import re
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(REPO, "scripts", "scale_curve.sh")


def _lines():
    src = open(SCRIPT).read()
    # the `line CONFIG SECTION N LIMIT [ENV...] -- ARGS` calls, joined across continuation lines
    src = re.sub(r"\\\n\s*", " ", src)
    return src, [l.strip() for l in src.splitlines() if l.strip().startswith("line ")]


def test_script_parses():
    assert subprocess.run(["bash", "-n", SCRIPT]).returncode == 0


def test_configs_3_4_5_and_rccl_sweep_present():
    src, lines = _lines()
    cfgs = {l.split()[1] for l in lines}
    assert {"2-3", "3", "4", "5"} <= cfgs
    # config 3: LeNet at N = 8 under the reference's semantics (global batch 32 split over the ranks)
    assert 'NS="1 2 4 8"' in src and "for scaling in weak reference" in src
    # config 4: BERT-base over N (the loop), DDP with auto-planned buckets (no --bucket-mb) + ZeRO-1 A/B
    bert = [l for l in lines if l.split()[1] == "4" and "bert_base" in l]
    assert any("--model bert-base" in l and "--bucket-mb" not in l for l in bert)
    assert any("--zero 1" in l for l in bert)
    # config 5: the fp8 `large` model at DDP = 8 with gradient accumulation, and its ZeRO-1 A/B
    c5 = [l for l in lines if l.split()[1] == "5"]
    assert c5 and all("--model large" in l for l in c5) and any("--zero 1" in l for l in c5)
    assert "N5=8" in src and "$N5" in " ".join(c5)
    m = re.search(r'LARGE_B="--batch (\d+) --grad-accum (\d+)"', src)
    assert m and int(m.group(1)) == 512 and int(m.group(2)) > 1
    # RCCL sweep: channels x algorithm x protocol as environment variables of the bench process
    assert re.search(r"for ch in 8 16 32 64", src)
    assert re.search(r"for algo in Ring Tree", src) and re.search(r"for proto in Simple LL128", src)
    sweep = [l for l in lines if "rccl_sweep" in l][0]
    for k in ("NCCL_MIN_NCHANNELS=$ch", "NCCL_MAX_NCHANNELS=$ch", "NCCL_ALGO=$algo", "NCCL_PROTO=$proto"):
        assert k in sweep
    assert "--model bert-base" in sweep
