"""bench.py contract on CPU: the self-launch of N ranks and the no-capture-in-the-timed-region
guarantee (the round-1 driver bench measured graph capture instead of steps)."""
import json
import os
import subprocess
import sys

import pytest

import bench
from ml_trainer_amd.models.lenet_engine import LeNetStepEngine
from ml_trainer_amd.parallel.sampler import shard_indices

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _FakeCEngine:
    """Stands in for _C.LeNetEngine: records captures and replays."""

    def __init__(self):
        self.graphs = set()
        self.replayed = []

    def has_graph(self, mode, B, k):
        return (mode, B, k) in self.graphs

    def capture(self, mode, B, k):
        self.graphs.add((mode, B, k))

    def replay(self, mode, B, k):
        assert (mode, B, k) in self.graphs
        self.replayed.append((B, k))

    def run(self, mode, B):
        self.replayed.append((B, 1))

    def flush(self):
        pass


class _FakeC:
    LENET_FWD, LENET_CE, LENET_BWD, LENET_OPT, LENET_REDUCE = 1, 2, 4, 8, 16


def _fake_engine():
    e = object.__new__(LeNetStepEngine)
    e.C = _FakeC
    e.eng = _FakeCEngine()
    e.world_size = 1
    e.dp_transport = "none"
    e.precision = "fp32"
    e.captures = 0
    e.comm = e.xgmi = None
    return e


@pytest.mark.parametrize("steps,warmup,n_data,world,per_gpu", [
    (20, 5, 50000, 1, 32),      # the driver's call
    (3000, 300, 50000, 1, 32),  # crosses an epoch boundary (1563 steps/epoch, partial last batch)
    (7, 1, 100, 1, 32),         # tiny dataset: several epochs, partial batches
    (40, 3, 1000, 4, 8),        # sharded
])
def test_precapture_covers_timed_region(steps, warmup, n_data, world, per_gpu):
    eng = _fake_engine()
    spg = max(1, min(64, steps))
    state = {"epoch": 0, "shard_len": 0, "step_in_epoch": 0, "steps_per_epoch": 0}

    def run(n):
        done = 0
        for ev in bench.lenet_plan(n, state, n_data, world, 0, per_gpu, spg, shard_indices):
            if ev[0] == "steps":
                eng.train_steps(ev[1], ev[2], use_graph=True, steps_per_graph=ev[3])
                done += ev[2]
        return done

    assert run(warmup) == warmup
    bench.precapture(eng, bench.lenet_plan(steps, dict(state), n_data, world, 0, per_gpu, spg, shard_indices),
                     True)
    before = eng.captures
    n_replayed = len(eng.eng.replayed)
    assert run(steps) == steps
    assert eng.captures == before, "graph captured inside the timed region"
    assert sum(k for _, k in eng.eng.replayed[n_replayed:]) == steps


def test_driver_shape_is_one_replay():
    eng = _fake_engine()
    mode = 1 | 2 | 4 | 8  # fwd | ce | bwd | fused optimizer
    assert eng.graph_shapes(32, 20, True, 20) == [(mode, 32, 20)]
    assert eng.graph_shapes(32, 3000, True, 64) == [(mode, 32, 64), (mode, 32, 56)]


def test_bench_self_launch_two_ranks_gloo():
    env = dict(os.environ, MLT_BENCH_BACKEND="gloo", OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu",
                        "--steps", "4", "--warmup", "1"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 4 and out["warmup"] == 1
    assert out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 64
    assert out["config"]["loss_finite"]
    for k in ("metric", "value", "unit", "ms_per_step", "higher_is_better", "scaling", "vs_baseline", "dtype",
              "data"):
        assert k in out


def test_debug_checks_compile_for_gfx950():
    """-DMLT_DEBUG turns MLT_DCHECK into device printf checks in the LeNet / GEMM / attention
    index math; they must parse for host and gfx950 device (syntax-only compile, no codegen)."""
    import subprocess
    import shutil
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc")
    inc = os.path.join(ROOT, "ml_trainer_amd", "csrc", "include")
    for f in ("lenet.hip", "gemm_tile.hip", "attention.hip"):
        src = os.path.join(ROOT, "ml_trainer_amd", "csrc", "kernels", f)
        r = subprocess.run([hipcc, "-fsyntax-only", "-std=c++17", "--offload-arch=gfx950", "-DMLT_DEBUG=1",
                            f"-I{inc}", src], capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
        txt = open(src).read()
        assert "MLT_DCHECK(" in txt
