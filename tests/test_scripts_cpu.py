"""Static checks of the GPU run recipes (no GPU): every rocprofv3 invocation puts the program it
profiles DIRECTLY after `--` (no launcher, shell or env hop behind the profiler), and a multi-rank
bench is profiled per rank with the launcher outside the profiler (scripts/prof_rank.sh)."""
import glob
import os
import re
import shlex

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOPS = {"env", "bash", "sh", "taskset", "numactl", "torchrun", "timeout", "nohup"}


def _logical_lines(path):
    buf = ""
    for line in open(path):
        line = line.rstrip("\n")
        if line.endswith("\\"):
            buf += line[:-1] + " "
            continue
        yield buf + line
        buf = ""


def _rocprof_cmds(path):
    for line in _logical_lines(path):
        code = line.split("#", 1)[0]
        if "rocprofv3" not in code:
            continue
        try:
            toks = shlex.split(code)
        except ValueError:
            continue
        for i, t in enumerate(toks):
            if t == "rocprofv3":
                yield toks[i + 1:]


def test_every_rocprof_runs_the_program_directly():
    found = 0
    for path in glob.glob(os.path.join(ROOT, "scripts", "*.sh")):
        for args in _rocprof_cmds(path):
            if "--" not in args:
                continue
            prog = args[args.index("--") + 1:]
            found += 1
            assert prog, path
            head = os.path.basename(prog[0].strip('"'))
            assert head not in HOPS, (path, prog[:3])
            assert not (head == "python3" and len(prog) > 2 and prog[1] == "-m"
                        and prog[2].startswith("torch.distributed")), (path, prog[:4])
            # a multi-rank bench under one profiler would self-launch its ranks behind it
            if any(os.path.basename(p) == "bench.py" for p in prog):
                m = re.search(r"--gpus\s+(\S+)", " ".join(prog))
                gpus = m.group(1) if m else "1"
                assert gpus == "1" or "prof_rank.sh" in path, (path, prog)
    assert found >= 1


def test_n8_trace_launcher_outside_profiler():
    lines = [l for l in _logical_lines(os.path.join(ROOT, "scripts", "scale_curve.sh"))
             if "prof_n8" in l and "bench.py" in l and not l.lstrip().startswith("#")]
    assert len(lines) == 1, lines
    toks = shlex.split(lines[0])
    assert "rocprofv3" not in toks  # the profiler is exec'ed per rank by prof_rank.sh
    i = toks.index("torch.distributed.run")
    assert "--no-python" in toks[i:]
    w = [j for j, t in enumerate(toks) if t.endswith("prof_rank.sh")]
    assert w and w[0] > i
    after = toks[toks.index("--", w[0]) + 1:]
    assert after[0] == "python3" and "bench.py" in after and "--gpus" in after
    wrap = open(os.path.join(ROOT, "scripts", "prof_rank.sh")).read()
    execs = [l for l in wrap.splitlines() if l.startswith("exec ")]
    assert len(execs) == 1 and execs[0].startswith("exec rocprofv3 ") and execs[0].rstrip().endswith('-- "$@"')
    assert "WORLD_SIZE:?" in wrap and "LOCAL_RANK:?" in wrap
