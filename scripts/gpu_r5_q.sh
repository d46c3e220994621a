# (the device step limit / limited-replay build this A/B measured was reverted: see profiles/README.md)
# Device step limit (ctrl[2]) + warmup through the timed graph (bench: limited replay): LeNet GPU
# tests on the new build (bitwise limited-replay test included), then a same-box A/B:
#   new/old .so with --steps-per-graph 5 (the previous flow: kernel-side cost of the limit checks)
#   new .so, default flow (one 20-step graph, warmed by the limited replay) vs --steps-per-graph 5
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0 && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5q
mkdir -p $O
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_lenet_bf16.py tests/test_lenet_native.py tests/test_multiproc_gpu.py tests/test_trainer_parallel_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
[ -n "${SKIP_TESTS:-}" ] || tail -1 $O/tests.log
# the 2-rank data-parallel bench on the one GPU (warmup through the limited replay at W > 1)
MLT_BENCH_BACKEND=gloo MLT_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 20 --warmup 5 --no-fp32-companion \
  > $O/dp2.log 2>&1 || { tail -30 $O/dp2.log; exit 1; }
grep '^{' $O/dp2.log | cut -c1-400
bash scripts/ab_so.sh "python bench.py --steps 20 --warmup 5 --steps-per-graph 5 --no-fp32-companion" \
  "python bench.py --steps 20 --warmup 5 --no-fp32-companion" "python bench.py --no-fp32-companion" \
  "python bench.py --batch 4 --steps 20 --warmup 5 --no-fp32-companion" || exit 1
cp gpurun_out/ab.jsonl $O/ab.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/r5q/ab.jsonl"):
    d = json.loads(l); o = json.loads(d["out"])
    print(d["variant"], d["cmd"][13:70], o["value"], o["ms_per_step"], o["config"].get("hipgraph_steps"))
PY
