# LeNet bf16 per-sample kernel with the fc3 forward image staged into LDS in P1 (in-tree) vs the
# previous build (ab/): the LeNet GPU tests on the new build, then a same-box A/B of the steady
# state (b32, b4) and the driver protocol.
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5m
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_lenet_bf16.py tests/test_lenet_native.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/ab_so.sh "python bench.py --no-fp32-companion" "python bench.py --batch 4 --no-fp32-companion" \
  "python bench.py --steps 20 --warmup 5 --no-fp32-companion" || exit 1
cp gpurun_out/ab.jsonl $O/ab.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/r5m/ab.jsonl"):
    d = json.loads(l); o = json.loads(d["out"])
    print(d["variant"], d["cmd"][:40], o["value"], o["ms_per_step"])
PY
