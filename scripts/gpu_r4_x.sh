#!/bin/bash
# Round 4: conv1 forward wave count (kC1W 8 / 13 / 16) on the per-sample LeNet kernel: bf16 tests per
# build, then alternated benches over ab/*.so (scripts/ab_multi_so.sh), same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4x
mkdir -p $O
SO=$(ls ml_trainer_amd/_C*.so)
cp "$SO" /tmp/x_intree.so
for v in ab/*.so; do
  cp "$v" "$SO"
  timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_lenet_bf16.py -k "not quality" \
    > $O/t_$(basename $v .so).log 2>&1 || { tail -20 $O/t_$(basename $v .so).log; cp /tmp/x_intree.so "$SO"; exit 1; }
  echo "$(basename $v): $(tail -1 $O/t_$(basename $v .so).log)"
done
cp /tmp/x_intree.so "$SO"
bash scripts/ab_multi_so.sh "python bench.py --steps 3000 --warmup 300 --no-fp32-companion" \
  "python bench.py --steps 3000 --warmup 300 --batch 4 --no-fp32-companion" \
  "python bench.py --steps 20 --warmup 5 --no-fp32-companion" || exit 1
cp gpurun_out/ab_multi.jsonl $O/ab_multi.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/r4x/ab_multi.jsonl"):
    d = json.loads(l); o = json.loads(d["out"])
    print(d["variant"], o["steps"], o["config"]["per_gpu_batch"], o["ms_per_step"], o["config"]["device_ms_per_step"])
PY
