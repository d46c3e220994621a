#!/bin/bash
# Round 4: the LDS-resident fc1 image (new in-tree build) vs the previous per-sample kernel (ab/),
# numerics first (every bf16 LeNet test on the new build), then same-box alternated benches.
set -o pipefail
O=gpurun_out/r4ab
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_lenet_bf16.py \
  -k "not quality" > $O/t_bf16.log 2>&1 || { tail -40 $O/t_bf16.log; exit 1; }
tail -3 $O/t_bf16.log
: > gpurun_out/ab.jsonl
bash scripts/ab_so.sh "python bench.py --steps 3000 --warmup 300 --no-fp32-companion" \
  "python bench.py --steps 3000 --warmup 300 --batch 4 --no-fp32-companion" \
  "python bench.py --steps 20 --warmup 5 --no-fp32-companion" || exit 1
cp gpurun_out/ab.jsonl $O/ab.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/r4ab/ab.jsonl"):
    d = json.loads(l); o = json.loads(d["out"])
    print(d["variant"], d["cmd"][-45:], o["config"]["per_gpu_batch"], o["ms_per_step"], o["config"]["device_ms_per_step"])
PY
