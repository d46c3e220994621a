#!/bin/bash
# Round 4: per-sample kernel variants, same box. Numerics first (every bf16 LeNet test on the in-tree
# build), then alternated benches over ab/*.so: v0 = round-3 kernel, v1 = LDS fc1 image,
# v3 = v1 + kernarg preload of the first-load pointers (KS and KW), v4 = v3 + the optimizer kind dispatched once per KW block, v5 = v4 + the LDS fc2 image.
set -o pipefail
O=gpurun_out/r4ab
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_lenet_bf16.py \
  -k "not quality" > $O/t_bf16.log 2>&1 || { tail -40 $O/t_bf16.log; exit 1; }
tail -3 $O/t_bf16.log
bash scripts/ab_multi_so.sh "python bench.py --steps 3000 --warmup 300 --no-fp32-companion" \
  "python bench.py --steps 3000 --warmup 300 --batch 4 --no-fp32-companion" \
  "python bench.py --steps 20 --warmup 5 --no-fp32-companion" || exit 1
cp gpurun_out/ab_multi.jsonl $O/ab_multi.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/r4ab/ab_multi.jsonl"):
    d = json.loads(l); o = json.loads(d["out"])
    print(d["variant"], o["steps"], o["config"]["per_gpu_batch"], o["ms_per_step"], o["config"]["device_ms_per_step"])
PY
