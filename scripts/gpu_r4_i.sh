#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4i
mkdir -p $O
for g in 4 8 16; do
  MLT_GEMM_GROUP_M=$g timeout -k 10 300 python -u benchmarks/gemm_w4_sweep.py >> $O/sweep.jsonl 2>$O/sweep.err || { tail $O/sweep.err; exit 1; }
done
python3 -c "
import json
for d in map(json.loads, open('$O/sweep.jsonl')): print(d['group_m'], d['N'], d['K'], d['cfg7_ms'], d['torch_ms'], d['cfg7_tflops'], d['torch_tflops'])"
