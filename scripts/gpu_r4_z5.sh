#!/bin/bash
# Round 4: amax / cast grid-stride loops with 4 loads in flight per thread. fp8 GPU tests, then A/B
# ab/{a_base,b_unroll}.so: fp8_cast_bench and the fp8 `large` step (driver protocol).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4z5
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fp8_gpu.py tests/test_fp8_fused_gpu.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/ab_multi_so.sh "python benchmarks/fp8_cast_bench.py | grep 262144" "python bench.py --model large --steps 20 --warmup 5" || exit 1
cp gpurun_out/ab_multi.jsonl $O/ab_multi.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/r4z5/ab_multi.jsonl"):
    d = json.loads(l); o = json.loads(d["out"])
    print(d["variant"], o.get("value") or o)
PY
