#!/bin/bash
# Round 4: persistent fp8 cfg 7: fp8 / GEMM tests, fp8 large A/B (MLT_W4_PERSIST 1/0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4u
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_fp8_gpu.py tests/test_fp8_fused_gpu.py tests/test_gemm_gpu.py \
  > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for p in 1 0 1 0; do
  MLT_W4_PERSIST=$p timeout -k 10 400 python -u bench.py --model large --steps 6 --warmup 2 > $O/_b.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/_b.json').read().strip().splitlines()[-1]); d['persist']=$p; print(json.dumps(d))" >> $O/ab_large.jsonl
  tail -1 $O/ab_large.jsonl | cut -c1-100
done
