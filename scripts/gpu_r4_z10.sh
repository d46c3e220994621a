#!/bin/bash
# Round 4: RES epilogue side operand per half (b_res1) vs both halves up front (a_res2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4z10
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_transformer_gpu.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/ab_multi_so.sh "GEMM_BENCH_TOKENS=262144 python benchmarks/gemm_epi_bench.py" "python bench.py --model bert-base --steps 20 --warmup 5" || exit 1
cp gpurun_out/ab_multi.jsonl $O/ab_multi.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/r4z10/ab_multi.jsonl"):
    d = json.loads(l); o = json.loads(d["out"])
    print(d["variant"], o.get("value") or {k: v for k, v in o.items() if "out_fwd" in k and k.endswith("tflops")})
PY
