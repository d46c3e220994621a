#!/bin/bash
# Round 4: cfg 7 epilogue image written straight from the AGPRs (ds_write_b128 a[..], no
# v_accvgpr_read per element). GEMM / fp8 / transformer GPU tests, then A/B ab/{c_pk_q8,d_img}.so.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4z4
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_fp8_gpu.py tests/test_fp8_fused_gpu.py tests/test_transformer_gpu.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/ab_multi_so.sh "GEMM_BENCH_TOKENS=262144 python benchmarks/gemm_epi_bench.py" "python bench.py --model bert-base --steps 20 --warmup 5" || exit 1
cp gpurun_out/ab_multi.jsonl $O/ab_multi.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/r4z4/ab_multi.jsonl"):
    d = json.loads(l); o = json.loads(d["out"])
    print(d["variant"], o.get("value") or {k: v for k, v in o.items() if k.endswith("tflops")})
PY
