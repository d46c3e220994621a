#!/bin/bash
# Round 4: two-wide GELU / dGELU in the fp8 q8 epilogue (8-wave pp kernel) and the store8 pass:
# fp8 GPU tests on the new build, then same-box A/B ab/{b_pk,c_pk_q8}.so on the fp8 `large` model.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4z2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fp8_gpu.py tests/test_fp8_fused_gpu.py tests/test_gemm_gpu.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/ab_multi_so.sh "python bench.py --model large --steps 6 --warmup 2" || exit 1
cp gpurun_out/ab_multi.jsonl $O/ab_multi.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/r4z2/ab_multi.jsonl"):
    d = json.loads(l); o = json.loads(d["out"])
    print(d["variant"], o.get("value"))
PY
