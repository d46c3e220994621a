#!/bin/bash
# Round 4: after the AGPR-spill fixes: GEMM / fp8 / transformer tests, BERT-base + fp8 large benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4v
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_fp8_gpu.py tests/test_fp8_fused_gpu.py tests/test_gemm_gpu.py tests/test_transformer_gpu.py \
  > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python -u bench.py --model bert-base --steps 20 --warmup 5 > $O/bert.json 2>$O/b.err || { tail $O/b.err; exit 1; }
tail -1 $O/bert.json | cut -c1-120
timeout -k 10 400 python -u bench.py --model large --steps 6 --warmup 2 > $O/large.json 2>$O/b.err || { tail $O/b.err; exit 1; }
tail -1 $O/large.json | cut -c1-120
