#!/bin/bash
# Round 4: fp8 cfg 7 split-K (fp8 weight gradients): tests, fp8 large + BERT-base A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4r
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_fp8_gpu.py tests/test_gemm_gpu.py tests/test_fp8_fused_gpu.py tests/test_transformer_gpu.py \
  > $O/t_gemm.log 2>&1 || { tail -30 $O/t_gemm.log; exit 1; }
tail -1 $O/t_gemm.log
for w in 1 0 1 0; do
  MLT_GEMM_W4F8=$w MLT_GEMM_W4Q8=$w timeout -k 10 400 python -u bench.py --model large --steps 6 --warmup 2 > $O/_b.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/_b.json').read().strip().splitlines()[-1]); d['w4f8']=$w; print(json.dumps(d))" >> $O/ab_large.jsonl
  tail -1 $O/ab_large.jsonl | cut -c1-110
done
for w in 1 0 1 0; do
  MLT_GEMM_W4=$w timeout -k 10 400 python -u bench.py --model bert-base --steps 6 --warmup 2 > $O/_b.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/_b.json').read().strip().splitlines()[-1]); d['w4']=$w; print(json.dumps(d))" >> $O/ab_bert.jsonl
  tail -1 $O/ab_bert.jsonl | cut -c1-110
done
