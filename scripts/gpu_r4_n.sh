#!/bin/bash
# Round 4: fp8 cfg 7 tests + bench; attention -delta fold tests + B512 timing; BERT-base and fp8 large
# A/B (MLT_GEMM_W4 1/0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4n
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_fp8_gpu.py tests/test_gemm_gpu.py \
  > $O/t_gemm.log 2>&1 || { tail -30 $O/t_gemm.log; exit 1; }
tail -1 $O/t_gemm.log
timeout -k 10 400 python -u benchmarks/gemm_w4_f8_bench.py > $O/f8_bench.jsonl 2>$O/f8.err || { tail $O/f8.err; exit 1; }
cat $O/f8_bench.jsonl
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests -k "attn or attention" \
  > $O/t_attn.log 2>&1 || { tail -30 $O/t_attn.log; exit 1; }
tail -1 $O/t_attn.log
for b in 512 512; do ATTN_B=$b timeout -k 10 120 python3 -u benchmarks/attn_bench.py >> $O/attn_bench.jsonl 2>$O/attn.err || exit 1; done
cut -c1-150 $O/attn_bench.jsonl
for m in large bert-base; do
  for w in 1 0 1 0; do
    MLT_GEMM_W4=$w timeout -k 10 400 python -u bench.py --model $m --steps 6 --warmup 2 > $O/_b.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/_b.json').read().strip().splitlines()[-1]); d['w4']=$w; print(json.dumps(d))" >> $O/ab_$m.jsonl
    tail -1 $O/ab_$m.jsonl | cut -c1-110
  done
done
