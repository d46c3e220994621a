#!/bin/bash
# Round 4: the 4-wave asm GEMM (cfg 7): correctness tests, timing vs cfg 5 / hipBLASLt, one PMC pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_gpu.py -k "w4" \
  > $O/t_w4.log 2>&1 || { tail -40 $O/t_w4.log; exit 1; }
tail -4 $O/t_w4.log
timeout -k 10 300 python -u benchmarks/gemm_w4_bench.py > $O/w4_bench.jsonl 2>$O/w4_bench.err || { tail $O/w4_bench.err; exit 1; }
cat $O/w4_bench.jsonl
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d $O/pmc_w4_p1 -o run -- python3 benchmarks/gemm_pmc.py \
  --M 8192 --N 8192 --K 8192 --cfgs 7 --reps 5 > $O/pmc_w4_p1.log 2>&1 || { tail -5 $O/pmc_w4_p1.log; exit 1; }
python3 scripts/pmc_summary.py $O/pmc_w4_p1 --match gemm
