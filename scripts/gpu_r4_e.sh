#!/bin/bash
# Round 4: attention ring-kernel change (GPU tests, B512 timing + kernel stats + PMC) and a GEMM PMC
# comparison of the native ping-pong kernel with hipBLASLt (torch.matmul) on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests -k "attn or attention" \
  > $O/t_attn.log 2>&1 || { tail -30 $O/t_attn.log; exit 1; }
tail -2 $O/t_attn.log
for b in 512 512; do ATTN_B=$b timeout -k 10 120 python3 -u benchmarks/attn_bench.py >> $O/attn_bench.jsonl 2>$O/attn.err || exit 1; done
cat $O/attn_bench.jsonl
bash scripts/attn_prof.sh r4 512 > $O/attn_prof.log 2>&1 || { tail -20 $O/attn_prof.log; exit 1; }
tail -12 $O/attn_prof.log
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES GRBM_COUNT"
for shp in "65536 2304 768" "8192 8192 8192"; do
  set -- $shp
  i=0
  for grp in "$P1" "$P2"; do
    i=$((i + 1))
    d=$O/gemm_pmc_${1}_${2}_${3}_p$i
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $d -o run -- python3 benchmarks/gemm_pmc.py \
      --M $1 --N $2 --K $3 --cfgs 5 --reps 5 --torch 5 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  done
done
echo gemm pmc done
