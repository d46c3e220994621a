#!/bin/bash
# Attention kernels on one MI355X: kernel stats + two PMC passes (own runs, own time limits) over
# benchmarks/attn_bench.py at ATTN_B (default 128). Outputs under gpurun_out/attn_prof/<tag>/.
#   usage: bash scripts/attn_prof.sh [tag] [batch]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
tag=${1:-cur}
export ATTN_B=${2:-128}
O=gpurun_out/attn_prof/$tag
mkdir -p "$O"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== [$name] $*"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== [$name] rc=$rc"; tail -n 2 "$O/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
run bench 120 python3 -u benchmarks/attn_bench.py
run stats 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats" -o run -- python3 -u benchmarks/attn_bench.py
i=0
for grp in "$P1" "$P2"; do
  i=$((i + 1))
  run pmc_p$i 120 rocprofv3 --pmc $grp --output-format csv -d "$O/pmc_p$i" -o run -- python3 -u benchmarks/attn_bench.py
done
python3 scripts/pmc_summary.py "$O/pmc_p1" "$O/pmc_p2" --match attn --jsonl "$O/pmc.jsonl" > "$O/pmc_summary.txt"
cat "$O/pmc_summary.txt"
