#!/bin/bash
# LeNet step evidence on one MI355X: driver-protocol + steady-state bench at batch 32 and 4,
# rocprofv3 kernel stats at both batches, and two PMC passes per batch (each its own run and
# time limit; stops at the first failure). Outputs under gpurun_out/lenet_prof/.
#   usage: bash scripts/lenet_prof.sh [tag]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
tag=${1:-cur}
O=gpurun_out/lenet_prof/$tag
mkdir -p "$O"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM"
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== [$name] $*"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== [$name] rc=$rc"; tail -n 3 "$O/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
for B in 32 4; do
  run drv_b$B 120 python3 -u bench.py --batch $B --steps 20 --warmup 5
  run ss_b$B 120 python3 -u bench.py --batch $B --steps 3000 --warmup 300
  run prof_b$B 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_b$B" -o run -- \
      python3 -u bench.py --batch $B --steps 400 --warmup 20
  i=0
  for grp in "$P1" "$P2"; do
    i=$((i + 1))
    run pmc_b${B}_p$i 90 rocprofv3 --pmc $grp --output-format csv -d "$O/pmc_b${B}_p$i" -o run -- \
        python3 -u bench.py --batch $B --steps 100 --warmup 10
  done
  python3 scripts/pmc_summary.py "$O/pmc_b${B}_p1" "$O/pmc_b${B}_p2" --match lenet --jsonl "$O/pmc_b$B.jsonl" > /dev/null
done
echo done
