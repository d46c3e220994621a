#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, each under its own time limit) over
# benchmarks/gemm_pmc_probe.py: forward-layout vs weight-gradient-layout GEMM.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES GRBM_COUNT"; do
  i=$((i + 1))
  echo "=== pass $i: $grp"
  timeout -s KILL 90 rocprofv3 --pmc $grp -d gpurun_out/pmc/p$i -o run --output-format csv -- python3 benchmarks/gemm_pmc_probe.py > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc/p$i.log; exit $rc; }
done
exit 0
