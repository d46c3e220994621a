# kernel-level profile of the fp8 `large` step with the 4-wave quantising epilogues
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ag
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o large -- python3 -u bench.py --model large --steps 4 --warmup 2 > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
grep '^{' $O/p.log
find $O/prof -name '*kernel_stats.csv' | head -3
