# Instruction-cache behaviour of the LeNet step kernels (SQC counters, if the pool's rocprofv3 lists
# them): hits / misses per kernel over a short bench run.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/icache
O=gpurun_out/icache
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1
grep -oE "SQC_[A-Z0-9_]+" $O/avail.txt | sort -u > $O/sqc.txt
C=$(grep -E "^SQC_ICACHE_(HITS|MISSES|MISSES_DUPLICATE|REQ)$" $O/sqc.txt | tr '\n' ' ')
echo "counters: $C"
[ -n "$C" ] || exit 0
timeout -s KILL 90 rocprofv3 --pmc $C SQ_WAVES SQ_INSTS_VALU --output-format csv -d $O/pmc -o run -- python3 -u bench.py --steps 200 --warmup 20 --no-fp32-companion > $O/pmc.log 2>&1
echo "rc=$?"
