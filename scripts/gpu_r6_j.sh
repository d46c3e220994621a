# Kernel-level profile of the shipped LeNet step (bf16 two-kernel + the fp32 companion's four
# kernels), bench.py --steps 1000, and the fp32 fused-variant phase trace (trace build).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6j
O=gpurun_out/r6j
SO=$(ls ml_trainer_amd/_C*.so)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o lenet -- python3 -u bench.py --steps 1000 --warmup 100 > $O/prof.log 2>&1 &&
cp "$SO" /tmp/intree.so && cp ab_trace.so "$SO" &&
timeout -k 10 120 python3 -u benchmarks/lenet_phase_trace.py 32 > $O/fp32_ph32.log 2>&1
rc=$?
cp /tmp/intree.so "$SO"
echo "rc=$rc"
exit $rc
