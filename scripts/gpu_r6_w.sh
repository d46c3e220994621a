# Per-dispatch trace of the fp8 `large` step's cast-transposes (grid = columns / 128 x rows / 128):
# which tensors each kernel form quantises, and its time per call.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6w
O=gpurun_out/r6w
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o large -- python3 -u bench.py --model large --steps 2 --warmup 1 > $O/p.log 2>&1
echo "rc=$?"
