# LeNet chain: v6 = v1 + fc1 DMA issued by waves 8-15 at P1 start while waves 0-7 do P1 + conv1 behind
# an LDS-counter hand-off (steady-state prep path), counted vmcnt before P4a; v7 = v6 + conv1 wgrad
# over 14 waves. Tests + phases on the in-tree build (v7), then A/B base / v1 / v6 / v7.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6e
O=gpurun_out/r6e
timeout -k 10 300 python -u -m pytest tests/test_lenet_bf16.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 &&
timeout -k 10 120 python3 -u benchmarks/lenet_bf16_phases.py 32 > $O/ph32.log 2>&1 &&
bash scripts/ab_multi_so.sh "python -u bench.py --no-fp32-companion" "python -u bench.py --steps 20 --warmup 5 --no-fp32-companion" "python -u bench.py --batch 4 --transport xgmi-loopback --no-fp32-companion" &&
cp gpurun_out/ab_multi.jsonl $O/ab.jsonl
echo "rc=$?"
