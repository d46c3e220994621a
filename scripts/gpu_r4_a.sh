#!/bin/bash
# Round 4, part A (one GPU): fused data-parallel step (loopback) timing, phase trace + rocprof of the
# current per-sample kernel, headline bench under the driver protocol (with the fp32 companion), MFMA
# shape probe, prefetcher overlap, bf16-vs-fp32 training quality.
set -o pipefail
O=gpurun_out/r4a
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 ./benchmarks/bin/mfma_shape_probe 20000 > $O/mfma_shape.jsonl 2>&1 || exit 1
cat $O/mfma_shape.jsonl
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_lenet_native.py -k "prefetch" \
  > $O/t_prefetch.log 2>&1 || { tail -30 $O/t_prefetch.log; exit 1; }
tail -3 $O/t_prefetch.log
for b in 4 32; do
  timeout -k 10 120 python -u bench.py --steps 3000 --warmup 300 --batch $b --no-fp32-companion > $O/b_local_$b.json 2>$O/b_local_$b.err || exit 1
  timeout -k 10 120 python -u bench.py --steps 3000 --warmup 300 --batch $b --no-fp32-companion --transport xgmi-loopback > $O/b_loop_$b.json 2>$O/b_loop_$b.err || exit 1
  cat $O/b_local_$b.json $O/b_loop_$b.json
done
timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > $O/b_driver.json 2>$O/b_driver.err || exit 1
cat $O/b_driver.json
timeout -k 10 120 python3 -u benchmarks/lenet_bf16_phases.py 32 --jsonl $O/phases.jsonl > $O/ph32.log 2>&1 || exit 1
timeout -k 10 120 python3 -u benchmarks/lenet_bf16_phases.py 4 --jsonl $O/phases.jsonl > $O/ph4.log 2>&1 || exit 1
cat $O/ph32.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o b32 -- python3 -u bench.py --batch 32 --steps 400 --warmup 20 --no-fp32-companion > $O/prof.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_lenet_bf16.py -k quality \
  > $O/t_quality.log 2>&1 || { tail -30 $O/t_quality.log; }
tail -3 $O/t_quality.log
timeout -k 10 300 python -u scripts/bf16_quality.py --out $O/quality.jsonl > $O/quality.log 2>&1 || exit 1
cat $O/quality.jsonl
