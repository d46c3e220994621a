#!/bin/bash
# Round 4, part A: fused data-parallel step on one GPU (loopback), headline bench, fetch probes of the
# per-sample kernel, MFMA shape probe, prefetcher overlap, bf16-vs-fp32 quality.
set -o pipefail
O=gpurun_out/r4a
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 60 ./benchmarks/bin/mfma_shape_probe 20000 > $O/mfma_shape.jsonl 2>&1 || exit 1
cat $O/mfma_shape.jsonl
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_lenet_bf16.py -k "fused_dp or reduce_mode" tests/test_lenet_native.py -k "prefetch" \
  > $O/t_bf16.log 2>&1 || { tail -30 $O/t_bf16.log; exit 1; }
tail -3 $O/t_bf16.log
for b in 4 32; do
  timeout -k 10 120 python -u bench.py --steps 2000 --warmup 200 --batch $b --no-fp32-companion > $O/b_local_$b.json 2>$O/b_local_$b.err || exit 1
  timeout -k 10 120 python -u bench.py --steps 2000 --warmup 200 --batch $b --no-fp32-companion --transport xgmi-loopback > $O/b_loop_$b.json 2>$O/b_loop_$b.err || exit 1
  cat $O/b_local_$b.json $O/b_loop_$b.json
done
for pr in 131072 262144 524288 917504; do
  MLT_LENET_PROBE=$pr timeout -k 10 120 python -u bench.py --steps 2000 --warmup 200 --no-fp32-companion > $O/b_probe_$pr.json 2>$O/b_probe_$pr.err || exit 1
  echo "probe $pr: $(cat $O/b_probe_$pr.json)"
done
timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > $O/b_driver.json 2>$O/b_driver.err || exit 1
cat $O/b_driver.json
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_lenet_bf16.py -k quality \
  > $O/t_quality.log 2>&1 || { tail -30 $O/t_quality.log; exit 1; }
tail -3 $O/t_quality.log
timeout -k 10 300 python -u scripts/bf16_quality.py --out $O/quality.jsonl > $O/quality.log 2>&1 || exit 1
cat $O/quality.jsonl
