#!/bin/bash
# Round-4 check of the fused data-parallel LeNet step: new GPU tests, loopback timing, headline bench,
# prefetcher overlap, bf16-vs-fp32 training quality.
set -o pipefail
O=gpurun_out/r4dp
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_lenet_bf16.py -k "fused_dp or reduce_mode or quality" tests/test_lenet_native.py -k "prefetch" \
  > $O/t_bf16.log 2>&1 || { tail -30 $O/t_bf16.log; exit 1; }
tail -3 $O/t_bf16.log
for b in 4 32; do
  timeout -k 10 120 python -u bench.py --steps 2000 --warmup 200 --batch $b --no-fp32-companion > $O/b_local_$b.json 2>$O/b_local_$b.err || exit 1
  timeout -k 10 120 python -u bench.py --steps 2000 --warmup 200 --batch $b --no-fp32-companion --transport xgmi-loopback > $O/b_loop_$b.json 2>$O/b_loop_$b.err || exit 1
  cat $O/b_local_$b.json $O/b_loop_$b.json
done
timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > $O/b_driver.json 2>$O/b_driver.err || exit 1
cat $O/b_driver.json
timeout -k 10 300 python -u scripts/bf16_quality.py --out $O/quality.jsonl > $O/quality.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_multiproc_gpu.py -k "fused_dp or three_four_eight" tests/test_trainer_parallel_gpu.py > $O/t_mp.log 2>&1 || { tail -40 $O/t_mp.log; exit 1; }
tail -15 $O/t_mp.log
