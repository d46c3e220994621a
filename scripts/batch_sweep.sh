#!/bin/bash
# Per-GPU batch sweep of the transformer benches (one GPU): how samples/s moves with the micro-batch.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/batch_sweep.jsonl
: > $out
for spec in "bert-base 32" "bert-base 64" "bert-base 128" "large 16" "large 32" "large 64"; do
  set -- $spec
  timeout -k 10 240 python bench.py --model $1 --batch $2 --steps 10 --warmup 3 >> $out 2>gpurun_out/sweep_err.log || exit 1
done
