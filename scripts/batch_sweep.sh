#!/bin/bash
# Per-GPU micro-batch sweep of the transformer benches (one GPU): samples/s and peak HBM vs batch.
# usage: bash scripts/batch_sweep.sh "bert-base 32" "large 64" ...
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/batch_sweep.jsonl
: > $out
for spec in "$@"; do
  set -- $spec
  timeout -k 10 300 python bench.py --model $1 --batch $2 --steps ${3:-8} --warmup 3 >> $out 2>gpurun_out/sweep_err.log || exit 1
done
