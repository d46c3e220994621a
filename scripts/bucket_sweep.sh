#!/bin/bash
# DDP bucket-size sweep for the 8-GPU node (BERT-base classifier, BASELINE config 4):
# bench.py --model bert-base on N ranks for bucket caps 4..128 MB, fp32 and bf16 gradient
# all-reduce; every run prints one JSON line whose config.ddp_comm holds allreduce_ms,
# exposed_ms, overlap_pct and the bucket layout.  Results: gpurun_out/bucket_sweep.jsonl
#   usage: scripts/bucket_sweep.sh [N_GPUS=8] [STEPS=10]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=${1:-8}
STEPS=${2:-10}
mkdir -p gpurun_out
out=gpurun_out/bucket_sweep.jsonl
: > "$out"
for comm in fp32 bf16; do
  for mb in 4 8 16 32 64 128; do
    echo "=== bucket ${mb} MB, grad comm ${comm}, ${N} ranks"
    timeout -k 10 300 python -u bench.py --gpus "$N" --model bert-base --steps "$STEPS" --warmup 3 \
      --bucket-mb "$mb" --first-bucket-mb "$(( mb < 8 ? mb : 8 ))" --grad-comm "$comm" \
      --json-out gpurun_out/_sweep_last.json > "gpurun_out/bucket_sweep_${comm}_${mb}.log" 2>&1
    rc=$?
    if [ "$rc" -ne 0 ]; then
      echo "=== stopping: rc=$rc (see gpurun_out/bucket_sweep_${comm}_${mb}.log)"
      exit "$rc"
    fi
    cat gpurun_out/_sweep_last.json >> "$out"
    tail -n 1 gpurun_out/_sweep_last.json
  done
done
