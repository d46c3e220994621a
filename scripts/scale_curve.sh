#!/bin/bash
# One-command scaling curve for an 8-GPU MI355X node (BASELINE.json metric: samples/sec/node +
# step time, src/model.py default, DDP 1/2/4/8): bench.py at N = 1, 2, 4, 8 in both batch
# semantics -- weak (32 per GPU) and the reference's (global batch 32 split over the ranks,
# src/trainer.py:62-64) -- for the bf16 and the fp32 LeNet step, then the BERT-base DDP bucket
# sweep. Every bench run appends its JSON line (plus the mode) to gpurun_out/scale_curve.jsonl;
# efficiency = value(N) / (N * value(1)) is left to the reader / driver.
#   usage: scripts/scale_curve.sh [STEPS=2000] [WARMUP=200]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STEPS=${1:-2000}
WARMUP=${2:-200}
export TMPDIR=/tmp PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
out=gpurun_out/scale_curve.jsonl
: > "$out"
ngpu=$(python3 -c "import torch; print(torch.cuda.device_count())")
for prec in bf16 fp32; do
  for scaling in weak reference; do
    for n in 1 2 4 8; do
      if [ "$n" -gt "$ngpu" ]; then echo "=== skip N=$n ($ngpu GPUs visible)"; continue; fi
      echo "=== LeNet $prec, $scaling, N=$n"
      timeout -k 10 300 python3 -u bench.py --gpus "$n" --steps "$STEPS" --warmup "$WARMUP" --precision "$prec" \
        --scaling "$scaling" --no-fp32-companion \
        --json-out gpurun_out/_scale_last.json > "gpurun_out/scale_${prec}_${scaling}_${n}.log" 2>&1
      rc=$?
      if [ "$rc" -ne 0 ]; then echo "=== stopping: rc=$rc (gpurun_out/scale_${prec}_${scaling}_${n}.log)"; exit "$rc"; fi
      python3 -c "import json,sys; d=json.load(open('gpurun_out/_scale_last.json')); d['mode']='$scaling'; print(json.dumps(d))" >> "$out"
      tail -n 1 "$out"
    done
  done
done
if [ "$ngpu" -ge 8 ]; then
  # N = 8 transport A/B of the bf16 step under both batch semantics: whatever the bring-up vote
  # picks (the xGMI-fused two-launch step when it wins), the four-launch step with the one-/two-shot vote (MLT_LENET_FUSED_DP=0),
  # and RCCL forced (MLT_XGMI_AR=0)
  for scaling in weak reference; do
    for variant in fused fourlaunch rccl; do
      case $variant in
        fused) envs="";;
        fourlaunch) envs="MLT_LENET_FUSED_DP=0";;
        rccl) envs="MLT_XGMI_AR=0";;
      esac
      echo "=== LeNet bf16 $scaling N=8 transport=$variant"
      env $envs timeout -k 10 300 python3 -u bench.py --gpus 8 --steps "$STEPS" --warmup "$WARMUP" --scaling "$scaling" \
        --no-fp32-companion --json-out gpurun_out/_scale_last.json > "gpurun_out/scale_ab_${variant}_${scaling}.log" 2>&1 \
        || { echo "=== stopping: transport A/B $variant failed"; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/_scale_last.json')); d['mode']='$scaling'; d['transport_ab']='$variant'; print(json.dumps(d))" >> "$out"
      tail -n 1 "$out"
    done
  done
  # kernel trace of the 8-rank reference-semantics step (per-kernel time of every rank): the
  # launcher OUTSIDE the profiler, one rocprofv3 per rank with bench.py directly after its `--`
  # (scripts/prof_rank.sh); bench.py sees WORLD_SIZE and does not self-launch
  mkdir -p gpurun_out/prof_n8
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29537 --no-python scripts/prof_rank.sh gpurun_out/prof_n8 -- \
    python3 -u bench.py --gpus 8 --steps 500 --warmup 50 --scaling reference --no-fp32-companion \
    > gpurun_out/prof_n8/bench.log 2>&1 || echo "=== rocprofv3 N=8 trace failed (see gpurun_out/prof_n8/bench.log)"
  bash scripts/bucket_sweep.sh 8 10 && cat gpurun_out/bucket_sweep.jsonl >> "$out"
fi
echo "=== $(wc -l < "$out") records in $out"
