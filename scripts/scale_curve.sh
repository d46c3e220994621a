#!/bin/bash
# One-command node recipe for an 8-GPU MI355X node: every BASELINE.json DDP config as bench.py lines,
# each appended (with its config id and section) to gpurun_out/scale_curve.jsonl. Efficiency =
# value(N) / (N * value(1)) is left to the reader / driver.
#
#   config 2/3  LeNet (src/model.py default) bf16 + fp32, N = 1/2/4/8, weak (32 per GPU) and the
#               reference's semantics (global batch 32 split over the ranks, src/trainer.py:62-64);
#               at N = 8 a transport A/B (xgmi-fused / four-launch / RCCL) and a per-rank rocprofv3 trace
#   config 4    BERT-base seq 512 bf16, N = 1/2/4/8 weak, DDP with the alpha-beta bucket auto-plan
#               (no caps given) and hipEvent bucket timings; ZeRO-1 A/B at every N > 1
#   config 5    `large` (24L/1024H) fp8 at N = 8: micro-batch 512 per GPU (245 GiB of the 288 GB HBM,
#               bench.py's default -- the largest that fits) x --grad-accum 4 (all-reduce once per 4
#               micro-batches: global batch 16,384 sequences); ZeRO-1 A/B
#   RCCL sweep  BERT-base at N = 8 (its auto-planned bucket sizes) over NCCL_MIN_NCHANNELS =
#               NCCL_MAX_NCHANNELS in {8, 16, 32, 64} x NCCL_ALGO in {Ring, Tree} x NCCL_PROTO in
#               {Simple, LL128} -- plain environment variables of the bench process
#   buckets     the BERT-base DDP bucket-cap sweep (scripts/bucket_sweep.sh)
#
#   usage: scripts/scale_curve.sh [STEPS=2000] [WARMUP=200]     (LeNet steps; BERT / large use 10 / 3)
#   MLT_SCALE_REHEARSE=1: the same lines as a rehearsal on a ONE-GPU box -- N in {1, 2}, both ranks on
#   GPU 0 over gloo (MLT_BENCH_SAME_DEVICE=1), small batches; the RCCL sweep and N = 8 parts are listed
#   but skipped. Its times measure processes sharing one GPU, not a node.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STEPS=${1:-2000}
WARMUP=${2:-200}
REH=${MLT_SCALE_REHEARSE:-0}
export TMPDIR=/tmp PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
out=gpurun_out/scale_curve.jsonl
: > "$out"
if [ "$REH" = 1 ]; then
  export MLT_BENCH_SAME_DEVICE=1 MLT_BENCH_BACKEND=gloo
  NS="1 2"; ngpu=8; STEPS=${1:-50}; WARMUP=${2:-5}
  BERT_B="--batch 4 --seq-len 128"; LARGE_B="--batch 4 --seq-len 128 --grad-accum 2"; BSTEPS="--steps 3 --warmup 1"
else
  NS="1 2 4 8"
  ngpu=$(python3 -c "import torch; print(torch.cuda.device_count())")
  BERT_B=""; LARGE_B="--batch 512 --grad-accum 4"; BSTEPS="--steps 10 --warmup 3"
fi

# line CONFIG SECTION N LIMIT_S [ENV=VALUE ...] -- BENCH_ARGS...: one bench.py run, its JSON line tagged
line() {
  local cfg=$1 sec=$2 n=$3 lim=$4; shift 4
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  if [ "$n" -gt "$ngpu" ]; then echo "=== skip $sec N=$n ($ngpu GPUs visible)"; return 0; fi
  local log="gpurun_out/scale_${cfg}_${sec}_${n}.log"
  echo "=== config $cfg / $sec / N=$n ${envs[*]:-} $*"
  env "${envs[@]}" timeout -k 10 "$lim" python3 -u bench.py --gpus "$n" "$@" \
    --json-out gpurun_out/_scale_last.json > "$log" 2>&1
  local rc=$?
  if [ "$rc" -ne 0 ]; then echo "=== stopping: rc=$rc ($log)"; exit "$rc"; fi
  python3 -c "import json,sys; d=json.load(open('gpurun_out/_scale_last.json')); d['baseline_config']=sys.argv[1]; d['section']=sys.argv[2]; d['env']=sys.argv[3]; d['rehearsal']=sys.argv[4]=='1'; print(json.dumps(d))" \
    "$cfg" "$sec" "${envs[*]:-}" "$REH" >> "$out"
  tail -n 1 "$out"
}

# ---- configs 2 / 3: LeNet, both batch semantics, bf16 and fp32 ---------------------------------
for prec in bf16 fp32; do
  for scaling in weak reference; do
    for n in $NS; do
      line 2-3 "lenet_${prec}_${scaling}" "$n" 300 -- --steps "$STEPS" --warmup "$WARMUP" --precision "$prec" \
        --scaling "$scaling" --no-fp32-companion
    done
  done
done
if [ "$ngpu" -ge 8 ] && [ "$REH" != 1 ]; then
  # N = 8 transport A/B of the bf16 step under both batch semantics: whatever the bring-up vote
  # picks (the xGMI-fused two-launch step when it wins), the four-launch step (MLT_LENET_FUSED_DP=0),
  # and RCCL forced (MLT_XGMI_AR=0)
  for scaling in weak reference; do
    line 3 "lenet_ab_fused_${scaling}" 8 300 -- --steps "$STEPS" --warmup "$WARMUP" --scaling "$scaling" --no-fp32-companion
    line 3 "lenet_ab_fourlaunch_${scaling}" 8 300 MLT_LENET_FUSED_DP=0 -- --steps "$STEPS" --warmup "$WARMUP" \
      --scaling "$scaling" --no-fp32-companion
    line 3 "lenet_ab_rccl_${scaling}" 8 300 MLT_XGMI_AR=0 -- --steps "$STEPS" --warmup "$WARMUP" --scaling "$scaling" \
      --no-fp32-companion
  done
  # kernel trace of the 8-rank reference-semantics step (per-kernel time of every rank): the
  # launcher OUTSIDE the profiler, one rocprofv3 per rank with bench.py directly after its `--`
  # (scripts/prof_rank.sh); bench.py sees WORLD_SIZE and does not self-launch
  mkdir -p gpurun_out/prof_n8
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29537 --no-python scripts/prof_rank.sh gpurun_out/prof_n8 -- \
    python3 -u bench.py --gpus 8 --steps 500 --warmup 50 --scaling reference --no-fp32-companion \
    > gpurun_out/prof_n8/bench.log 2>&1 || echo "=== rocprofv3 N=8 trace failed (see gpurun_out/prof_n8/bench.log)"
fi

# ---- config 4: BERT-base seq 512 bf16, N = 1/2/4/8 weak, auto-planned DDP buckets; ZeRO-1 A/B ----
for n in $NS; do
  # shellcheck disable=SC2086
  line 4 bert_base_ddp "$n" 600 -- --model bert-base $BERT_B $BSTEPS --ddp-timing
  if [ "$n" -gt 1 ]; then
    # shellcheck disable=SC2086
    line 4 bert_base_zero1 "$n" 600 -- --model bert-base $BERT_B $BSTEPS --zero 1
  fi
done

# ---- config 5: large fp8, DDP = 8, HBM-filling micro-batch x grad-accum; ZeRO-1 A/B ---------------
N5=8
[ "$REH" = 1 ] && N5=2
# shellcheck disable=SC2086
line 5 large_fp8_ddp "$N5" 900 -- --model large $LARGE_B $BSTEPS --ddp-timing
# shellcheck disable=SC2086
line 5 large_fp8_zero1 "$N5" 900 -- --model large $LARGE_B $BSTEPS --zero 1

# ---- RCCL channel / algorithm / protocol sweep at the BERT-base bucket sizes (N = 8) -------------
if [ "$ngpu" -ge 8 ] && [ "$REH" != 1 ]; then
  for ch in 8 16 32 64; do
    for algo in Ring Tree; do
      for proto in Simple LL128; do
        line 4 "rccl_sweep_c${ch}_${algo}_${proto}" 8 600 NCCL_MIN_NCHANNELS=$ch NCCL_MAX_NCHANNELS=$ch \
          NCCL_ALGO=$algo NCCL_PROTO=$proto -- --model bert-base --steps 10 --warmup 3 --ddp-timing
      done
    done
  done
  bash scripts/bucket_sweep.sh 8 10 && cat gpurun_out/bucket_sweep.jsonl >> "$out"
else
  echo "=== skip RCCL sweep (8 x {Ring,Tree} x {Simple,LL128} x {8,16,32,64} channels) and bucket sweep: needs 8 GPUs"
fi
echo "=== $(wc -l < "$out") records in $out"
