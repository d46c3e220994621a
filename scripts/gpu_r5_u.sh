# 8-rank rehearsal of the driver's N=8 LeNet bench with this round's build (all ranks on the one GPU,
# gloo process group, xGMI exchanges through IPC on the same device): weak and reference semantics,
# then 2 and 4 ranks; the JSON lines + the transport each run chose
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0 && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5u
mkdir -p $O
export MLT_BENCH_SAME_DEVICE=1 MLT_BENCH_BACKEND=gloo MLT_XGMI_ALLOW_GLOO=1
L="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
for spec in "8 29541 weak" "8 29542 reference" "2 29543 weak" "4 29544 weak"; do
  set -- $spec
  timeout -k 10 240 $L --nproc-per-node $1 --master-port $2 bench.py --gpus $1 --steps 20 --warmup 5 --scaling $3 \
    --no-fp32-companion > $O/r$1_$3.log 2>&1 || { echo "FAILED: $spec"; tail -30 $O/r$1_$3.log; exit 1; }
  grep '^{' $O/r$1_$3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$spec', d['value'], d['ms_per_step'], c['dp_transport'], c.get('transport_ms'))"
done
