# Two-phase fused xGMI exchange (chunk owners reduce and publish the sums): the multi-process GPU
# tests (W = 2 and 8 ranks on the box's one GPU: bitwise vs the four-launch step; its self-test and
# forced selection), the LeNet / trainer GPU tests, then the 8-rank rehearsal of the bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0 && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5v
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_multiproc_gpu.py tests/test_lenet_bf16.py tests/test_trainer_parallel_gpu.py > $O/tests.log 2>&1 \
  || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
export MLT_BENCH_SAME_DEVICE=1 MLT_BENCH_BACKEND=gloo MLT_XGMI_ALLOW_GLOO=1
L="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
for spec in "8 29551 auto" "8 29552 1" "4 29553 1"; do
  set -- $spec
  MLT_XGMI_FUSED_TWO=$3 timeout -k 10 240 $L --nproc-per-node $1 --master-port $2 bench.py --gpus $1 --steps 20 --warmup 5 \
    --no-fp32-companion > $O/r$1_$3.log 2>&1 || { echo "FAILED: $spec"; tail -30 $O/r$1_$3.log; exit 1; }
  grep '^{' $O/r$1_$3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$spec', d['value'], c['dp_transport'], (c.get('ddp_comm') or {}).get('fused_two_phase'), c.get('transport_ms'))"
done
