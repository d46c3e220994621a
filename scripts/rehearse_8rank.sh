# 8-rank rehearsal of the driver's N=8 LeNet bench launch on a 1-GPU box: all ranks on GPU 0 over
# gloo, the xGMI one-/two-shot kernels instantiated for W=8 (MLT_XGMI_ALLOW_GLOO), transport vote,
# per-GPU batch 32 (weak) and 4 (reference semantics); then 4 and 8 ranks with the transport vote
# forced through the full step graph for a few hundred steps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export MLT_BENCH_SAME_DEVICE=1 MLT_BENCH_BACKEND=gloo MLT_XGMI_ALLOW_GLOO=1
L="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 240 $L --nproc-per-node 8 --master-port 29521 bench.py --gpus 8 --steps 200 --warmup 20 > gpurun_out/r8_lenet_xgmi.log 2>&1 &&
timeout -k 10 240 $L --nproc-per-node 8 --master-port 29522 bench.py --gpus 8 --steps 200 --warmup 20 --scaling reference > gpurun_out/r8_lenet_xgmi_ref.log 2>&1 &&
timeout -k 10 240 $L --nproc-per-node 4 --master-port 29523 bench.py --gpus 4 --steps 200 --warmup 20 > gpurun_out/r4_lenet_xgmi.log 2>&1
