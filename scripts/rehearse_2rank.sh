# 2-rank rehearsal of the driver's N>1 bench launch on a 1-GPU box (both ranks on GPU 0, gloo)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export MLT_BENCH_SAME_DEVICE=1 MLT_BENCH_BACKEND=gloo
L="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port"
timeout -k 10 180 $L 29511 bench.py --gpus 2 --steps 200 --warmup 20 > gpurun_out/r2_lenet.log 2>&1 &&
timeout -k 10 240 $L 29512 bench.py --gpus 2 --model large --batch 16 --steps 3 --warmup 2 > gpurun_out/r2_large.log 2>&1 &&
timeout -k 10 240 $L 29513 bench.py --gpus 2 --model bert-base --batch 16 --zero 1 --steps 3 --warmup 2 > gpurun_out/r2_bert_zero.log 2>&1 &&
timeout -k 10 240 $L 29514 bench.py --gpus 2 --model bert-base --batch 16 --grad-comm bf16 --steps 3 --warmup 2 > gpurun_out/r2_bert_ddp_bf16.log 2>&1 &&
MLT_XGMI_ALLOW_GLOO=1 timeout -k 10 180 $L 29515 bench.py --gpus 2 --steps 200 --warmup 20 > gpurun_out/r2_lenet_xgmi.log 2>&1
