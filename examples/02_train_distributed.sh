#!/bin/bash
# Distributed training on one 8x MI355X node: what the reference's
# 02_ML_Training_SageMaker_distributed.ipynb does through a SageMaker estimator with
# smdistributed.dataparallel (cells :92-101 hyperparameters, :115-118 distribution,
# :156-158 fit, :172-186 load_history + plot_history). Here: one process per GPU via
# torch.distributed.run, RCCL over xGMI, and the fused LeNet engine in bf16 (BASELINE.json config 3:
# "default config bf16, DDP world_size=8"): two launches per step, the second of which exchanges
# the gradient over xGMI inside its update blocks when the bring-up vote picks that transport
# (PRECISION=fp32 runs the reference dtype's four-kernel step instead).
#
#   examples/02_train_distributed.sh [NGPUS] [extra main.py flags...]
set -euo pipefail
NGPUS="${1:-8}"
shift || true
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -m torch.distributed.run --nnodes=1 --nproc-per-node "$NGPUS" \
    --master-addr 127.0.0.1 --master-port "${MASTER_PORT:-29511}" \
    main.py --backend nccl --epochs "${EPOCHS:-10}" --batch_size "${BATCH:-256}" --lr 0.01 --momentum 0.9 \
            --optimizer sgd --metric accuracy --pred_function softmax --precision "${PRECISION:-bf16}" \
            --model_dir "${MODEL_DIR:-model_output}" "$@"
python - <<PY
from src.utils.utils import load_history
h = load_history("${MODEL_DIR:-model_output}")
for e, tl, vl, tm, vm in zip(h["epochs"], h["train_loss"], h["val_loss"], h["train_metric"], h["val_metric"]):
    print(f"epoch {e}: train loss {tl:.4f} acc {tm:.4f} | val loss {vl:.4f} acc {vm:.4f}")
PY
