"""CLI entrypoint (reference ``main.py:1-84``): same flags and defaults.

    python main.py --optimizer sgd --lr 0.001 --momentum 0.9 --backend smddp ...
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 main.py ...

Fixes over the reference: ``--epochs`` / ``--batch_size``
are honoured (the reference hard-codes 250 / 32), ``--custom_function`` parses
booleans properly, the SageMaker ``SM_*`` environment variables are optional
(defaults: model_dir ``model_output``, data_dir ``cifar10-dataset``), and a
dataset without transform yields tensors instead of crashing default_collate.
When ``--data_dir`` holds no CIFAR-10 batches (there is no network to download
them) ``--synthetic`` (or a missing directory) falls back to a seeded synthetic
CIFAR-shaped dataset and says so in the log.

Extension flags (not in the reference): ``--model`` (default/tiny/bert-base/
large), ``--synthetic``, ``--per_device_batch``, ``--no_engine``,
``--no_parallel``, ``--resume``, ``--amp bf16``, ``--precision bf16``, ``--metrics_jsonl``, ``--log_jsonl``, ``--zero_stage``, ``--async_checkpoint``.
"""
from __future__ import annotations

import argparse
import json
import os

from ml_trainer_amd.utils.logging import get_logger

logger = get_logger("main")


def str2bool(v) -> bool:
    if isinstance(v, bool):
        return v
    s = str(v).strip().lower()
    if s in ("1", "true", "t", "yes", "y"):
        return True
    if s in ("0", "false", "f", "no", "n", "none", ""):
        return False
    raise argparse.ArgumentTypeError(f"boolean expected, got {v!r}")


def build_datasets(args):
    from ml_trainer_amd.data.cifar10 import CIFAR10, SyntheticCIFAR10
    tf = None
    if args.custom_function:
        from ml_trainer_amd.utils.functions import custom_pre_process_function
        tf = custom_pre_process_function()
    use_synth = args.synthetic
    if not use_synth:
        try:
            train_set = CIFAR10(root=args.data_dir, train=True, download=False, transform=tf)
            val_set = CIFAR10(root=args.data_dir, train=False, download=False, transform=tf)
            return train_set, val_set
        except FileNotFoundError as e:
            logger.warning("CIFAR-10 not found; using synthetic CIFAR-shaped data", error=str(e))
    n_train = args.synthetic_size or 50000
    return (SyntheticCIFAR10(n_train, train=True, transform=tf, seed=args.seed),
            SyntheticCIFAR10(max(n_train // 5, 1), train=False, transform=tf, seed=args.seed))


def main(args):
    import torch
    from ml_trainer_amd.models import build_model
    from ml_trainer_amd.trainer import Trainer
    torch.manual_seed(args.seed)
    model = build_model(args.model)
    if args.model in ("default", "tiny", "lenet"):
        datasets = build_datasets(args)
    else:  # BERT configs: synthetic token classification (no network for GLUE downloads)
        from ml_trainer_amd.data.text import SyntheticTextClassification
        c = model.config
        seq = min(args.seq_len, c.max_position)
        n = args.synthetic_size or 4096
        datasets = (SyntheticTextClassification(n, seq_len=seq, vocab_size=c.vocab_size, num_labels=c.num_labels,
                                                seed=args.seed, learnable=True),
                    SyntheticTextClassification(max(n // 8, 1), seq_len=seq, vocab_size=c.vocab_size,
                                                num_labels=c.num_labels, seed=args.seed + 1, learnable=True))
    config = {
        "seed": args.seed,
        "scheduler": args.scheduler,
        "optimizer": args.optimizer,
        "momentum": args.momentum,
        "weight_decay": args.weight_decay,
        "lr": args.lr,
        "criterion": args.criterion,
        "pred_function": args.pred_function,
        "metric": args.metric,
        "model_dir": args.model_dir,
        "backend": args.backend,
    }
    options = {"per_device_batch": args.per_device_batch, "resume": args.resume,
               "metrics_jsonl": args.metrics_jsonl, "amp": args.amp, "progress": not args.no_progress,
               "precision": getattr(args, "precision", "fp32"),
               "zero_stage": args.zero_stage, "async_checkpoint": args.async_checkpoint}
    if args.no_engine:
        options["use_engine"] = False
    if args.log_jsonl:  # every structured log record, one JSON object per line
        from ml_trainer_amd.utils.logging import add_jsonl_sink
        add_jsonl_sink(args.log_jsonl)
    trainer = Trainer(model, datasets=datasets, epochs=args.epochs, batch_size=args.batch_size,
                      is_parallel=not args.no_parallel, save_history=True, options=options, **config)
    trainer.fit()
    return trainer


def build_parser() -> argparse.ArgumentParser:
    parser = argparse.ArgumentParser()
    parser.add_argument("--batch_size", type=int, default=32, help="input batch size for training (default: 32)")
    parser.add_argument("--epochs", type=int, default=10, help="number of epochs to train (default: 10)")
    parser.add_argument("--optimizer", type=str, default="sgd", help="optimizer for backward pass (default: sgd)")
    parser.add_argument("--lr", type=float, default=0.001, help="learning rate (default: 0.001)")
    parser.add_argument("--momentum", type=float, default=0.9, help="Optimizer momentum (default: 0.9)")
    parser.add_argument("--weight_decay", type=float, default=0.0, help="Optimizer weight decay (default: 0.0)")
    parser.add_argument("--seed", type=int, default=32, help="random seed (default: 32)")
    parser.add_argument("--scheduler", type=str, default=None,
                        help="apply scheduler for learning rate (default: None)")
    parser.add_argument("--criterion", type=str, default="cross_entropy",
                        help="loss function to apply (default: cross_entropy)")
    parser.add_argument("--metric", type=str, default=None, help="metric for model evaluation (default: None)")
    parser.add_argument("--backend", type=str, default="smddp",
                        help="backend for dist. training: smddp|rccl|nccl (RCCL over xGMI) or gloo")
    parser.add_argument("--custom_function", type=str2bool, default=False,
                        help="apply a pre-processing function (default: False)")
    parser.add_argument("--pred_function", type=str, default=None,
                        help="probability function to apply to make predictions (default: None)")
    # SageMaker environment (optional here)
    parser.add_argument("--hosts", type=json.loads, default=json.loads(os.environ.get("SM_HOSTS", "[]")))
    parser.add_argument("--current-host", type=str, default=os.environ.get("SM_CURRENT_HOST", "localhost"))
    parser.add_argument("--model_dir", type=str, default=os.environ.get("SM_MODEL_DIR", "model_output"))
    parser.add_argument("--data_dir", type=str, default=os.environ.get("SM_CHANNEL_TRAIN", "cifar10-dataset"))
    # extensions
    parser.add_argument("--model", type=str, default="default", help="default|tiny|bert-base|large")
    parser.add_argument("--synthetic", action="store_true", help="use the seeded synthetic dataset")
    parser.add_argument("--synthetic_size", type=int, default=0)
    parser.add_argument("--seq_len", type=int, default=512)
    parser.add_argument("--per_device_batch", action="store_true",
                        help="batch_size is per GPU (weak scaling) instead of global")
    parser.add_argument("--no_engine", action="store_true", help="disable the fused LeNet step engine")
    parser.add_argument("--no_parallel", action="store_true", help="do not initialise torch.distributed")
    parser.add_argument("--resume", action="store_true")
    parser.add_argument("--async_checkpoint", action="store_true",
                        help="write model.pth / trainer_state.pt from a pinned-host snapshot in a background thread")
    parser.add_argument("--zero_stage", type=int, default=0, choices=(0, 1),
                        help="1: ZeRO-1 sharded optimizer state (reduce-scatter / all-gather) under DDP")
    parser.add_argument("--amp", type=str, default=None, choices=[None, "bf16"])
    parser.add_argument("--precision", type=str, default="fp32", choices=["fp32", "bf16"],
                        help="fused LeNet step: fp32 (reference dtype) or bf16 MFMA (fp32 masters)")
    parser.add_argument("--metrics_jsonl", type=str, default=None)
    parser.add_argument("--log_jsonl", type=str, default=None, help="mirror log records into this JSON-lines file")
    parser.add_argument("--no_progress", action="store_true")
    return parser


if __name__ == "__main__":
    main(build_parser().parse_args())
