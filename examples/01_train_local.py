"""Local training walkthrough: the flow of the reference's ``01_ML_Training_local.ipynb``
(cells :29-32 imports, :56-97 datasets with augmentation, :162-174 config, :202 Trainer,
:417 fit, :439 save_history_, :476 plot_history, :505-507 load_model + test) as a script.

    python examples/01_train_local.py --epochs 6                # CIFAR-10 if --data_dir has it
    python examples/01_train_local.py --epochs 1 --synthetic --n_train 2048 --n_val 512

Uses the reference import paths (``src.*``); on a GPU the Trainer runs the fused native
LeNet step engine, on CPU the eager path.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from src.dataloader import Loader  # noqa: E402
from src.model import MLModel  # noqa: E402
from src.trainer import Trainer  # noqa: E402
from src.utils.functions import custom_pre_process_function  # noqa: E402
from src.utils.utils import load_history, load_model, plot_history  # noqa: E402


def datasets(args):
    from ml_trainer_amd.data.cifar10 import CIFAR10, SyntheticCIFAR10
    tf = custom_pre_process_function()
    if not args.synthetic:
        try:
            return (CIFAR10(args.data_dir, train=True, transform=tf),
                    CIFAR10(args.data_dir, train=False, transform=tf))
        except (FileNotFoundError, OSError):
            print(f"no CIFAR-10 batches under {args.data_dir!r}: using the synthetic dataset")
    return (SyntheticCIFAR10(args.n_train, train=True, transform=tf, learnable=True),
            SyntheticCIFAR10(args.n_val, train=False, transform=tf, learnable=True))


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--data_dir", default="cifar10-dataset")
    p.add_argument("--synthetic", action="store_true")
    p.add_argument("--n_train", type=int, default=None)
    p.add_argument("--n_val", type=int, default=None)
    p.add_argument("--epochs", type=int, default=6)
    p.add_argument("--batch_size", type=int, default=32)
    p.add_argument("--model_dir", default="model_output")
    p.add_argument("--plot", default="", help="write the history plot to this PNG (needs matplotlib)")
    args = p.parse_args(argv)

    train_set, val_set = datasets(args)
    counts = torch.bincount(torch.as_tensor(train_set.targets), minlength=10).tolist()
    print("class counts:", dict(zip(train_set.classes, counts)))  # notebook :226-232

    config = {"seed": 32, "scheduler": None, "optimizer": "sgd", "momentum": 0.9, "weight_decay": 0.0,
              "lr": 0.001, "criterion": "cross_entropy", "metric": "accuracy", "pred_function": "softmax",
              "model_dir": args.model_dir}
    trainer = Trainer(MLModel(), (train_set, val_set), epochs=args.epochs, batch_size=args.batch_size,
                      **config)
    trainer.fit()
    trainer.save_history_(args.model_dir)
    history = load_history(args.model_dir)
    if args.plot:
        try:
            plot_history(history, show=False).savefig(args.plot)
        except ImportError:
            print("matplotlib is not installed: skipping the plot")

    model = load_model(MLModel(), os.path.join(args.model_dir, "model.pth"))
    loss, acc = trainer.test(model, trainer.val_loader)
    print(f"test loss={float(loss):.4f} accuracy={float(acc):.4f}")
    return history, float(loss), float(acc)


if __name__ == "__main__":
    main()
