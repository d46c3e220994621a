"""Evaluation of a saved checkpoint: the reference's ``03_ML_Testing.ipynb`` (:89 val loader,
:100-101 load_model, :124 ``Trainer(model)`` test-only mode, :150 ``trainer.test``).

    python examples/03_test.py --model_path model_output/model.pth [--synthetic]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from src.dataloader import Loader  # noqa: E402
from src.model import MLModel  # noqa: E402
from src.trainer import Trainer  # noqa: E402
from src.utils.functions import custom_pre_process_function  # noqa: E402
from src.utils.utils import load_model  # noqa: E402


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--model_path", default="model_output/model.pth")
    p.add_argument("--data_dir", default="cifar10-dataset")
    p.add_argument("--synthetic", action="store_true")
    p.add_argument("--n_val", type=int, default=None)
    args = p.parse_args(argv)
    from ml_trainer_amd.data.cifar10 import CIFAR10, SyntheticCIFAR10
    tf = custom_pre_process_function()
    val_set = None
    if not args.synthetic:
        try:
            val_set = CIFAR10(args.data_dir, train=False, transform=tf)
        except (FileNotFoundError, OSError):
            print(f"no CIFAR-10 batches under {args.data_dir!r}: using the synthetic dataset")
    if val_set is None:
        val_set = SyntheticCIFAR10(args.n_val, train=False, transform=tf, learnable=True)
    test_loader = Loader(val_set, 32, shuffle=True)
    model = load_model(MLModel(), args.model_path)
    trainer = Trainer(model)  # no datasets: "Testing only available."
    loss, acc = trainer.test(model, test_loader)
    print(f"test loss={float(loss):.4f} accuracy={float(acc):.4f}")
    return float(loss), float(acc)


if __name__ == "__main__":
    main()
