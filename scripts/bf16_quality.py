"""bf16 vs fp32 training quality of the fused LeNet engine (writes one JSON line per precision):
the per-epoch train loss / val accuracy trajectories of tests/test_lenet_bf16.py's quality test,
at a configurable size. Usage: python scripts/bf16_quality.py [--epochs 6] [--n 8192] [--out f.jsonl]"""
import argparse
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=6)
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from tests.test_lenet_bf16 import _quality_run
    lines = []
    for p in ("fp32", "bf16"):
        with tempfile.TemporaryDirectory() as d:
            h = _quality_run(p, d, epochs=a.epochs, n_train=a.n)
        rec = {"precision": p, "epochs": a.epochs, "n_train": a.n, "dataset": "SyntheticCIFAR10(learnable='pattern')",
               "train_loss": h["train_loss"], "val_loss": h["val_loss"], "train_acc": h["train_metric"],
               "val_acc": h["val_metric"]}
        lines.append(json.dumps(rec))
        print(lines[-1], flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
