"""The notebook-equivalent example scripts (reference 01/03 notebooks) run end to end on CPU."""
import importlib.util
import os

import pytest

ROOT = os.path.join(os.path.dirname(__file__), "..")


def _load(name):
    spec = importlib.util.spec_from_file_location(name.replace(".py", ""), os.path.join(ROOT, "examples", name))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.timeout(300)
def test_train_local_then_test(tmp_path):
    out = str(tmp_path / "out")
    hist, loss, acc = _load("01_train_local.py").main(
        ["--epochs", "1", "--synthetic", "--n_train", "256", "--n_val", "64", "--model_dir", out])
    assert hist["epochs"] == [1] and set(hist) >= {"train_loss", "val_loss", "train_metric", "val_metric"}
    assert os.path.exists(os.path.join(out, "model.pth"))
    loss2, acc2 = _load("03_test.py").main(
        ["--model_path", os.path.join(out, "model.pth"), "--synthetic", "--n_val", "64"])
    # same checkpoint and val set; random crop/flip augmentation differs between the two passes
    assert abs(loss2 - loss) < 0.05 and 0.0 <= acc2 <= 1.0


def test_distributed_example_runs_config3_bf16():
    """examples/02 (the SageMaker-distributed flow) trains BASELINE config 3 -- the bf16 step --
    unless PRECISION overrides it; main.py's own default stays the reference dtype (fp32)."""
    import shlex
    src = open(os.path.join(ROOT, "examples", "02_train_distributed.sh")).read()
    cmd = " ".join(l.rstrip("\\") for l in src.splitlines() if not l.lstrip().startswith("#"))
    toks = shlex.split(cmd.replace('"${PRECISION:-bf16}"', "bf16"), posix=True)
    i = toks.index("--precision")
    assert toks[i + 1] == "bf16"
    import main
    assert main.build_parser().parse_args([]).precision == "fp32"
