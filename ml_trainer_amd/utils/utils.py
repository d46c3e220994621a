"""Post-processing utilities (reference ``src/utils/utils.py:9-68``).

* ``load_history(dir)`` -- reads ``dir/history.pkl`` with a restricted
  unpickler (plain containers / numbers / strings only: a history file can not
  execute code);
* ``load_model(model, PATH)`` -- loads ``model.pth`` with
  ``torch.load(weights_only=True)``, stripping the ``module.`` prefix of DDP
  checkpoints and falling back to the raw keys (the reference's try/except
  behaviour, ``src/utils/utils.py:15-28``);
* ``plot_history(history)`` -- loss / metric curves (tick logic changes above
  25 epochs, as in the reference).
"""
from __future__ import annotations

import os
import pickle
from collections import OrderedDict

import numpy as np
import torch


class _HistoryUnpickler(pickle.Unpickler):
    _SAFE = {("builtins", "list"), ("builtins", "dict"), ("builtins", "tuple"), ("builtins", "float"),
             ("builtins", "int"), ("builtins", "str"), ("collections", "OrderedDict"),
             ("numpy", "float64"), ("numpy", "float32"), ("numpy.core.multiarray", "scalar"),
             ("numpy._core.multiarray", "scalar"), ("numpy", "dtype")}

    def find_class(self, module, name):
        if (module, name) in self._SAFE:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"history.pkl may only contain plain data, found {module}.{name}")


def load_history(file_dir):
    path = os.path.join(file_dir, "history.pkl")
    with open(path, "rb") as f:
        return _HistoryUnpickler(f).load()


def load_model(model, PATH):
    state_dict = torch.load(PATH, map_location="cpu", weights_only=True)
    try:
        # If model was trained in parallel: drop the `module.` prefix
        new_state_dict = OrderedDict()
        for k, v in state_dict.items():
            new_state_dict[k[7:] if k.startswith("module.") else k] = v
        model.load_state_dict(new_state_dict)
    except Exception:
        model.load_state_dict(state_dict)
    return model


def plot_history(history: dict, show: bool = True):
    import matplotlib
    if not show:
        matplotlib.use("Agg")
    from matplotlib import pyplot as plt
    x = history["epochs"]
    train_loss = history["train_loss"]
    val_loss = history["val_loss"]
    if history["metric_type"] is not None:
        train_metric = history["train_metric"]
        val_metric = history["val_metric"]
        fig, axes = plt.subplots(2, 1, figsize=(10, 10))
        axes[0].plot(x, train_loss, c="C0", label="train")
        axes[0].plot(x, val_loss, c="C1", label="validation")
        axes[1].plot(x, train_metric, c="C0", label="train")
        axes[1].plot(x, val_metric, c="C1", label="validation")
        if len(x) > 25:
            for ax in axes:
                ax.set_xticks(np.arange(0, len(x) + 1, 5))
                ax.set_xticklabels(np.arange(0, len(x) + 1, 5), rotation=45)
        else:
            axes[0].set_xticks(x)
            axes[1].set_xticks(x)
        axes[0].set_xlabel("Epochs")
        axes[0].set_ylabel("Loss")
        axes[1].set_ylabel(history["metric_type"])
        axes[0].set_title("Training Loss vs. Validation Loss")
        axes[1].set_title(f"{history['metric_type']} - Training vs. Validation")
        axes[0].legend()
        axes[1].legend()
    else:
        fig = plt.figure(figsize=(10, 5))
        plt.plot(x, train_loss, c="C0", label="train")
        plt.plot(x, val_loss, c="C1", label="validation")
        plt.xticks(x, rotation=45)
        plt.xlabel("Epochs")
        plt.ylabel("Loss")
        plt.title("Training Loss vs. Validation Loss")
        plt.legend()
    plt.tight_layout()
    if show:
        plt.show()
    return fig
