"""``src.utils.utils`` (reference src/utils/utils.py:9-68)."""
from ml_trainer_amd.utils.utils import load_history, load_model, plot_history  # noqa: F401

__all__ = ["load_history", "load_model", "plot_history"]
