"""``src.utils.functions`` (reference src/utils/functions.py:5-17)."""
from ml_trainer_amd.utils.functions import custom_loss_function, custom_pre_process_function  # noqa: F401

__all__ = ["custom_pre_process_function", "custom_loss_function"]
