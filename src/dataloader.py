"""``from src.dataloader import Loader`` (reference src/dataloader.py:5-6)."""
from ml_trainer_amd.data.loader import Loader  # noqa: F401

__all__ = ["Loader"]
