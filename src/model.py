"""``from src.model import MLModel`` (reference src/model.py:7-24) -> native LeNet."""
from ml_trainer_amd.models import build_model  # noqa: F401
from ml_trainer_amd.models.lenet import MLModel  # noqa: F401

__all__ = ["MLModel", "build_model"]
