"""``from src.trainer import Trainer`` (reference src/trainer.py) -> ml_trainer_amd.trainer."""
from ml_trainer_amd.config import TrainerOptions  # noqa: F401
from ml_trainer_amd.trainer import Trainer  # noqa: F401

__all__ = ["Trainer", "TrainerOptions"]
