"""User hooks of the reference (``src/utils/functions.py:5-17``).

``custom_pre_process_function()`` returns the reference augmentation built from
this framework's torchvision-compatible transforms; the Trainer maps it onto the
fused GPU augmentation kernel when the dataset lives in HBM.
"""
import torch

from ml_trainer_amd.data import transforms


def custom_pre_process_function():
    transform = transforms.Compose([
        transforms.RandomCrop(32, padding=4),
        transforms.RandomHorizontalFlip(),
        transforms.ToTensor(),
        transforms.Normalize((0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010)),
    ])
    return transform


def custom_loss_function(output, target):
    """``mean((output - target) ** 2)``; same-shape device tensors take the native MSE kernel."""
    if output.is_cuda and target.is_cuda and output.shape == target.shape and target.is_floating_point():
        from ml_trainer_amd.ops.losses import MSELoss
        return MSELoss()(output, target)
    return torch.mean((output - target) ** 2)
