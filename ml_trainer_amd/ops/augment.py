"""GPU-side CIFAR augmentation iterator for the generic (non-engine) path.

Yields ``(x [B,3,32,32] fp32, y [B] int64)`` device batches produced by the
``cifar_augment`` kernel from an HBM-resident uint8 dataset: RandomCrop(32,
pad) + RandomHorizontalFlip + ToTensor + Normalize exactly as
``src/utils/functions.py:5-12`` specifies, with a counter-based RNG
(reproducible, no host work per batch beyond the launch).
"""
from __future__ import annotations

import torch

from ml_trainer_amd.ops._ext import require_native


class DeviceAugmentIterator:
    def __init__(self, dd, indices: torch.Tensor, batch_size: int, seed: int = 0, step0: int = 0,
                 advance_step: bool = True):
        self.C = require_native()
        self.dd = dd
        self.idx = indices.to(torch.int32).to(dd.device)
        self.B = int(batch_size)
        self.seed = int(seed)
        self.step0 = int(step0)
        self.advance = advance_step  # eval passes keep one RNG step per epoch (same as the engine's eval)
        self.n = self.idx.numel()

    def __len__(self):
        return (self.n + self.B - 1) // self.B

    def __iter__(self):
        s = self.dd.spec
        for i in range(len(self)):
            b = min(self.B, self.n - i * self.B)
            x = torch.empty(b, 3, 32, 32, dtype=torch.float32, device=self.dd.device)
            y = torch.empty(b, dtype=torch.int64, device=self.dd.device)
            self.C.cifar_augment(self.dd.data, self.idx, None, self.dd.targets, x, y, self.seed, s["pad"],
                                 1 if s["flip"] else 0, self.B, list(s["mean"]), list(s["std"]), b,
                                 self.step0 + (i if self.advance else 0), i)
            yield x, y
