"""Losses and metrics with native gfx950 kernels (csrc/kernels/losses.hip).

``CrossEntropyLoss`` is the reference's default criterion
(``src/trainer.py:141-142``); on device tensors it runs one fused
softmax-cross-entropy kernel (loss + gradient in one pass, no host sync),
on CPU the plain torch op. ``accuracy`` is the reference's sklearn metric
(``src/trainer.py:164-166``) computed on device: first arg-max == target,
averaged over the batch, returned as a device scalar.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from ml_trainer_amd.ops._ext import require_native


class _CEFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, targets, ignore_index, label_smoothing):
        C = require_native()
        z = logits.contiguous()
        if z.dtype not in (torch.float32, torch.bfloat16):
            z = z.float()
        t = targets.contiguous().to(torch.int64)
        B, K = z.shape
        dl = torch.empty(B, K, dtype=torch.float32, device=z.device)
        acc = torch.zeros(2, dtype=torch.float32, device=z.device)
        loss = torch.empty(1, dtype=torch.float32, device=z.device)
        C.ce_fwd(z, t, dl, acc, None, loss, int(ignore_index), float(label_smoothing))
        ctx.save_for_backward(dl, acc)
        ctx.out_dtype = logits.dtype
        return loss.view(())

    @staticmethod
    def backward(ctx, gout):
        C = require_native()
        dl, acc = ctx.saved_tensors
        out = torch.empty(dl.shape, dtype=ctx.out_dtype if ctx.out_dtype in (torch.float32, torch.bfloat16)
                          else torch.float32, device=dl.device)
        C.ce_bwd(dl, gout.reshape(1).float().contiguous(), acc, out)
        return out, None, None, None


class CrossEntropyLoss(nn.Module):
    """Mean-reduced softmax cross-entropy (torch semantics incl. ignore_index / label_smoothing)."""

    def __init__(self, ignore_index: int = -100, label_smoothing: float = 0.0):
        super().__init__()
        self.ignore_index = ignore_index
        self.label_smoothing = label_smoothing

    def forward(self, logits: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
        if logits.is_cuda and logits.dim() == 2 and targets.dtype in (torch.int64, torch.int32):
            return _CEFunction.apply(logits, targets, self.ignore_index, self.label_smoothing)
        return F.cross_entropy(logits, targets, ignore_index=self.ignore_index,
                               label_smoothing=self.label_smoothing)


def accuracy(logits: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
    """Batch accuracy (device scalar): mean(first argmax(logits) == targets)."""
    if logits.is_cuda and logits.dim() == 2:
        C = require_native()
        z = logits.contiguous()
        if z.dtype not in (torch.float32, torch.bfloat16):
            z = z.float()
        out = torch.zeros(1, dtype=torch.float32, device=z.device)
        C.accuracy(z, targets.contiguous().to(torch.int64), out)
        return out.view(())
    return (torch.argmax(logits, dim=-1) == targets).float().mean()
