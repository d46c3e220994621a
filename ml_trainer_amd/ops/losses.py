"""Losses and metrics with native gfx950 kernels (csrc/kernels/losses.hip).

``CrossEntropyLoss`` is the reference's default criterion
(``src/trainer.py:141-142``); on device tensors it runs one fused
softmax-cross-entropy kernel (loss + gradient in one pass, no host sync),
on CPU the plain torch op. ``accuracy`` is the reference's sklearn metric
(``src/trainer.py:164-166``) computed on device: first arg-max == target,
averaged over the batch, returned as a device scalar.

The other reference criteria (``src/trainer.py:143-148``: 'neg-loss' = NLL,
'l1', 'l2', and the custom MSE of ``src/utils/functions.py:15-17``) and the
'mcrmse' metric (``src/trainer.py:161-163``) run on the regression kernels of
the same file: fixed-order two-pass reductions (bitwise reproducible), the
forward also writing the unscaled elementwise gradient, the backward one
scale by grad_out / n. Differences from torch: a batch whose NLL targets are
all ``ignore_index`` gives 0 instead of nan.
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


_PARTIALS = {}


def _partials(dev: torch.device) -> torch.Tensor:
    """Per-device scratch for the block partials of the regression reductions (reused: the
    finalize kernel consumes them in stream order before the next forward can overwrite them)."""
    key = (dev.type, dev.index)
    buf = _PARTIALS.get(key)
    if buf is None:
        buf = torch.empty(require_native().loss_partials_needed(), dtype=torch.float32, device=dev)
        _PARTIALS[key] = buf
    return buf


def _f32(x: torch.Tensor) -> torch.Tensor:
    return x.contiguous() if x.dtype == torch.float32 else x.float().contiguous()


class _PointwiseLossFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target, mode):
        C = require_native()
        p, t = _f32(pred), _f32(target)
        g = torch.empty_like(p)
        stats = torch.empty(2, dtype=torch.float32, device=p.device)
        C.pointwise_loss_fwd(p, t, int(mode), g, _partials(p.device), stats)
        ctx.save_for_backward(g, stats)
        ctx.pred_dtype = pred.dtype
        ctx.tgt_grad = target.requires_grad
        return stats[0].clone()

    @staticmethod
    def backward(ctx, gout):
        C = require_native()
        g, stats = ctx.saved_tensors
        d = torch.empty_like(g)
        C.loss_scale_grad(g, gout.reshape(1).float().contiguous(), stats, d)
        return d.to(ctx.pred_dtype), (-d if ctx.tgt_grad else None), None


class _NLLFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logp, targets, ignore_index):
        C = require_native()
        lp = _f32(logp)
        t = targets.contiguous().to(torch.int64)
        stats = torch.empty(2, dtype=torch.float32, device=lp.device)
        C.nll_fwd(lp, t, int(ignore_index), _partials(lp.device), stats)
        ctx.save_for_backward(t, stats)
        ctx.shape = lp.shape
        ctx.ignore_index = int(ignore_index)
        ctx.in_dtype = logp.dtype
        return stats[0].clone()

    @staticmethod
    def backward(ctx, gout):
        C = require_native()
        t, stats = ctx.saved_tensors
        d = torch.empty(ctx.shape, dtype=torch.float32, device=t.device)
        C.nll_bwd(t, ctx.shape[1], ctx.ignore_index, gout.reshape(1).float().contiguous(), stats, d)
        return d.to(ctx.in_dtype), None, None


def _native_ok(*ts: torch.Tensor) -> bool:
    return all(t.is_cuda for t in ts)


class L1Loss(nn.Module):
    """Mean absolute error (reference criterion 'l1', ``src/trainer.py:145-146``)."""

    def forward(self, pred, target):
        if _native_ok(pred, target) and pred.shape == target.shape and target.is_floating_point():
            return _PointwiseLossFunction.apply(pred, target, 0)
        return F.l1_loss(pred, target)


class MSELoss(nn.Module):
    """Mean squared error (reference criterion 'l2' and the custom loss
    ``mean((o - t) ** 2)`` of ``src/utils/functions.py:15-17``)."""

    def forward(self, pred, target):
        if _native_ok(pred, target) and pred.shape == target.shape and target.is_floating_point():
            return _PointwiseLossFunction.apply(pred, target, 1)
        return F.mse_loss(pred, target)


class NLLLoss(nn.Module):
    """Mean negative log-likelihood over log-probabilities (reference criterion 'neg-loss')."""

    def __init__(self, ignore_index: int = -100):
        super().__init__()
        self.ignore_index = ignore_index

    def forward(self, logp, targets):
        if _native_ok(logp, targets) and logp.dim() == 2 and targets.dtype in (torch.int64, torch.int32):
            return _NLLFunction.apply(logp, targets, self.ignore_index)
        return F.nll_loss(logp, targets, ignore_index=self.ignore_index)


def mcrmse(outputs: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
    """Mean column-wise RMSE (reference metric 'mcrmse', ``src/trainer.py:161-163``), device scalar."""
    if _native_ok(outputs, targets) and outputs.dim() == 2 and outputs.shape == targets.shape:
        C = require_native()
        p, t = _f32(outputs), _f32(targets)
        col = torch.empty(p.shape[1], dtype=torch.float32, device=p.device)
        out = torch.empty(1, dtype=torch.float32, device=p.device)
        C.mcrmse(p, t, col, out)
        return out.view(())
    colwise_mse = torch.mean(torch.square(targets - outputs), dim=0)
    return torch.mean(torch.sqrt(colwise_mse), dim=0)
