"""LeNet-5 for CIFAR-10 -- the reference model (``src/model.py:7-24``).

``MLModel()`` keeps the reference's exact module names and shapes
(``conv1``/``pool``/``conv2``/``fc1``/``fc2``/``fc3``; 62,006 parameters) and the
flatten order ``c*25 + h*5 + w`` (``src/model.py:20``), so ``model.pth``
checkpoints are interchangeable with the reference and with a stock ``torch.nn``
LeNet.

Configs (BASELINE.json names them; the reference has none -- SURVEY.md §7.1):

* ``default`` -- the reference LeNet (3->6->16 conv, 400->120->84->10).
* ``tiny``    -- same topology at reduced width (3->4->8, 200->64->32->10) for
  the CPU/gloo plumbing config.

On a GPU tensor ``forward`` runs the hand-written gfx950 kernels
(``csrc/kernels/lenet.hip``) through :class:`LeNetFunction`; on CPU it runs the
plain torch ops of the reference. The Trainer's fast path bypasses autograd
altogether and drives the fused step engine (``models/lenet_engine.py``).
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch
import torch.nn.functional as F
from torch import nn

from ml_trainer_amd.ops._ext import require_native

LENET_CONFIGS: Dict[str, Dict[str, int]] = {
    "default": dict(c1=6, c2=16, f1=120, f2=84, cfg_id=0),
    "tiny": dict(c1=4, c2=8, f1=64, f2=32, cfg_id=1),
}


class MLModel(nn.Module):
    """Reference-compatible LeNet. ``MLModel()`` == reference ``MLModel()``."""

    def __init__(self, config: str = "default", num_classes: int = 10):
        super().__init__()
        if config not in LENET_CONFIGS:
            raise ValueError(f"unknown LeNet config {config!r}; choose from {sorted(LENET_CONFIGS)}")
        if num_classes != 10:
            raise ValueError("the native LeNet kernels are built for 10 classes")
        c = LENET_CONFIGS[config]
        self.config = config
        self.cfg_id = c["cfg_id"]
        self.dims = (c["c1"], c["c2"], c["f1"], c["f2"], num_classes)
        self.conv1 = nn.Conv2d(3, c["c1"], 5)
        self.pool = nn.MaxPool2d(2, 2)
        self.conv2 = nn.Conv2d(c["c1"], c["c2"], 5)
        self.fc1 = nn.Linear(c["c2"] * 5 * 5, c["f1"])
        self.fc2 = nn.Linear(c["f1"], c["f2"])
        self.fc3 = nn.Linear(c["f2"], num_classes)

    @property
    def flat_features(self) -> int:
        return self.dims[1] * 25

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:
            return LeNetFunction.apply(x, self.cfg_id, *self.param_list())
        return self.forward_reference(x)

    def forward_reference(self, x: torch.Tensor) -> torch.Tensor:
        """The reference forward in plain torch ops (CPU path, numerics oracle)."""
        x = self.pool(F.relu(self.conv1(x)))
        x = self.pool(F.relu(self.conv2(x)))
        x = x.view(-1, self.flat_features)
        x = F.relu(self.fc1(x))
        x = F.relu(self.fc2(x))
        return self.fc3(x)

    def param_list(self) -> Tuple[torch.Tensor, ...]:
        return (self.conv1.weight, self.conv1.bias, self.conv2.weight, self.conv2.bias, self.fc1.weight,
                self.fc1.bias, self.fc2.weight, self.fc2.bias, self.fc3.weight, self.fc3.bias)


def _align4(n: int) -> int:
    return (n + 3) // 4 * 4


def lenet_buffers(cfg_id: int, B: int, device) -> Dict[str, torch.Tensor]:
    """Activation workspace for the native LeNet kernels at batch ``B``."""
    c1, c2, f1, f2 = (4, 8, 64, 32) if cfg_id == 1 else (6, 16, 120, 84)
    flat = c2 * 25
    f32 = dict(dtype=torch.float32, device=device)
    bufs = {
        "x": torch.empty(B * 3072, **f32),
        "p1": torch.empty(B * c1 * 196, **f32),
        "p2": torch.empty(B * flat, **f32),
        "h1": torch.empty(B * f1, **f32),
        "h2": torch.empty(B * f2, **f32),
        "logits": torch.empty(B * 10, **f32),
        "dlogits": torch.empty(_align4(B * 10), **f32),
        "dh2": torch.empty(B * f2, **f32),
        "dh1": torch.empty(B * f1, **f32),
        "dflat": torch.empty(B * flat, **f32),
        "g1": torch.empty(B * c1 * 196, **f32),
        "slab1": torch.empty(B * c1 * 640, **f32),  # conv wgrad slabs, 2.5 KB per (sample, channel)
        "i1": torch.empty(_align4(B * c1 * 196), dtype=torch.uint8, device=device),
        "i2": torch.empty(_align4(B * flat), dtype=torch.uint8, device=device),
        "targets": torch.zeros(B, dtype=torch.int64, device=device),
        "stats": torch.zeros(2, dtype=torch.float64, device=device),
        # arrival counters of the in-launch last-arriver reductions (zeroed once; reset by the kernel)
        "counters": torch.zeros(16, dtype=torch.int32, device=device),
        # next-step input staging (engine path): K4 gathers the raw uint8 images of the NEXT step
        # into `stage`, tagged in `stage_meta` [B][4] = (perm position, dataset row, target, 0);
        # conv1 uses a staged image only when its tag matches the position it computes (-1 = none)
        "stage": torch.zeros(B * 3072, dtype=torch.uint8, device=device),
        "stage_meta": torch.full((B * 4,), -1, dtype=torch.int64, device=device),
        # per-sample (loss / B, hit / B) of a training step, summed in sample order by K4
        "cestat": torch.zeros(B * 2, dtype=torch.float64, device=device),
        # bf16 MFMA engine (lenet_mfma.hip): raw next-step images staged by the per-sample kernel,
        # tagged (global step, perm position, dataset row, target); metaN = the perm lookup one step
        # further; stepinfo = (step, step in epoch, lr bits) handed to the wgrad kernel
        "stage2": torch.zeros(B * 3072, dtype=torch.uint8, device=device),
        "meta2": torch.full((B * 4,), -1, dtype=torch.int64, device=device),
        "metaN": torch.full((B * 4,), -1, dtype=torch.int64, device=device),
        "stepinfo": torch.zeros(4, dtype=torch.int64, device=device),
        # bf16 engine: the next step's augmented inputs, prepared by the batch-reduction kernel's
        # prep blocks (bf16 pixels, 8 KB per sample) and their (step, position, target) tags
        "prep": torch.zeros(B * 8192, dtype=torch.uint8, device=device),
        "pmeta": torch.full((B * 4,), -1, dtype=torch.int64, device=device),
    }
    return bufs


def _param_names():
    return ["w1", "b1", "w2", "b2", "w3", "b3", "w4", "b4", "w5", "b5"]


def flat_layout(params) -> Tuple[list, int]:
    """16-byte aligned offsets of the 10 LeNet tensors inside one flat buffer."""
    offs, off = [], 0
    for p in params:
        offs.append(off)
        off += _align4(p.numel())
    return offs, off


class LeNetFunction(torch.autograd.Function):
    """Autograd bridge over the native kernels (generic Trainer path / user code)."""

    @staticmethod
    def forward(ctx, x, cfg_id, *params):
        C = require_native()
        x = x.contiguous().float()
        B = x.shape[0]
        if tuple(x.shape[1:]) != (3, 32, 32):
            raise ValueError(f"LeNet expects [B,3,32,32] input, got {tuple(x.shape)}")
        bufs = lenet_buffers(cfg_id, B, x.device)
        bufs["x"] = x.view(-1)
        ps = [p.detach().contiguous() for p in params]
        offs, total = flat_layout(ps)
        gflat = torch.zeros(total, dtype=torch.float32, device=x.device)
        for name, p in zip(_param_names(), ps):
            bufs[name] = p.view(-1)
        for name, p, o in zip(_param_names(), ps, offs):
            bufs["g" + name] = gflat[o:o + p.numel()]
        eng = C.LeNetEngine(cfg_id, B, bufs)
        eng.set_opt(gflat, gflat, None, None, 0, 0.0, 0.0, 0.0, 0.0, 0.9, 0.999, 1e-8, 0.0, 1.0, False, False,
                    None, False, offs)
        eng.run(C.LENET_FWD, B)
        ctx.eng, ctx.bufs, ctx.B, ctx.gflat, ctx.offs = eng, bufs, B, gflat, offs
        ctx.shapes = [p.shape for p in ps]
        ctx.x_requires_grad = x.requires_grad
        ctx.save_for_backward(x, params[0])
        return bufs["logits"].view(B, 10).clone()

    @staticmethod
    def backward(ctx, dlogits):
        C = require_native()
        B = ctx.B
        ctx.bufs["dlogits"][:B * 10].copy_(dlogits.reshape(-1).float())
        ctx.eng.run(C.LENET_BWD, B)
        grads = [ctx.gflat[o:o + int(torch.Size(s).numel())].view(s) for o, s in zip(ctx.offs, ctx.shapes)]
        dx = None
        if ctx.needs_input_grad[0]:
            # conv1 dgrad is never needed by the reference (inputs do not require grad,
            # SURVEY.md §2.7 K1b); computed with torch's conv transpose when asked for.
            x, w1 = ctx.saved_tensors
            g1 = ctx.bufs["g1"].view(B, -1, 14, 14)
            i1 = ctx.bufs["i1"][:g1.numel()].view_as(g1).long()
            dc1 = torch.zeros(B, g1.shape[1], 28, 28, device=g1.device)
            dy, dxo = (i1.clamp(max=3) // 2), (i1.clamp(max=3) % 2)
            ys = torch.arange(14, device=g1.device).view(1, 1, 14, 1) * 2 + dy
            xs = torch.arange(14, device=g1.device).view(1, 1, 1, 14) * 2 + dxo
            dc1.view(B, g1.shape[1], -1).scatter_(2, (ys * 28 + xs).view(B, g1.shape[1], -1),
                                                  g1.reshape(B, g1.shape[1], -1))
            dx = torch.nn.grad.conv2d_input(x.shape, w1.detach(), dc1)
        return (dx, None, *grads)
