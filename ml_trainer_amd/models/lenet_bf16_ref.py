"""Plain-torch reference of one bf16 LeNet training step (csrc/kernels/lenet_mfma.hip).

The native step rounds to bf16 exactly where an MFMA operand is formed and nowhere else:

* the (augmented) input image, the conv weights, the pooled conv1 map (conv2's input), the
  unpooled conv2-output gradient (conv2 dgrad / wgrad operand), the unpooled conv1-output
  gradient (conv1 wgrad operand), the fc weights, and every fc layer's input row / output
  gradient row (the fc forward and backward-data products run on the matrix cores);
* every sum is accumulated in fp32 (here: float64); the stored activations and gradients (ReLU
  masks, biases, softmax), the loss, every weight gradient and the optimizer stay fp32.

``lenet_bf16_grads`` reproduces those rounding points in float64, so the kernel can be checked to
within fp32 accumulation-order noise. With ``rnd=identity`` it is the exact fp32 model
(reference ``src/model.py:17-24`` + ``F.cross_entropy``), which the CPU tests check against
autograd -- that pins the index math of the hand-written backward (unpooling, transposed
convolution, weight-gradient correlations) independently of any GPU.
"""
from __future__ import annotations

from typing import Callable, Dict, Tuple

import torch
import torch.nn.functional as F


def bf16_round(t: torch.Tensor) -> torch.Tensor:
    """Round-to-nearest-even to bf16, returned in t's dtype."""
    return t.to(torch.bfloat16).to(t.dtype)


def _pool_codes(c: torch.Tensor, bias: torch.Tensor):
    """2x2/2 max-pool + bias + ReLU as the kernel does it: first maximum of the window in
    (0,0),(0,1),(1,0),(1,1) order (strict >), bias added after the max, dead cells (max <= 0)
    code 4. Returns pooled values, codes [B,C,H/2,W/2] and the liveness mask."""
    B, C, H, W = c.shape
    win = c.view(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, H // 2, W // 2, 4)
    m = win[..., 0].clone()
    code = torch.zeros_like(m, dtype=torch.int64)
    for k in range(1, 4):
        gt = win[..., k] > m
        m = torch.where(gt, win[..., k], m)
        code = torch.where(gt, torch.full_like(code, k), code)
    m = m + bias.view(1, C, 1, 1)
    alive = m > 0
    return torch.where(alive, m, torch.zeros_like(m)), code, alive


def _unpool(g: torch.Tensor, code: torch.Tensor, alive: torch.Tensor) -> torch.Tensor:
    """Route each pooled cell's gradient to its arg-max position (dead cells drop it)."""
    B, C, h, w = g.shape
    out = torch.zeros(B, C, h, w, 4, dtype=g.dtype)
    out.scatter_(4, code.unsqueeze(-1), torch.where(alive, g, torch.zeros_like(g)).unsqueeze(-1))
    return out.view(B, C, h, w, 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, 2 * h, 2 * w)


def lenet_bf16_grads(params: Dict[str, torch.Tensor], x: torch.Tensor, y: torch.Tensor,
                     rnd: Callable[[torch.Tensor], torch.Tensor] = bf16_round
                     ) -> Tuple[float, float, Dict[str, torch.Tensor]]:
    """Loss, accuracy and parameter gradients of one step (mean cross-entropy over the batch).

    ``params``: conv1.weight, conv1.bias, ..., fc3.bias (any device / dtype; computed on CPU in
    float64). ``x`` [B,3,32,32] is the normalised input before rounding; ``y`` [B] labels."""
    d = torch.float64
    P = {k: v.detach().to("cpu", d) for k, v in params.items()}
    x = x.detach().to("cpu", d)
    y = y.detach().to("cpu")
    B = x.shape[0]
    w1, w2 = rnd(P["conv1.weight"]), rnd(P["conv2.weight"])
    w3, w4, w5 = rnd(P["fc1.weight"]), rnd(P["fc2.weight"]), rnd(P["fc3.weight"])
    xb = rnd(x)
    # forward
    p1, code1, alive1 = _pool_codes(F.conv2d(xb, w1), P["conv1.bias"])
    p1b = rnd(p1)
    p2, code2, alive2 = _pool_codes(F.conv2d(p1b, w2), P["conv2.bias"])
    f = p2.reshape(B, -1)
    h1 = torch.relu(rnd(f) @ w3.t() + P["fc1.bias"])  # fc1 on the matrix cores: bf16 input row
    h2 = torch.relu(rnd(h1) @ w4.t() + P["fc2.bias"])
    logits = rnd(h2) @ w5.t() + P["fc3.bias"]
    loss = F.cross_entropy(logits, y)
    acc = (logits.argmax(1) == y).double().mean()
    # backward
    dlog = (torch.softmax(logits, 1) - F.one_hot(y, logits.shape[1]).to(d)) / B
    dh2 = (rnd(dlog) @ w5) * (h2 > 0)
    dh1 = (rnd(dh2) @ w4) * (h1 > 0)
    dflat = rnd(dh1) @ w3  # fc1 dgrad on the matrix cores: bf16 gradient row
    dc = rnd(_unpool(dflat.view_as(p2), code2, alive2))
    g1 = torch.nn.grad.conv2d_input(p1b.shape, w2, dc)
    d1 = rnd(_unpool(g1, code1, alive1))
    g = {
        "fc3.weight": dlog.t() @ h2, "fc3.bias": dlog.sum(0),
        "fc2.weight": dh2.t() @ h1, "fc2.bias": dh2.sum(0),
        "fc1.weight": dh1.t() @ f, "fc1.bias": dh1.sum(0),
        "conv2.weight": torch.nn.grad.conv2d_weight(p1b, w2.shape, dc), "conv2.bias": dc.sum((0, 2, 3)),
        "conv1.weight": torch.nn.grad.conv2d_weight(xb, w1.shape, d1), "conv1.bias": d1.sum((0, 2, 3)),
    }
    return float(loss), float(acc), g
