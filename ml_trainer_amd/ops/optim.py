"""Fused flat-buffer optimizers: SGD / Adam / AdamW / Adagrad / Adamax.

The reference builds one of five ``torch.optim`` optimizers by name
(``src/trainer.py:123-138``). These classes are drop-in ``torch.optim.Optimizer``
subclasses (so ``torch.optim.lr_scheduler`` works on them unchanged) whose
``step()`` is ONE HIP launch over the contiguous parameter buffer of each param
group (``csrc/kernels/optim.hip``), with the exact torch update rules
(``csrc/include/mlt_optim.h``).

State lives in flat buffers (``exp_avg`` etc. as one tensor per group) instead
of per-parameter dicts; ``state_dict()``/``load_state_dict()`` round-trip it.
On CPU tensors the same math runs as vectorised torch ops over the flat buffers
(plumbing config).
"""
from __future__ import annotations

import math
from typing import Any, Dict, List, Optional

import torch

from ml_trainer_amd.ops._ext import require_native
from ml_trainer_amd.utils.flat import FlatParams

KIND = {"sgd": 0, "adam": 1, "adamw": 2, "adagrad": 3, "adamax": 4}


class FusedOptimizer(torch.optim.Optimizer):
    kind_name = "sgd"

    def __init__(self, params, defaults: Dict[str, Any], flat: Optional[FlatParams] = None):
        super().__init__(params, defaults)
        self.kind = KIND[self.kind_name]
        self._flats: List[FlatParams] = []
        for gi, group in enumerate(self.param_groups):
            ps = group["params"]
            # reuse the caller's flat buffer (e.g. DDP's, laid out in reverse order) when it holds
            # exactly this group's parameters: the update runs over the whole buffer, order is irrelevant
            if flat is not None and len(self.param_groups) == 1 and \
                    sorted(id(p) for p in flat.params) == sorted(id(p) for p in ps if p.requires_grad):
                fp = flat
            else:
                fp = FlatParams(ps)
            self._flats.append(fp)
        self._s1: List[Optional[torch.Tensor]] = [None] * len(self._flats)
        self._s2: List[Optional[torch.Tensor]] = [None] * len(self._flats)
        self._steps: List[int] = [0] * len(self._flats)
        self._lr_dev: List[Optional[torch.Tensor]] = [None] * len(self._flats)
        self._lr_dev_val: List[Optional[float]] = [None] * len(self._flats)
        self.grad_scale = 1.0  # applied to incoming gradients (e.g. AMP unscale)
        for gi in range(len(self._flats)):
            self._alloc_state(gi)

    # ------------------------------------------------------------------
    @property
    def flats(self) -> List[FlatParams]:
        return self._flats

    def _needs(self, group) -> tuple:
        s2 = self.kind in (1, 2, 4)
        s1 = s2 or self.kind == 3 or (self.kind == 0 and group.get("momentum", 0.0) != 0.0)
        return s1, s2

    def _alloc_state(self, gi: int) -> None:
        fp = self._flats[gi]
        s1, s2 = self._needs(self.param_groups[gi])
        if s1 and self._s1[gi] is None:
            self._s1[gi] = torch.zeros_like(fp.data)
        if s2 and self._s2[gi] is None:
            self._s2[gi] = torch.zeros_like(fp.data)

    def state_buffers(self, gi: int = 0):
        return self._s1[gi], self._s2[gi]

    def lr_tensor(self, gi: int = 0) -> torch.Tensor:
        """Device scalar holding the group's current lr (kept in sync with group['lr'])."""
        fp = self._flats[gi]
        lr = float(self.param_groups[gi]["lr"])
        if self._lr_dev[gi] is None:
            self._lr_dev[gi] = torch.full((1,), lr, dtype=torch.float32, device=fp.device)
            self._lr_dev_val[gi] = lr
        elif self._lr_dev_val[gi] != lr:
            self._lr_dev[gi].fill_(lr)  # a tiny kernel with lr as an argument: graph/stream safe
            self._lr_dev_val[gi] = lr
        return self._lr_dev[gi]

    def hyper(self, gi: int = 0) -> Dict[str, Any]:
        g = self.param_groups[gi]
        betas = g.get("betas", (0.9, 0.999))
        return dict(kind=self.kind, lr=float(g["lr"]), momentum=float(g.get("momentum", 0.0)),
                    dampening=float(g.get("dampening", 0.0)), weight_decay=float(g.get("weight_decay", 0.0)),
                    beta1=float(betas[0]), beta2=float(betas[1]), eps=float(g.get("eps", 1e-8)),
                    lr_decay=float(g.get("lr_decay", 0.0)), grad_scale=float(self.grad_scale),
                    nesterov=bool(g.get("nesterov", False)), maximize=bool(g.get("maximize", False)))

    # ------------------------------------------------------------------
    def zero_grad(self, set_to_none: bool = False) -> None:  # keep grads as flat views
        for fp in self._flats:
            fp.rebind_grads()
            fp.zero_grad()

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, fp in enumerate(self._flats):
            fp.rebind_params()
            fp.rebind_grads()
            self._alloc_state(gi)
            self._steps[gi] += 1
            h = self.hyper(gi)
            if fp.device.type == "cuda":
                C = require_native()
                shadow = fp.shadow if fp.shadow is not None and fp._shadow_ver == fp.data._version else None
                C.flat_optim(fp.data, fp.grad, self._s1[gi], self._s2[gi], h["kind"], h["lr"], h["momentum"],
                             h["dampening"], h["weight_decay"], h["beta1"], h["beta2"], h["eps"], h["lr_decay"],
                             h["grad_scale"], h["nesterov"], h["maximize"], None, None, None,
                             float(self._steps[gi]), shadow, None)
                if shadow is not None:
                    fp.mark_shadow_fresh()  # the kernel rewrote the bf16 copy of every updated weight
            else:
                _cpu_update(h, float(self._steps[gi]), fp.data, fp.grad, self._s1[gi], self._s2[gi])
            fp.generation += 1  # weights changed: derived copies (fp8 casts) are stale
        return loss

    # ------------------------------------------------------------------
    def state_dict(self) -> Dict[str, Any]:
        groups = []
        for g in self.param_groups:
            groups.append({k: v for k, v in g.items() if k != "params"})
        return {"kind": self.kind_name, "param_groups": groups,
                "flat_state": [{"step": self._steps[i],
                                "s1": self._export(i, self._s1[i]), "s2": self._export(i, self._s2[i])}
                               for i in range(len(self._flats))]}

    def _export(self, i: int, buf: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        if buf is None:
            return None
        fp = self._flats[i]
        # a ZeRO shard (parallel/zero.py) gathers its state into the full flat layout (collective)
        return fp.export_state(buf) if hasattr(fp, "export_state") else buf.detach().cpu()

    def load_state_dict(self, sd: Dict[str, Any]) -> None:
        if sd.get("kind") != self.kind_name:
            raise ValueError(f"optimizer kind mismatch: {sd.get('kind')} vs {self.kind_name}")
        for g, sg in zip(self.param_groups, sd["param_groups"]):
            for k, v in sg.items():
                g[k] = v
        for i, st in enumerate(sd["flat_state"]):
            self._steps[i] = int(st["step"])
            for name, buf in (("s1", self._s1), ("s2", self._s2)):
                if st[name] is not None:
                    if buf[i] is None:
                        buf[i] = torch.zeros_like(self._flats[i].data)
                    if hasattr(self._flats[i], "import_state"):
                        self._flats[i].import_state(st[name], buf[i])
                    else:
                        buf[i].copy_(st[name].to(buf[i].device))
            self._lr_dev_val[i] = None if self._lr_dev[i] is None else -1.0


def _cpu_update(h, t, p, g, s1, s2) -> None:
    """Reference math for CPU flat buffers (mirrors mlt_optim.h)."""
    g = g * h["grad_scale"]
    if h["maximize"]:
        g = -g
    lr, wd, k = h["lr"], h["weight_decay"], h["kind"]
    if k == 0:
        if wd:
            g = g + wd * p
        if h["momentum"]:
            if t <= 1:
                s1.copy_(g)
            else:
                s1.mul_(h["momentum"]).add_(g, alpha=1 - h["dampening"])
            g = g + h["momentum"] * s1 if h["nesterov"] else s1
        p.add_(g, alpha=-lr)
    elif k in (1, 2):
        if k == 2:
            p.mul_(1 - lr * wd)
        elif wd:
            g = g + wd * p
        s1.mul_(h["beta1"]).add_(g, alpha=1 - h["beta1"])
        s2.mul_(h["beta2"]).addcmul_(g, g, value=1 - h["beta2"])
        bc1 = 1 - h["beta1"] ** t
        bc2 = 1 - h["beta2"] ** t
        denom = (s2.sqrt() / math.sqrt(bc2)).add_(h["eps"])
        p.addcdiv_(s1, denom, value=-lr / bc1)
    elif k == 3:
        if wd:
            g = g + wd * p
        clr = lr / (1 + (t - 1) * h["lr_decay"])
        s1.addcmul_(g, g, value=1)
        p.addcdiv_(g, s1.sqrt().add_(h["eps"]), value=-clr)
    elif k == 4:
        if wd:
            g = g + wd * p
        s1.mul_(h["beta1"]).add_(g, alpha=1 - h["beta1"])
        torch.maximum(s2.mul_(h["beta2"]), g.abs().add_(h["eps"]), out=s2)
        p.addcdiv_(s1, s2, value=-lr / (1 - h["beta1"] ** t))


class FusedSGD(FusedOptimizer):
    kind_name = "sgd"

    def __init__(self, params, lr=1e-3, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False,
                 maximize=False, flat=None):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                                      nesterov=nesterov, maximize=maximize), flat)


class FusedAdam(FusedOptimizer):
    kind_name = "adam"

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, maximize=False,
                 flat=None):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, maximize=maximize),
                         flat)


class FusedAdamW(FusedOptimizer):
    kind_name = "adamw"

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, maximize=False,
                 flat=None):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, maximize=maximize),
                         flat)


class FusedAdagrad(FusedOptimizer):
    kind_name = "adagrad"

    def __init__(self, params, lr=1e-2, lr_decay=0.0, weight_decay=0.0, eps=1e-10, maximize=False, flat=None):
        super().__init__(params, dict(lr=lr, lr_decay=lr_decay, weight_decay=weight_decay, eps=eps,
                                      maximize=maximize), flat)


class FusedAdamax(FusedOptimizer):
    kind_name = "adamax"

    def __init__(self, params, lr=2e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, maximize=False,
                 flat=None):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, maximize=maximize),
                         flat)


OPTIMIZERS = {"sgd": FusedSGD, "adam": FusedAdam, "adamw": FusedAdamW, "adagrad": FusedAdagrad,
              "adamax": FusedAdamax}


def build_optimizer(name: str, params, lr: float, momentum: float = 0.9, weight_decay: float = 0.0,
                    flat: Optional[FlatParams] = None) -> Optional[FusedOptimizer]:
    """Factory with the reference's name->optimizer mapping (src/trainer.py:123-138):
    only SGD takes momentum; the others get lr + weight_decay with torch defaults."""
    name = (name or "").lower()
    if name == "sgd":
        return FusedSGD(params, lr=lr, momentum=momentum, weight_decay=weight_decay, flat=flat)
    if name in OPTIMIZERS:
        return OPTIMIZERS[name](params, lr=lr, weight_decay=weight_decay, flat=flat)
    return None


def clip_grad_norm_flat(flat: FlatParams, max_norm: float) -> torch.Tensor:
    """torch.nn.utils.clip_grad_norm_ over a flat gradient buffer: one fused
    sum-of-squares kernel + one scale, no host sync (returns the device norm)."""
    g = flat.grad
    if g.is_cuda:
        C = require_native()
        sq = torch.zeros(1, dtype=torch.float32, device=g.device)
        coef = torch.empty(1, dtype=torch.float32, device=g.device)
        total = torch.empty(1, dtype=torch.float32, device=g.device)
        C.sq_norm(g, sq)
        C.clip_coef(sq, float(max_norm), coef, total)
        g.mul_(coef)
        return total.view(())
    total = g.norm()
    g.mul_(torch.clamp(max_norm / (total + 1e-6), max=1.0))
    return total
