"""Contiguous flat parameter / gradient storage.

Every trainable parameter of a model becomes a *view* into one fp32 buffer and
its ``.grad`` a view into a matching gradient buffer. Consequences:

* an optimizer step is one fused HIP launch over the whole buffer
  (``ops/optim.py``) instead of ~3 launches per tensor (reference SGD step:
  ``mul_`` x10 + ``add_`` x20, SURVEY.md App. A census);
* DDP buckets are contiguous slices of the gradient buffer, so the all-reduce
  needs no copy-in/copy-out (``parallel/ddp.py``);
* checkpointing the state is a single D2H copy.

Segments start at multiples of ``align`` elements (default 16: 64 B of fp32, 32 B of the
bf16 shadow) so kernels can use 16-byte vector accesses on any parameter and on its bf16
shadow view (the bf16 GEMM / embedding kernels require 16-byte aligned operands).
"""
from __future__ import annotations

import weakref
from typing import Dict, Iterable, List, Optional, Tuple

import torch

# parameter id -> FlatParams that owns it (lets ops find a param's bf16 shadow view)
_OWNER: "weakref.WeakValueDictionary[int, FlatParams]" = weakref.WeakValueDictionary()


def _round_up(x: int, a: int) -> int:
    return (x + a - 1) // a * a


class FlatParams:
    def __init__(self, params: Iterable[torch.nn.Parameter], device: Optional[torch.device] = None,
                 align: int = 16, reverse: bool = False, dtype: torch.dtype = torch.float32):
        ps = [p for p in params if p.requires_grad]
        if reverse:
            ps = ps[::-1]
        self.params: List[torch.nn.Parameter] = ps
        dev = device or (ps[0].device if ps else torch.device("cpu"))
        self.device = torch.device(dev)
        self.offsets: List[int] = []
        off = 0
        for p in ps:
            self.offsets.append(off)
            off += _round_up(p.numel(), align)
        self.numel = max(_round_up(off, align), align)
        self.data = torch.zeros(self.numel, dtype=dtype, device=self.device)
        self.grad = torch.zeros(self.numel, dtype=dtype, device=self.device)
        self._index: Dict[int, int] = {}
        with torch.no_grad():
            for i, (p, o) in enumerate(zip(ps, self.offsets)):
                n = p.numel()
                self.data[o:o + n].copy_(p.detach().reshape(-1).to(self.device, dtype))
                p.data = self.data[o:o + n].view_as(p)
                p.grad = self.grad[o:o + n].view_as(p)
                self._index[id(p)] = i
                _OWNER[id(p)] = self
        self.shadow: Optional[torch.Tensor] = None  # bf16 copy of `data` for mixed-precision compute
        self._shadow_ver = -1
        self.generation = 0  # bumped by every optimizer update (keys caches of derived weight copies)
        self.grad_ready_hooks: List = []  # called as hook(p) when a fused kernel wrote p's gradient

    # ------------------------------------------------------------------
    def segment(self, p: torch.nn.Parameter) -> Tuple[int, int]:
        i = self._index[id(p)]
        return self.offsets[i], self.params[i].numel()

    def grad_view(self, i: int) -> torch.Tensor:
        p, o = self.params[i], self.offsets[i]
        return self.grad[o:o + p.numel()].view_as(p)

    def rebind_grads(self) -> None:
        """Re-attach ``p.grad`` to the flat buffer if user code replaced it
        (e.g. ``module.zero_grad(set_to_none=True)``)."""
        gp = self.grad.data_ptr()
        for i, p in enumerate(self.params):
            g = p.grad
            o = self.offsets[i]
            if g is not None and g.data_ptr() == gp + o * self.grad.element_size():
                continue
            view = self.grad_view(i)
            with torch.no_grad():
                if g is None:
                    view.zero_()
                else:
                    view.copy_(g)
            p.grad = view

    def rebind_params(self) -> bool:
        """Re-attach ``p.data`` views if something (e.g. ``module.to()``) replaced
        them; copies the current values back in. Returns True when anything moved."""
        moved = False
        dp = self.data.data_ptr()
        for i, p in enumerate(self.params):
            o = self.offsets[i]
            if p.data.data_ptr() == dp + o * self.data.element_size() and p.device == self.device:
                continue
            with torch.no_grad():
                self.data[o:o + p.numel()].copy_(p.detach().reshape(-1).to(self.device, self.data.dtype))
            p.data = self.data[o:o + p.numel()].view_as(p)
            moved = True
        if moved:
            self.rebind_grads()
        return moved

    def zero_grad(self) -> None:
        self.grad.zero_()

    # ------------------------------------------------------------------ direct gradient writes
    def grad_sink(self, p: torch.Tensor) -> Optional[torch.Tensor]:
        """``p.grad`` when it is this buffer's view of p (a fused backward may then accumulate
        into it in place), else None."""
        i = self._index.get(id(p))
        g = p.grad
        if i is None or g is None:
            return None
        if g.data_ptr() != self.grad.data_ptr() + self.offsets[i] * self.grad.element_size():
            return None
        return g

    def notify_grad_ready(self, p: torch.Tensor) -> None:
        for h in self.grad_ready_hooks:
            h(p)

    # ------------------------------------------------------------------ bf16 shadow
    @staticmethod
    def owner(p: torch.Tensor) -> Optional["FlatParams"]:
        fp = _OWNER.get(id(p))
        if fp is not None and id(p) in fp._index:
            return fp
        return None

    def refresh_shadow(self) -> torch.Tensor:
        """(Re)build the bf16 shadow when the fp32 master changed outside the fused optimizer
        (load_state_dict, manual edits bump the tensor version counter; the optimizer kernel
        writes the shadow itself and leaves the counter alone)."""
        if self.shadow is None:
            self.shadow = torch.empty(self.numel, dtype=torch.bfloat16, device=self.device)
            self._shadow_ver = -1
        if self._shadow_ver != self.data._version:
            if self.device.type == "cuda":
                from ml_trainer_amd.ops._ext import require_native
                require_native().cast_bf16(self.data, self.shadow)
            else:
                self.shadow.copy_(self.data)
            self._shadow_ver = self.data._version
        return self.shadow

    def shadow_view(self, p: torch.Tensor) -> torch.Tensor:
        sh = self.refresh_shadow()
        o, n = self.segment(p)
        return sh[o:o + n].view(p.shape)

    def mark_shadow_fresh(self) -> None:
        self._shadow_ver = self.data._version

    def state_dict_views(self) -> List[torch.Tensor]:
        return [self.data[o:o + p.numel()].view_as(p) for p, o in zip(self.params, self.offsets)]


_DIGEST_PRIMES = ((2 ** 31 - 1, 0x5BD1E995, 0x27D4EB2F), (2 ** 31 - 19, 0x9E3779B1, 0x165667B1))


@torch.no_grad()
def bitwise_digest(t: torch.Tensor, chunk: int = 1 << 24) -> Tuple[int, int]:
    """Order- and bit-sensitive digest of a tensor's raw 32-bit words (SURVEY.md §5.2's cross-rank
    parameter hash), computed on the tensor's own device: for each of two primes p,
    ``sum_i (u_i + 1) * r_i mod p`` with u_i the i-th word as an unsigned 32-bit integer and
    r_i = (A i + C) mod p distinct for every index. Flipping any bit of any word, or swapping two
    different words, changes each digest (the difference is (u_i - u_j) * A * (j - i) != 0 mod p),
    where a floating-point sum can miss both. Fixed order, integer arithmetic: bitwise
    reproducible. Returns two integers < 2^31."""
    flat = t.detach().reshape(-1)
    if flat.element_size() != 4:
        flat = flat.contiguous().view(torch.uint8)
        pad = (-flat.numel()) % 4
        if pad:
            flat = torch.cat([flat, flat.new_zeros(pad)])
    words = flat.contiguous().view(torch.int32)
    out = []
    for p, a, c in _DIGEST_PRIMES:
        acc = 0
        for s in range(0, words.numel(), chunk):
            u = words[s:s + chunk].to(torch.int64) & 0xFFFFFFFF
            idx = torch.arange(s, s + u.numel(), dtype=torch.int64, device=u.device)
            r = (idx % p * a + c) % p                      # < 2^31
            acc = (acc + int((((u % p) + 1) * r % p).sum().item())) % p  # products < 2^62, sums < 2^55
        out.append(acc)
    return out[0], out[1]
