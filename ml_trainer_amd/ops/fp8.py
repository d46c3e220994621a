"""FP8 linear layers for the ``large`` config (BASELINE.json config 5: "large config fp8
(CDNA4 fp8 MFMA)").

Numerics (the standard delayed-scaling recipe, on MI355X's OCP formats):

* forward GEMM  y  = x . W^T  : x e4m3 x W e4m3  (v_mfma_scale_f32_16x16x128_f8f6f4, unit MX
  block scales; per-tensor scales folded into the epilogue alpha from device memory);
* dgrad GEMM    dx = dy . W   : dy e5m2 x W^T e4m3 (W^T from the same cast-transpose pass, so
  both operands are k-contiguous);
* wgrad GEMM    dW = dy^T . x : bf16 (split-K tile kernel), fp32 output into the master grads;
* scales: every quantised tensor role (x, W, dy of each linear) owns a meta slot: the cast
  kernels record amax(|t|) while quantising, and ``Fp8Context.update()`` (once per step, one
  launch for all slots) pushes it into a 16-step history and sets scale = fmax / max(history).
  A slot's very first use computes its exact amax first (current scaling), so step 0 is sane.
* weights are re-quantised (cast + transpose, one pass over the fp32 master) only when the
  optimizer has updated them (``FlatParams.generation``).

Everything else in the block (bias, GELU, residual, LayerNorm, attention) is unchanged bf16.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import torch

from ml_trainer_amd.ops._ext import require_native
from ml_trainer_amd.utils.flat import FlatParams

E4M3, E5M2 = 0, 1
_FMAX = {E4M3: 448.0, E5M2: 57344.0}
_DT = {E4M3: torch.float8_e4m3fn, E5M2: torch.float8_e5m2}


class Fp8Context:
    """Device-resident fp8 scaling state for up to ``capacity`` tensor roles."""

    def __init__(self, device: torch.device, capacity: int = 4096, history: int = 16, margin: int = 0):
        self.device = device
        self.slots = int(require_native().FP8_AMAX_SLOTS)
        self.amax = torch.zeros(capacity, self.slots, device=device)  # per-tensor amax sub-slots
        self.scale = torch.ones(capacity, device=device)
        self.inv_scale = torch.ones(capacity, device=device)
        self.fmax = torch.zeros(capacity, device=device)
        self.hist = torch.zeros(capacity, history, device=device)
        self.margin = margin
        self.n = 0
        self.step = 0
        self._ready: list = []

    def new_meta(self, fmt: int) -> int:
        if self.n >= self.amax.shape[0]:
            raise RuntimeError("fp8 context capacity exhausted")
        i = self.n
        self.fmax[i] = _FMAX[fmt]
        self.n += 1
        self._ready.append(False)
        return i

    def update(self) -> None:
        """Delayed scaling: fold the amaxes recorded since the last call into every slot's scale."""
        if self.n:
            require_native().fp8_update_scale(self.hist[:self.n], self.amax[:self.n], self.scale[:self.n],
                                              self.inv_scale[:self.n], self.fmax[:self.n], self.step, self.margin)
            self.step += 1

    def _init_exact(self, i: int, x: torch.Tensor) -> None:
        C = require_native()
        sl = slice(i, i + 1)
        self.amax[sl].zero_()
        C.fp8_amax(x, self.amax[i])
        C.fp8_update_scale(self.hist[sl], self.amax[sl], self.scale[sl], self.inv_scale[sl], self.fmax[sl],
                           self.step, self.margin)
        self._ready[i] = True

    def cast(self, x: torch.Tensor, i: int, fmt: int) -> torch.Tensor:
        if not self._ready[i]:
            self._init_exact(i, x)
        y = torch.empty(x.shape, dtype=_DT[fmt], device=x.device)
        require_native().fp8_cast(x, y, self.scale[i:i + 1], self.amax[i], fmt)
        return y

    def cast_t(self, x: torch.Tensor, i: int, fmt: int, colsum_out: Optional[torch.Tensor] = None,
               colsum_accumulate: bool = False):
        """fp8 copy of a bf16 [R, C] tensor plus its transpose [C, R] in one pass (same scale);
        ``colsum_out`` (fp32 [C]) also receives the column sums of x from the same read (set or
        accumulated): the bias gradient when x is a linear's dY."""
        if not self._ready[i]:
            self._init_exact(i, x)
        y = torch.empty(x.shape, dtype=_DT[fmt], device=x.device)
        yt = torch.empty(x.shape[1], x.shape[0], dtype=_DT[fmt], device=x.device)
        require_native().fp8_cast_transpose(x, y, yt, self.scale[i:i + 1], self.amax[i], fmt,
                                            colsum_out=colsum_out, colsum_accumulate=colsum_accumulate)
        return y, yt

    def inv(self, i: int) -> torch.Tensor:
        return self.inv_scale[i:i + 1]


_CTX: Dict[torch.device, Fp8Context] = {}


def context(device: torch.device) -> Fp8Context:
    device = torch.device(device)
    if device not in _CTX:
        _CTX[device] = Fp8Context(device)
    return _CTX[device]


class _WeightState:
    __slots__ = ("mx", "mw", "mdy", "w8", "w8t", "key", "xt", "dy8", "dyt")

    def __init__(self, ctx: Fp8Context):
        self.mx = ctx.new_meta(E4M3)
        self.mw = ctx.new_meta(E4M3)
        self.mdy = ctx.new_meta(E5M2)
        self.w8: Optional[torch.Tensor] = None
        self.w8t: Optional[torch.Tensor] = None
        self.key = None
        self.xt = None   # (x.data_ptr(), X^T in e4m3) of the last forward, for the fp8 weight gradient
        self.dy8 = None  # (dy.data_ptr(), dY in e5m2) cast by wgrad, reused by the dgrad that follows
        self.dyt = None  # dY^T in e5m2 written by the producing GEMM's quantising epilogue (FFN1)


def _state(w: torch.Tensor, ctx: Fp8Context) -> _WeightState:
    st = getattr(w, "_mlt_f8", None)
    if st is None:
        st = _WeightState(ctx)
        w._mlt_f8 = st
    return st


def _weight_key(w: torch.Tensor):
    fp = FlatParams.owner(w)
    # generation: optimizer updates; data._version: load_state_dict / manual edits of the masters
    return ((fp.generation, fp.data._version) if fp is not None else w._version, w.data_ptr())


def weight_fp8(w: torch.Tensor, ctx: Fp8Context) -> _WeightState:
    """fp8 W and W^T of an fp32 master weight [out, in], re-quantised when the weight changed."""
    st = _state(w, ctx)
    key = _weight_key(w)
    if st.key != key:
        C = require_native()
        wd = w.detach()
        if st.w8 is None:
            st.w8 = torch.empty(wd.shape, dtype=torch.float8_e4m3fn, device=wd.device)
            st.w8t = torch.empty(wd.shape[1], wd.shape[0], dtype=torch.float8_e4m3fn, device=wd.device)
        if not ctx._ready[st.mw]:
            ctx._init_exact(st.mw, wd)
        C.fp8_cast_transpose(wd, st.w8, st.w8t, ctx.scale[st.mw:st.mw + 1], ctx.amax[st.mw], E4M3)
        st.key = key
    return st


def _fp8_wgrad_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    # the MX-scaled MFMA GEMM needs K (= tokens) % 128 and both output dims >= 64
    return x.shape[0] % 128 == 0 and x.shape[1] >= 64 and w.shape[0] >= 64 and x.shape[1] % 4 == 0


class Fp8Linear:
    """Linear arithmetic for ops.transformer blocks, all three GEMMs in fp8 (delayed scaling):
    forward X(e4m3) . W^T(e4m3), dgrad dY(e5m2) . W(e4m3), wgrad dY^T(e5m2) . X^T(e4m3) -- the
    activations are cast together with their transposes so every operand is k-contiguous.

    ``training``: whether a backward will follow (the block wrappers set it from the caller's
    grad mode, which autograd switches off inside Function.forward); only then are the
    transposed activations produced and kept."""

    training = True
    wgrad_fuses_bias = True  # wgrad(..., db_out=) reduces the bias gradient inside the dY cast

    @staticmethod
    def fwd(x, w, bias=None, gelu_aux=None, res=None):
        C = require_native()
        ctx = context(x.device)
        st = weight_fp8(w, ctx)
        if x.dtype == _DT[E4M3]:
            # quantised by the producer's epilogue with this weight's input scale (fwd_gelu_q),
            # which also left X^T in st.xt
            x8 = x
        elif Fp8Linear.training and _fp8_wgrad_ok(x, w):
            x8, x8t = ctx.cast_t(x, st.mx, E4M3)
            st.xt = (x.data_ptr(), x8t)
        else:
            x8 = ctx.cast(x, st.mx, E4M3)
            st.xt = None
        y = torch.empty(x.shape[0], w.shape[0], dtype=torch.bfloat16, device=x.device)
        C.gemm_f8(x8, st.w8, y, E4M3, E4M3, ctx.inv(st.mx), ctx.inv(st.mw), bias=bias, aux=gelu_aux, res=res,
                  mode=1 if gelu_aux is not None else 0)
        return y

    @staticmethod
    def wgrad(w, dy, x, out: Optional[torch.Tensor], db_out: Optional[torch.Tensor] = None, db_acc: bool = False):
        """dW = dY^T X in fp8 into ``out`` (accumulate) or a new fp32 tensor; None when the forward
        left no transposed input for this weight (the caller then uses the bf16 GEMM, and
        ``db_out`` is untouched). ``db_out``: bias gradient column sums of dY, from the cast."""
        st = getattr(w, "_mlt_f8", None)
        if st is None or st.xt is None or st.xt[0] != x.data_ptr() or not _fp8_wgrad_ok(x, w):
            return None
        C = require_native()
        ctx = context(dy.device)
        if dy.dtype == _DT[E5M2]:
            # dY (+ dY^T, + bias gradient) from the producer's quantising epilogue (dgrad_gelu_q)
            if st.dyt is None or st.dy8 is None or st.dy8[0] != dy.data_ptr():
                raise RuntimeError("fp8 wgrad: pre-quantised dY without its transpose")
            dy8t, st.dyt = st.dyt, None
        elif st.dyt is not None and st.dy8 is not None and st.dy8[0] == dy.data_ptr():
            # bf16 dY whose e5m2 copy and transpose the producing LayerNorm backward already wrote
            # (ln_bwd_q8, which also reduced the bias gradient)
            if db_out is not None:
                raise RuntimeError("fp8 wgrad: LayerNorm-quantised dY carries its bias gradient already")
            dy8t, st.dyt = st.dyt, None
        else:
            dy8, dy8t = ctx.cast_t(dy, st.mdy, E5M2, colsum_out=db_out, colsum_accumulate=db_acc)
            st.dy8 = (dy.data_ptr(), dy8)
        acc = out is not None
        if out is None:
            out = torch.empty(w.shape[0], w.shape[1], dtype=torch.float32, device=dy.device)
        C.gemm_f8(dy8t, st.xt[1], out, E5M2, E4M3, ctx.inv(st.mdy), ctx.inv(st.mx), accumulate=acc)
        st.xt = None
        return out

    @staticmethod
    def dgrad(dy, w, out, aux=None, res=None):
        C = require_native()
        ctx = context(dy.device)
        st = weight_fp8(w, ctx)
        if dy.dtype == _DT[E5M2]:
            dy8 = dy
        elif st.dy8 is not None and st.dy8[0] == dy.data_ptr():
            dy8 = st.dy8[1]
        else:
            dy8 = ctx.cast(dy, st.mdy, E5M2)
        st.dy8 = None
        C.gemm_f8(dy8, st.w8t, out, E5M2, E4M3, ctx.inv(st.mdy), ctx.inv(st.mw), aux=aux,
                  mode=2 if aux is not None else 0, res=res)
        return out


    # ---- attention backward quantises the QKV projection's dY ------------------------------------
    # The dQ and dK/dV kernels write dQKV as e5m2 with its transpose and amax (attn_bwd q8_*), from
    # the bf16-rounded values, bitwise what fp8_cast_transpose of the bf16 dQKV gives: the widest
    # cast of the layer (3 x hidden columns) and the bf16 dQKV itself disappear.
    fuse_attn = os.environ.get("MLT_FP8_ATTN_Q", "1") != "0"

    @staticmethod
    def attn_dy_q(wqkv, x, rows: int):
        """(dqkv8, dqkv8^T, scale, amax) buffers for attn_bwd's q8 outputs when Wqkv's e5m2 dY scale
        exists and the forward left X^T for its fp8 weight gradient; else None."""
        if not Fp8Linear.fuse_attn:
            return None
        st = getattr(wqkv, "_mlt_f8", None)
        if st is None or st.xt is None or st.xt[0] != x.data_ptr() or not _fp8_wgrad_ok(x, wqkv):
            return None
        ctx = context(x.device)
        if not ctx._ready[st.mdy] or rows % 16:
            return None
        n = wqkv.shape[0]
        d8 = torch.empty(rows, n, dtype=_DT[E5M2], device=x.device)
        d8t = torch.empty(n, rows, dtype=_DT[E5M2], device=x.device)
        return d8, d8t, ctx.scale[st.mdy:st.mdy + 1], ctx.amax[st.mdy]

    @staticmethod
    def attn_dy_q_done(wqkv, d8, d8t):
        """Hand the attention backward's e5m2 dY (and transpose) to Wqkv's wgrad / dgrad."""
        st = _state(wqkv, context(d8.device))
        st.dy8 = (d8.data_ptr(), d8)
        st.dyt = d8t

    # ---- LayerNorm backward quantises the out-proj / FFN2 dY ------------------------------------
    # In the post-LN blocks the LayerNorm backward's dx is the dY of the out-projection (attention
    # block) and of FFN2: C.ln_bwd_q8 writes its e5m2 copy and transpose with that weight's dY scale
    # (plus amax, plus the bias gradient it already reduced), so the separate cast-transpose pass
    # over dx disappears. Opt-in (MLT_FP8_LN_Q=1): measured slower -- 508 us per call against 308 us
    # of ln_bwd + 184 us of cast-transpose at 262144 x 1024, fp8 `large` 1,250 vs 1,254 samples/s
    # (profiles/r5/fp8_ln_bwd_q8_ab.jsonl). Its 32-row chunk barriers and the transposed pass leave
    # the loads idle; the two streaming kernels it replaces each run near 5.2-5.8 TB/s.
    fuse_ln = os.environ.get("MLT_FP8_LN_Q", "0") == "1"

    @staticmethod
    def ln_bwd_q_state(w, x):
        """(state, context) when a LayerNorm backward may quantise ``w``'s dY: its e5m2 scale exists
        and the forward left X^T (of ``x``) for w's fp8 weight gradient; else None."""
        if not Fp8Linear.fuse_ln:
            return None
        st = getattr(w, "_mlt_f8", None)
        if st is None or st.xt is None or st.xt[0] != x.data_ptr() or not _fp8_wgrad_ok(x, w):
            return None
        ctx = context(x.device)
        if not ctx._ready[st.mdy]:
            return None
        return st, ctx

    # ---- FFN fusion: the GEMM epilogues quantise for the next GEMM ------------------------------
    # FFN1's forward epilogue writes GELU(.) as FFN2's e4m3 input and its transpose (FFN2's wgrad
    # operand); FFN2's dgrad epilogue writes dGELU(.) as FFN1's e5m2 dY, its transpose and FFN1's
    # bias gradient. The bf16 intermediate [tokens, 4H] and its cast-transpose pass (one read +
    # two writes of the widest activation of the layer, twice per step) disappear.
    fuse_q = os.environ.get("MLT_FP8_FUSE", "1") != "0"

    @staticmethod
    def _q_shape_ok(x, w1) -> bool:
        return (x.shape[0] % 256 == 0 and w1.shape[0] % 256 == 0 and x.shape[1] % 128 == 0
                and _fp8_wgrad_ok(x, w1))

    @staticmethod
    def fwd_gelu_q(x, w1, b1, pre, w2):
        """a = GELU(x . W1^T + b1) quantised with W2's input scale: returns e4m3 ``a`` [M, F]
        (pre-activation saved in ``pre``; a^T kept for W2's wgrad), or None when not applicable
        (inference, shapes, or W2's input scale not initialised yet -- the first step)."""
        if not (Fp8Linear.fuse_q and Fp8Linear.training and Fp8Linear._q_shape_ok(x, w1)):
            return None
        C = require_native()
        ctx = context(x.device)
        st2 = _state(w2, ctx)
        if not ctx._ready[st2.mx]:
            return None
        st1 = weight_fp8(w1, ctx)
        x8, x8t = ctx.cast_t(x, st1.mx, E4M3)
        st1.xt = (x.data_ptr(), x8t)
        M, F = x.shape[0], w1.shape[0]
        a8 = torch.empty(M, F, dtype=_DT[E4M3], device=x.device)
        a8t = torch.empty(F, M, dtype=_DT[E4M3], device=x.device)
        C.gemm_f8_q(x8, st1.w8, a8, a8t, E4M3, E4M3, ctx.inv(st1.mx), ctx.inv(st1.mw), E4M3,
                    ctx.scale[st2.mx:st2.mx + 1], ctx.amax[st2.mx], bias=b1, aux=pre, mode=1)
        st2.xt = (a8.data_ptr(), a8t)
        return a8

    @staticmethod
    def dgrad_gelu_q_ready(w1, x) -> bool:
        """Whether dgrad_gelu_q can produce W1's dY: its e5m2 scale exists and the forward left
        X^T for W1's fp8 wgrad."""
        st1 = getattr(w1, "_mlt_f8", None)
        return (st1 is not None and context(x.device)._ready[st1.mdy] and st1.xt is not None
                and st1.xt[0] == x.data_ptr())

    @staticmethod
    def dgrad_gelu_q(dy, w2, pre, w1, db_out, db_acc: bool):
        """dpre = (dy . W2) * gelu'(pre) quantised with W1's dY scale: returns e5m2 dpre [M, F];
        dpre^T is left for W1's wgrad, sum over rows of dpre goes to ``db_out`` (set or
        accumulated). Call only when dgrad_gelu_q_ready(w1, x)."""
        C = require_native()
        ctx = context(dy.device)
        st2 = weight_fp8(w2, ctx)
        st1 = _state(w1, ctx)
        if st2.dy8 is not None and st2.dy8[0] == dy.data_ptr():
            dy8 = st2.dy8[1]
        else:
            dy8 = ctx.cast(dy, st2.mdy, E5M2)
        st2.dy8 = None
        M, F = dy.shape[0], w2.shape[1]
        d8 = torch.empty(M, F, dtype=_DT[E5M2], device=dy.device)
        d8t = torch.empty(F, M, dtype=_DT[E5M2], device=dy.device)
        C.gemm_f8_q(dy8, st2.w8t, d8, d8t, E5M2, E4M3, ctx.inv(st2.mdy), ctx.inv(st2.mw), E5M2,
                    ctx.scale[st1.mdy:st1.mdy + 1], ctx.amax[st1.mdy], aux=pre, mode=2,
                    colsum_out=db_out, colsum_accumulate=db_acc)
        st1.dy8 = (d8.data_ptr(), d8)
        st1.dyt = d8t
        return d8


FP8 = Fp8Linear()
