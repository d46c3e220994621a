"""Autograd blocks of the transformer path over the native gfx950 kernels.

Mixed precision: parameters are fp32 masters (in a FlatParams buffer when an
optimizer/DDP owns them); compute reads their bf16 *shadow* (refreshed by the
fused optimizer kernel in the same pass that updates the master, so there is
no separate cast per step). Weight / bias gradients come back in fp32.

Blocks (one autograd node each, so the backward can fuse across ops):

* ``attention_block``: x -> QKV GEMM(+bias) -> fused flash attention -> out-proj
  GEMM (+bias +residual x). Backward: wgrad/colsum/dgrad of out-proj, attention
  backward into the packed dQKV, wgrad/colsum of QKV and dgrad with the residual
  gradient folded into the GEMM epilogue.
* ``ffn_block``: x -> FFN1 GEMM (+bias, GELU epilogue that also stores the
  pre-activation) -> FFN2 GEMM (+bias +residual). Backward: FFN2's dgrad GEMM
  applies gelu'(pre) in its epilogue (no separate elementwise pass).
* ``attention_ln_block`` / ``ffn_ln_block``: the block followed by its post-LayerNorm as one
  node; the LayerNorm backward kernel also produces the column sums of its dx, which are the
  bias gradient of the block's last linear layer (no separate pass over dy).
* ``layer_norm``, ``embeddings``.

The linear-layer arithmetic is pluggable (``impl``): ``BF16`` (bf16 operands) or
``ops.fp8.FP8`` (OCP fp8 forward / dgrad GEMMs with delayed per-tensor scaling; wgrad bf16).

Linear layout conventions (nn.Linear weight [out, in]):
  fwd   y  = x . W^T         gemm(x, W, a_mn=0, b_mn=0)
  dgrad dx = dy . W          gemm(dy, W, a_mn=0, b_mn=1)
  wgrad dW = dy^T . x        gemm(dy, x, a_mn=1, b_mn=1) -> fp32
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from ml_trainer_amd.ops._ext import require_native
from ml_trainer_amd.utils.flat import FlatParams


def bf16_weight(p: torch.Tensor) -> torch.Tensor:
    """bf16 compute copy of an fp32 master parameter."""
    fp = FlatParams.owner(p)
    if fp is not None and fp.device.type == "cuda":
        return fp.shadow_view(p)
    cache = getattr(p, "_mlt_bf16", None)
    if cache is not None and cache[0] == p._version and cache[1] == p.data_ptr():
        return cache[2]
    w = p.detach().to(torch.bfloat16).contiguous()
    p._mlt_bf16 = (p._version, p.data_ptr(), w)
    return w


def bf16_weight_t(p: torch.Tensor) -> torch.Tensor:
    """W^T (bf16, contiguous [in, out]) of a weight [out, in], re-made once per optimizer update
    (FlatParams.generation) -- the k-contiguous B operand of the input-gradient GEMM."""
    fp = FlatParams.owner(p)
    # generation: optimizer updates; data._version: load_state_dict / manual edits of the masters
    key = ((fp.generation, fp.data._version) if fp is not None else p._version, p.data_ptr())
    cache = getattr(p, "_mlt_bf16_t", None)
    if cache is not None and cache[0] == key:
        return cache[1]
    w16 = bf16_weight(p)
    t = cache[1] if cache is not None else torch.empty(w16.shape[1], w16.shape[0], dtype=torch.bfloat16,
                                                        device=w16.device)
    require_native().transpose_bf16(w16, t)
    p._mlt_bf16_t = (key, t)
    return t


class Bf16Linear:
    """bf16 operands (bf16 shadows of the fp32 masters), fp32 accumulate, fused epilogues."""

    @staticmethod
    def fwd(x, w, bias=None, gelu_aux=None, res=None):
        return linear_fwd(x, bf16_weight(w), bias, gelu_aux=gelu_aux, res=res)

    fuse_colsum = os.environ.get("MLT_DGELU_COLSUM", "1") != "0"

    @staticmethod
    def dgrad(dy, w, out, aux=None, res=None, colsum_out=None, colsum_acc=False):
        """out = dy . W  (* gelu'(aux) when aux is given) (+ res). Large token counts take W^T as
        a k-contiguous copy (one transpose per weight per step): the forward-layout tile runs
        8-11 % faster than the n-contiguous-B one on the BERT dgrad shapes. ``colsum_out``: the
        column sums of the dGELU output (the bias gradient of the layer before the GELU) from the
        GEMM epilogue (set or accumulated; see dgelu_colsum_ok)."""
        C = require_native()
        mode = 2 if aux is not None else 0
        if dy.shape[0] >= 4096 and os.environ.get("MLT_DGRAD_WT", "1") != "0":
            C.gemm(dy, bf16_weight_t(w), out, False, False, aux=aux, mode=mode, res=res,
                   colsum_out=colsum_out, colsum_accumulate=colsum_acc)
        else:
            C.gemm(dy, bf16_weight(w), out, False, True, aux=aux, mode=mode, res=res,
                   colsum_out=colsum_out, colsum_accumulate=colsum_acc)
        return out

    @staticmethod
    def dgelu_colsum_ok(dy, w) -> bool:
        """Whether dgrad(dy, w, aux=..., colsum_out=...) can fuse the column sums (ping-pong tiles
        over the whole output: tokens and W's input width multiples of 256)."""
        return Bf16Linear.fuse_colsum and dy.shape[0] % 256 == 0 and w.shape[1] % 256 == 0 and dy.shape[1] % 64 == 0


BF16 = Bf16Linear()


def linear_fwd(x, w16, bias=None, gelu_aux=None, res=None):
    C = require_native()
    y = torch.empty(x.shape[0], w16.shape[0], dtype=torch.bfloat16, device=x.device)
    C.gemm(x, w16, y, False, False, bias=bias, aux=gelu_aux, res=res, mode=1 if gelu_aux is not None else 0)
    return y


def linear_wgrad(dy, x):
    C = require_native()
    dw = torch.empty(dy.shape[1], x.shape[1], dtype=torch.float32, device=dy.device)
    C.gemm(dy, x, dw, True, True)
    return dw


def colsum(dy):
    C = require_native()
    db = torch.empty(dy.shape[1], dtype=torch.float32, device=dy.device)
    C.colsum(dy, db, False)
    return db


class _Grads:
    """Weight / bias gradients of one fused backward.

    When a parameter's ``.grad`` is a view into a FlatParams gradient buffer (fused optimizer /
    native DDP), the producing kernel accumulates straight into it (GEMM ``accumulate`` epilogue,
    reduction ``accmask``, embedding atomics): no fp32 temporary, no AccumulateGrad add kernel,
    and the autograd return value for that parameter is None. The owner is then told the
    gradient is ready (``FlatParams.notify_grad_ready``) so DDP bucket countdowns still fire.
    Parameters without a flat gradient get ordinary returned tensors."""

    def __init__(self):
        self.ready = []

    def sink(self, p):
        fp = FlatParams.owner(p)
        g = fp.grad_sink(p) if fp is not None else None
        if g is not None:
            self.ready.append(p)
        return g

    def wgrad(self, p, dy, x, impl=None):
        g = self.sink(p)
        if impl is not None and hasattr(impl, "wgrad"):  # fp8 weight gradient
            r = impl.wgrad(p, dy, x, g)
            if r is not None:
                return None if g is not None else r
        if g is None:
            return linear_wgrad(dy, x)
        require_native().gemm(dy, x, g, True, True, accumulate=True)
        return None

    def wgrad_bias(self, pw, pb, dy, x, impl=None):
        """(dW, db) of one linear. With an fp8 ``impl`` the bias gradient is reduced inside the
        dY cast the fp8 weight gradient needs anyway (one read of dY instead of two)."""
        if pb is None or impl is None or not getattr(impl, "wgrad_fuses_bias", False):
            return self.wgrad(pw, dy, x, impl), self.colsum(pb, dy)
        C = require_native()
        g, gb = self.sink(pw), self.sink(pb)
        db = gb if gb is not None else torch.empty(dy.shape[1], dtype=torch.float32, device=dy.device)
        r = impl.wgrad(pw, dy, x, g, db_out=db, db_acc=gb is not None)
        if r is not None:
            return (None if g is not None else r), (None if gb is not None else db)
        # fp8 weight gradient not applicable here: separate kernels into the same sinks
        if g is None:
            dw = linear_wgrad(dy, x)
        else:
            C.gemm(dy, x, g, True, True, accumulate=True)
            dw = None
        if gb is None:
            C.colsum(dy, db, False)
            return dw, db
        C.colsum(dy, gb, accumulate=True)
        return dw, None

    def colsum(self, p, dy):
        g = self.sink(p)
        if g is None:
            return colsum(dy)
        require_native().colsum(dy, g, accumulate=True)
        return None

    def done(self):
        for p in self.ready:
            FlatParams.owner(p).notify_grad_ready(p)
        self.ready = []


def _attn_fwd(x, wqkv, bqkv, wo, bo, lens, B, S, H, impl=BF16):
    C = require_native()
    qkv = impl.fwd(x, wqkv, bqkv)
    attn = torch.empty(B * S, H * 64, dtype=torch.bfloat16, device=x.device)
    lse = torch.empty(B * H * S, dtype=torch.float32, device=x.device)
    C.attn_fwd(qkv, attn, lse, lens, B, S, H, _ATTN_SCALE)
    y = impl.fwd(attn, wo, bo, res=x)  # out-proj + bias + residual
    return y, (x, qkv, attn, lse)


def _attn_bwd(saved, params, lens, B, S, H, dy, G, dbo="colsum", impl=BF16):
    """Backward of the attention block. ``dbo``: "colsum" to reduce dy here, otherwise the
    out-proj bias gradient already produced by the LayerNorm backward (tensor or None)."""
    C = require_native()
    x, qkv, attn, lse = saved
    wqkv, bqkv, wo, bo = params
    dwo = G.wgrad(wo, dy, attn, impl)
    if isinstance(dbo, str):
        dbo = G.colsum(bo, dy)
    dattn = impl.dgrad(dy, wo, torch.empty_like(attn))
    dqkv = torch.empty_like(qkv)
    delta = torch.empty(B * S * H, dtype=torch.float32, device=dy.device)
    q8 = impl.attn_dy_q(wqkv, x, qkv.shape[0]) if (impl is not BF16 and hasattr(impl, "attn_dy_q")) else None
    if q8 is not None:
        # fp8: the backward kernels write dQKV as e5m2 + transpose + amax (no bf16 dQKV, no cast
        # pass) and the QKV bias gradient as their column sums
        d8, d8t, qs, qa = q8
        db = None
        if bqkv is not None:
            gb = G.sink(bqkv)
            db = gb if gb is not None else torch.empty(qkv.shape[1], dtype=torch.float32, device=dy.device)
        C.attn_bwd(qkv, attn, dattn, lse, delta, lens, dqkv, B, S, H, _ATTN_SCALE, colsum_out=db,
                   colsum_accumulate=bqkv is not None and gb is not None, q8_y=d8, q8_yt=d8t, q8_scale=qs,
                   q8_amax=qa)
        impl.attn_dy_q_done(wqkv, d8, d8t)
        dwqkv = G.wgrad(wqkv, d8, x, impl)
        dbqkv = None if (bqkv is None or gb is not None) else db
        dx = impl.dgrad(d8, wqkv, torch.empty_like(x), res=dy)  # dx = dqkv . Wqkv + dy (residual)
        return dx, dwqkv, dbqkv, dwo, dbo
    if impl is BF16 and bqkv is not None and _ATTN_COLSUM:
        # the QKV bias gradient (column sums of dQKV) from the backward kernels themselves
        gb = G.sink(bqkv)
        dbqkv = gb if gb is not None else torch.empty(qkv.shape[1], dtype=torch.float32, device=dy.device)
        C.attn_bwd(qkv, attn, dattn, lse, delta, lens, dqkv, B, S, H, _ATTN_SCALE, colsum_out=dbqkv,
                   colsum_accumulate=gb is not None)
        dwqkv = G.wgrad(wqkv, dqkv, x, impl)
        dbqkv = None if gb is not None else dbqkv
    else:
        C.attn_bwd(qkv, attn, dattn, lse, delta, lens, dqkv, B, S, H, _ATTN_SCALE)
        dwqkv, dbqkv = G.wgrad_bias(wqkv, bqkv, dqkv, x, impl)
    dx = impl.dgrad(dqkv, wqkv, torch.empty_like(x), res=dy)  # dx = dqkv . Wqkv + dy (residual)
    return dx, dwqkv, dbqkv, dwo, dbo


def _ffn_fwd(x, w1, b1, w2, b2, impl=BF16):
    pre = torch.empty(x.shape[0], w1.shape[0], dtype=torch.bfloat16, device=x.device)
    # fp8: FFN1's epilogue may emit FFN2's quantised input directly (Fp8Linear.fwd_gelu_q)
    a = impl.fwd_gelu_q(x, w1, b1, pre, w2) if hasattr(impl, "fwd_gelu_q") else None
    if a is None:
        a = impl.fwd(x, w1, b1, gelu_aux=pre)  # a = gelu(pre), pre saved
    y = impl.fwd(a, w2, b2, res=x)
    return y, (x, pre, a)


def _ffn_bwd(saved, params, dy, G, db2="colsum", impl=BF16):
    x, pre, a = saved
    w1, b1, w2, b2 = params
    dw2 = G.wgrad(w2, dy, a, impl)
    if isinstance(db2, str):
        db2 = G.colsum(b2, dy)
    if a.dtype == torch.float8_e4m3fn and impl.dgrad_gelu_q_ready(w1, x):
        # fp8 FFN fusion: FFN2's dgrad epilogue emits FFN1's e5m2 dY, dY^T and bias gradient
        gb = G.sink(b1)
        db1 = gb if gb is not None else torch.empty(w1.shape[0], dtype=torch.float32, device=dy.device)
        d8 = impl.dgrad_gelu_q(dy, w2, pre, w1, db1, gb is not None)
        dw1 = G.wgrad(w1, d8, x, impl)
        dx = impl.dgrad(d8, w1, torch.empty_like(x), res=dy)
        return dx, dw1, (None if gb is not None else db1), dw2, db2
    if impl is BF16 and impl.dgelu_colsum_ok(dy, w2):
        # FFN1's bias gradient from the dGELU epilogue (no separate pass over dpre)
        gb = G.sink(b1)
        db1 = gb if gb is not None else torch.empty(w1.shape[0], dtype=torch.float32, device=dy.device)
        dpre = impl.dgrad(dy, w2, torch.empty_like(pre), aux=pre, colsum_out=db1, colsum_acc=gb is not None)
        dw1 = G.wgrad(w1, dpre, x, impl)
        dx = impl.dgrad(dpre, w1, torch.empty_like(x), res=dy)
        return dx, dw1, (None if gb is not None else db1), dw2, db2
    dpre = impl.dgrad(dy, w2, torch.empty_like(pre), aux=pre)  # (dy . W2) * gelu'(pre)
    dw1, db1 = G.wgrad_bias(w1, b1, dpre, x, impl)
    dx = impl.dgrad(dpre, w1, torch.empty_like(x), res=dy)
    return dx, dw1, db1, dw2, db2


def _ln_fwd(x, gamma, beta, eps):
    C = require_native()
    rows = x.shape[0]
    y = torch.empty_like(x)
    mean = torch.empty(rows, dtype=torch.float32, device=x.device)
    rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
    C.ln_fwd(x, gamma, beta, y, mean, rstd, eps)
    return y, (x, gamma, mean, rstd)


def _ln_bwd(saved, beta, dy, G, dxsum_param=None, q8=None):
    """LayerNorm backward; with ``dxsum_param`` also the column sums of dx (= that bias's grad).
    ``q8`` = (impl, w, x): dx is the dY of linear ``w`` (input ``x``); an fp8 ``impl`` that can take
    it pre-quantised gets dx's e5m2 copy and transpose from this same kernel (C.ln_bwd_q8).
    Returns (dx, dgamma|None, dbeta|None, dbias|None)."""
    C = require_native()
    x, gamma, mean, rstd = saved
    D = gamma.numel()
    dev = x.device
    dx = torch.empty_like(x)
    want = dxsum_param is not None
    part = torch.empty(C.ln_partial_blocks(x.shape[0]) * (3 if want else 2) * D, dtype=torch.float32, device=dev)
    sg = FlatParams.owner(gamma)
    sg = sg.grad_sink(gamma) if sg is not None else None
    sb = FlatParams.owner(beta)
    sb = sb.grad_sink(beta) if sb is not None else None
    acc = sg is not None and sb is not None
    if acc:
        G.ready += [gamma, beta]
        dg = db = None
        dg_t, db_t = sg, sb
    else:
        dg = dg_t = torch.empty(D, dtype=torch.float32, device=dev)
        db = db_t = torch.empty(D, dtype=torch.float32, device=dev)
    dxs = dxs_t = None
    dxs_acc = False
    if want:
        so = G.sink(dxsum_param)
        if so is not None:
            dxs_t, dxs_acc = so, True
        else:
            dxs = dxs_t = torch.empty(D, dtype=torch.float32, device=dev)
    if want and q8 is not None and hasattr(q8[0], "ln_bwd_q_state"):
        r = q8[0].ln_bwd_q_state(q8[1], q8[2])
        if r is not None:
            st, fctx = r
            rows = x.shape[0]
            nq = C.ln_q8_partial_blocks(rows) * 3 * D
            if part.numel() < nq:
                part = torch.empty(nq, dtype=torch.float32, device=dev)
            y8 = torch.empty(rows, D, dtype=torch.float8_e5m2, device=dev)
            yt8 = torch.empty(D, rows, dtype=torch.float8_e5m2, device=dev)
            if C.ln_bwd_q8(dy, x, gamma, mean, rstd, dx, part, dg_t, db_t, acc, dxs_t, dxs_acc, y8, yt8,
                           fctx.scale[st.mdy:st.mdy + 1], fctx.amax[st.mdy]):
                st.dy8 = (dx.data_ptr(), y8)
                st.dyt = yt8
                return dx, dg, db, dxs
    C.ln_bwd(dy, x, gamma, mean, rstd, dx, part, dg_t, db_t, acc, None, dxsum=dxs_t, dxsum_acc=dxs_acc)
    return dx, dg, db, dxs


_ATTN_SCALE = 1.0 / 8.0  # 1/sqrt(head_dim = 64)
_ATTN_COLSUM = os.environ.get("MLT_ATTN_COLSUM", "1") != "0"  # QKV bias grad from the attention backward


class _AttentionBlock(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, wqkv, bqkv, wo, bo, lens, B, S, H, impl):
        y, saved = _attn_fwd(x, wqkv, bqkv, wo, bo, lens, B, S, H, impl)
        ctx.save_for_backward(*saved)
        ctx.params, ctx.impl = (wqkv, bqkv, wo, bo), impl
        ctx.lens, ctx.dims = lens, (B, S, H)
        return y

    @staticmethod
    def backward(ctx, dy):
        G = _Grads()
        grads = _attn_bwd(ctx.saved_tensors, ctx.params, ctx.lens, *ctx.dims, dy.contiguous().to(torch.bfloat16), G,
                          impl=ctx.impl)
        G.done()
        return grads + (None, None, None, None, None)


class _FFNBlock(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, impl):
        y, saved = _ffn_fwd(x, w1, b1, w2, b2, impl)
        ctx.save_for_backward(*saved)
        ctx.params, ctx.impl = (w1, b1, w2, b2), impl
        return y

    @staticmethod
    def backward(ctx, dy):
        G = _Grads()
        grads = _ffn_bwd(ctx.saved_tensors, ctx.params, dy.contiguous().to(torch.bfloat16), G, impl=ctx.impl)
        G.done()
        return grads + (None,)


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, eps):
        y, saved = _ln_fwd(x, gamma, beta, eps)
        ctx.save_for_backward(*saved)
        ctx.beta = beta
        return y

    @staticmethod
    def backward(ctx, dy):
        G = _Grads()
        dx, dg, db, _ = _ln_bwd(ctx.saved_tensors, ctx.beta, dy.contiguous().to(torch.bfloat16), G)
        G.done()
        return dx, dg, db, None


class _AttentionLNBlock(torch.autograd.Function):
    """LN(attention_block(x)) as one node: the LayerNorm backward also emits the out-proj bias
    gradient (column sums of its dx), so no separate pass over dy."""

    @staticmethod
    def forward(ctx, x, wqkv, bqkv, wo, bo, gamma, beta, lens, B, S, H, eps, impl):
        a, s1 = _attn_fwd(x, wqkv, bqkv, wo, bo, lens, B, S, H, impl)
        y, s2 = _ln_fwd(a, gamma, beta, eps)
        ctx.save_for_backward(*s1, *s2)
        ctx.params, ctx.beta, ctx.impl = (wqkv, bqkv, wo, bo), beta, impl
        ctx.lens, ctx.dims = lens, (B, S, H)
        return y

    @staticmethod
    def backward(ctx, dy):
        t = ctx.saved_tensors
        G = _Grads()
        da, dg, db, dbo = _ln_bwd(t[4:], ctx.beta, dy.contiguous().to(torch.bfloat16), G, dxsum_param=ctx.params[3],
                                  q8=(ctx.impl, ctx.params[2], t[2]))  # da = out-proj dY (input attn)
        dx, dwqkv, dbqkv, dwo, dbo = _attn_bwd(t[:4], ctx.params, ctx.lens, *ctx.dims, da, G, dbo=dbo,
                                               impl=ctx.impl)
        G.done()
        return dx, dwqkv, dbqkv, dwo, dbo, dg, db, None, None, None, None, None, None


class _FFNLNBlock(torch.autograd.Function):
    """LN(ffn_block(x)) as one node (FFN2 bias gradient fused into the LayerNorm backward)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, gamma, beta, eps, impl):
        f, s1 = _ffn_fwd(x, w1, b1, w2, b2, impl)
        y, s2 = _ln_fwd(f, gamma, beta, eps)
        ctx.save_for_backward(*s1, *s2)
        ctx.params, ctx.beta, ctx.impl = (w1, b1, w2, b2), beta, impl
        return y

    @staticmethod
    def backward(ctx, dy):
        t = ctx.saved_tensors
        G = _Grads()
        df, dg, db, db2 = _ln_bwd(t[3:], ctx.beta, dy.contiguous().to(torch.bfloat16), G, dxsum_param=ctx.params[3],
                                  q8=(ctx.impl, ctx.params[2], t[2]))  # df = FFN2 dY (input a)
        dx, dw1, db1, dw2, db2 = _ffn_bwd(t[:3], ctx.params, df, G, db2=db2, impl=ctx.impl)
        G.done()
        return dx, dw1, db1, dw2, db2, dg, db, None, None


class _Embeddings(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, tt, ww, wp, wt, S):
        C = require_native()
        ids = ids.contiguous().view(-1).to(torch.int64)
        ttf = tt.contiguous().view(-1).to(torch.int64) if tt is not None else None
        D = ww.shape[1]
        out = torch.empty(ids.numel(), D, dtype=torch.bfloat16, device=ids.device)
        C.embed_fwd(ids, ttf, bf16_weight(ww), bf16_weight(wp), bf16_weight(wt), out, S)
        ctx.save_for_backward(ids, ttf if ttf is not None else torch.empty(0, dtype=torch.int64))
        ctx.meta = (tt is not None, S, ww.shape, wp.shape, wt.shape)
        ctx.tables = (ww, wp, wt)
        return out

    @staticmethod
    def backward(ctx, dout):
        C = require_native()
        ids, ttf = ctx.saved_tensors
        has_tt, S, sw, sp, st = ctx.meta
        dout = dout.contiguous().to(torch.bfloat16)
        G = _Grads()
        ww, wp, wt = ctx.tables
        sinks = [G.sink(p) for p in (ww, wp, wt)]
        if all(s is not None for s in sinks):  # scatter-add straight into the flat gradients
            gw, gp, gt = sinks
            ret = (None, None, None)
        else:
            G.ready = []
            gw = torch.zeros(sw, dtype=torch.float32, device=dout.device)
            gp = torch.zeros(sp, dtype=torch.float32, device=dout.device)
            gt = torch.zeros(st, dtype=torch.float32, device=dout.device)
            ret = (gw, gp, gt)
        D = sw[1]
        # stable sort of the ids: the word-table scatter then has one writer per row, summing its
        # tokens in order (no atomics, bitwise reproducible)
        sid, perm = torch.sort(ids.view(-1).clamp(0, sw[0] - 1), stable=True)
        part = torch.empty(S * 2 * D, dtype=torch.float32, device=dout.device)
        C.embed_bwd(sid, perm, ttf if has_tt else None, dout, gw, gp, gt, part, S)
        G.done()
        return (None, None) + ret + (None,)


class _ClassifierHead(torch.autograd.Function):
    """BERT pooler + classifier (reference criterion input, src/trainer.py:141-142) on the native
    kernels: pooled = tanh(cls . W_p^T + b_p) is the bf16 GEMM with the tanh epilogue (fp32 out),
    logits = pooled . W_c^T + b_c and its backward (dpre = (dlogits . W_c) * (1 - pooled^2), dW_c,
    db_c) run in head.hip; the pooler's wgrad / bias grad / dgrad are the native GEMMs / colsum."""

    @staticmethod
    def forward(ctx, cls, wp, bp, wc, bc):
        C = require_native()
        B, h = cls.shape
        pooled = torch.empty(B, wp.shape[0], dtype=torch.float32, device=cls.device)
        C.gemm(cls, bf16_weight(wp), pooled, False, False, bias=bp, mode=3)
        logits = torch.empty(B, wc.shape[0], dtype=torch.float32, device=cls.device)
        C.head_cls_fwd(pooled, wc.detach().float().contiguous(), bc.detach().float().contiguous(), logits)
        ctx.save_for_backward(cls, pooled)
        ctx.params = (wp, bp, wc, bc)
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        C = require_native()
        cls, pooled = ctx.saved_tensors
        wp, bp, wc, bc = ctx.params
        G = _Grads()
        dpre = torch.empty(pooled.shape, dtype=torch.bfloat16, device=pooled.device)
        gwc, gbc = G.sink(wc), G.sink(bc)
        both = gwc is not None and gbc is not None
        dwc = gwc if both else torch.empty(wc.shape, dtype=torch.float32, device=wc.device)
        dbc = gbc if both else torch.empty(bc.shape, dtype=torch.float32, device=bc.device)
        if not both:
            G.ready = [p for p in G.ready if p is not wc and p is not bc]
        C.head_cls_bwd(dlogits.contiguous().float(), pooled, wc.detach().float().contiguous(), dpre, dwc, dbc,
                       accumulate=both)
        dwp = G.wgrad(wp, dpre, cls)
        dbp = G.colsum(bp, dpre)
        dcls = torch.empty(cls.shape, dtype=torch.bfloat16, device=cls.device)
        C.gemm(dpre, bf16_weight(wp), dcls, False, True)
        G.done()
        return dcls, dwp, dbp, (None if both else dwc), (None if both else dbc)


def classifier_head(cls, wp, bp, wc, bc):
    """cls [B, h] bf16 (may be a strided row view) -> logits [B, num_labels] fp32."""
    return _ClassifierHead.apply(cls, wp, bp, wc, bc)


def _mark_training(impl) -> None:
    # autograd runs Function.forward with grad mode off: tell the linear implementation here
    # whether a backward will follow (fp8 keeps transposed activations only then)
    if impl is not BF16:
        type(impl).training = torch.is_grad_enabled()


def attention_block(x, wqkv, bqkv, wo, bo, lens: Optional[torch.Tensor], B: int, S: int, H: int, impl=BF16):
    _mark_training(impl)
    return _AttentionBlock.apply(x, wqkv, bqkv, wo, bo, lens, B, S, H, impl)


def ffn_block(x, w1, b1, w2, b2, impl=BF16):
    _mark_training(impl)
    return _FFNBlock.apply(x, w1, b1, w2, b2, impl)


def attention_ln_block(x, wqkv, bqkv, wo, bo, gamma, beta, lens: Optional[torch.Tensor], B: int, S: int, H: int,
                       eps: float, impl=BF16):
    _mark_training(impl)
    return _AttentionLNBlock.apply(x, wqkv, bqkv, wo, bo, gamma, beta, lens, B, S, H, eps, impl)


def ffn_ln_block(x, w1, b1, w2, b2, gamma, beta, eps: float, impl=BF16):
    _mark_training(impl)
    return _FFNLNBlock.apply(x, w1, b1, w2, b2, gamma, beta, eps, impl)


def layer_norm(x, gamma, beta, eps: float):
    return _LayerNorm.apply(x, gamma, beta, eps)


def embeddings(ids, tt, ww, wp, wt, S: int):
    return _Embeddings.apply(ids, tt, ww, wp, wt, S)
