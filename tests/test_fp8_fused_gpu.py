"""fp8 GEMM with a quantising epilogue (gemm_tile.hip q8_quadrant, C.gemm_f8_q) and the fused
FFN path built on it (ops/fp8.py fwd_gelu_q / dgrad_gelu_q) vs plain torch fp32 references."""
import math

import pytest
import torch

from ml_trainer_amd.ops._ext import require_native

pytestmark = pytest.mark.gpu

F8 = {0: torch.float8_e4m3fn, 1: torch.float8_e5m2}
FMAX = {0: 448.0, 1: 57344.0}


def _rand_f8(shape, fmt, g, dev, scale=1.0):
    x = torch.randn(*shape, generator=g) * scale
    return x.clamp(-FMAX[fmt], FMAX[fmt]).to(F8[fmt]).to(dev)


def _gelu(x):
    return 0.5 * x * (1.0 + torch.erf(x / math.sqrt(2.0)))


def _gelu_grad(x):
    return 0.5 * (1.0 + torch.erf(x / math.sqrt(2.0))) + x * torch.exp(-0.5 * x * x) / math.sqrt(2.0 * math.pi)


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("shape", [(256, 256, 128), (512, 768, 384), (1024, 512, 1024),
                                   (8192, 2048, 512), (4096, 4096, 1024)])  # the last two: >= 240 tiles
def test_gemm_f8_q_matches_fp32(dev, mode, shape):
    C = require_native()
    M, N, K = shape
    g = torch.Generator().manual_seed(M + N + K + mode)
    fa = 1 if mode == 2 else 0        # dgrad: e5m2 dY x e4m3 W^T
    fo = 1 if mode == 2 else 0        # dgrad output is a gradient (e5m2)
    A = _rand_f8((M, K), fa, g, dev, 2.0)
    B = _rand_f8((N, K), 0, g, dev, 2.0)
    isa = torch.tensor([0.5], device=dev)
    isb = torch.tensor([0.125], device=dev)
    scale = torch.tensor([3.0], device=dev)
    amax = torch.zeros(C.FP8_AMAX_SLOTS, device=dev)
    acc = (A.float() @ B.float().t()) * (0.5 * 0.125)
    bias = torch.randn(N, generator=g).to(dev) if mode != 2 else None
    if bias is not None:
        acc = acc + bias
    aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    if mode == 1:
        ref = _gelu(acc.to(torch.bfloat16).float())
    elif mode == 2:
        aux.copy_((torch.randn(M, N, generator=g) * 2).to(torch.bfloat16))
        ref = acc * _gelu_grad(aux.float())
    else:
        ref = acc
    Y = torch.empty(M, N, dtype=F8[fo], device=dev)
    Yt = torch.empty(N, M, dtype=F8[fo], device=dev)
    cs = torch.full((N,), 7.0, device=dev) if mode == 2 else None
    C.gemm_f8_q(A, B, Y, Yt, fa, 0, isa, isb, fo, scale, amax, bias=bias, aux=aux if mode else None, mode=mode,
                colsum_out=cs, colsum_accumulate=True)
    # the transposed copy is the same bytes
    assert torch.equal(Yt.view(torch.uint8), Y.view(torch.uint8).t().contiguous())
    if mode == 1:  # saved pre-activation
        torch.testing.assert_close(aux.float(), acc, rtol=1e-2, atol=1e-2 * acc.abs().max().item())
    q_ref = (ref * 3.0).clamp(-FMAX[fo], FMAX[fo])
    # one fp8 ulp (2^-3 e4m3, 2^-2 e5m2 relative) for values near a rounding boundary of a
    # differently-ordered fp32 accumulation
    rel = 0.13 if fo == 0 else 0.26
    torch.testing.assert_close(Y.float(), q_ref, rtol=rel, atol=1e-2 * q_ref.abs().max().item())
    exact = (Y.float() == q_ref.to(F8[fo]).float()).float().mean().item()
    assert exact > 0.97, exact
    torch.testing.assert_close(amax.max().view(1), ref.abs().max().view(1), rtol=1e-3, atol=1e-5)
    if cs is not None:
        torch.testing.assert_close(cs, 7.0 + ref.sum(0), rtol=1e-3, atol=1e-3 * ref.abs().sum(0).max().item())


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("shape", [(1024, 512, 1024), (8192, 2048, 512), (4096, 4096, 1024)])
def test_gemm_f8_q_4wave_matches_pingpong(dev, mode, shape):
    """The quantising epilogues on the 4-wave kernel (gemm_w4.hip W4_Q8GELU: FFN1, e4m3; W4_Q8DGELU:
    FFN2-dgrad, e5m2) write the same bytes -- fp8 Y, Y^T, the bf16 pre-activation, amax -- as the
    ping-pong kernel's (q8_quadrant); the dGELU column sums (bias gradient) agree to fp32 rounding
    (their 64-row partials are summed in a different order)."""
    C = require_native()
    M, N, K = shape
    g = torch.Generator().manual_seed(M + N + K + mode)
    fa = fo = 1 if mode == 2 else 0
    A = _rand_f8((M, K), fa, g, dev, 2.0)
    B = _rand_f8((N, K), 0, g, dev, 2.0)
    bias = torch.randn(N, generator=g).to(dev) if mode == 1 else None
    pre = (torch.randn(M, N, generator=g) * 2).to(torch.bfloat16).to(dev)
    isa, isb = torch.tensor([0.5], device=dev), torch.tensor([0.125], device=dev)
    scale = torch.tensor([3.0], device=dev)
    outs = []
    try:
        for on in (1, 0):
            C.set_gemm_w4q8(on)
            Y = torch.empty(M, N, dtype=F8[fo], device=dev)
            Yt = torch.empty(N, M, dtype=F8[fo], device=dev)
            aux = pre.clone() if mode == 2 else torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            amax = torch.zeros(C.FP8_AMAX_SLOTS, device=dev)
            cs = torch.full((N,), 7.0, device=dev) if mode == 2 else None
            C.gemm_f8_q(A, B, Y, Yt, fa, 0, isa, isb, fo, scale, amax, bias=bias, aux=aux, mode=mode,
                        colsum_out=cs, colsum_accumulate=True)
            outs.append(((Y.view(torch.uint8), Yt.view(torch.uint8), aux, amax.max()), cs))
    finally:
        C.set_gemm_w4q8(-1)
    for a, b in zip(outs[0][0], outs[1][0]):
        assert torch.equal(a, b)
    if mode == 2:
        torch.testing.assert_close(outs[0][1], outs[1][1], rtol=1e-5, atol=1e-3)


def test_gemm_f8_q_rejects_edge_shapes(dev):
    C = require_native()
    A = torch.zeros(320, 128, dtype=torch.float8_e4m3fn, device=dev)
    B = torch.zeros(256, 128, dtype=torch.float8_e4m3fn, device=dev)
    Y = torch.empty(320, 256, dtype=torch.float8_e4m3fn, device=dev)
    Yt = torch.empty(256, 320, dtype=torch.float8_e4m3fn, device=dev)
    one = torch.ones(1, device=dev)
    amax = torch.zeros(C.FP8_AMAX_SLOTS, device=dev)
    with pytest.raises(RuntimeError):
        C.gemm_f8_q(A, B, Y, Yt, 0, 0, one, one, 0, one, amax)


def _ffn_step(dev, fuse, seed=0):
    """Two forward/backward passes of one fp8 FFN block (the first initialises the scales, the
    second takes the fused path when ``fuse``); returns output and gradients of the second."""
    from ml_trainer_amd.ops import fp8 as f8
    from ml_trainer_amd.ops.transformer import ffn_block
    f8._CTX.clear()
    old = f8.Fp8Linear.fuse_q
    f8.Fp8Linear.fuse_q = fuse
    try:
        g = torch.Generator().manual_seed(seed)
        H, F, M = 256, 1024, 512
        w1 = (torch.randn(F, H, generator=g) * 0.05).to(dev).requires_grad_()
        b1 = (torch.randn(F, generator=g) * 0.1).to(dev).requires_grad_()
        w2 = (torch.randn(H, F, generator=g) * 0.05).to(dev).requires_grad_()
        b2 = (torch.randn(H, generator=g) * 0.1).to(dev).requires_grad_()
        x = torch.randn(M, H, generator=g).to(dev).to(torch.bfloat16).requires_grad_()
        dy = torch.randn(M, H, generator=g).to(dev).to(torch.bfloat16)
        out = None
        for _ in range(2):
            for p in (w1, b1, w2, b2, x):
                p.grad = None
            out = ffn_block(x, w1, b1, w2, b2, impl=f8.FP8)
            out.backward(dy)
            f8.context(dev).update()
        return out.detach().float(), [p.grad.detach().float().clone() for p in (x, w1, b1, w2, b2)]
    finally:
        f8.Fp8Linear.fuse_q = old
        f8._CTX.clear()


def test_fused_ffn_matches_unfused(dev):
    """Fused (quantising epilogues) and unfused (bf16 intermediate + cast kernels) fp8 FFN agree
    to fp8 precision, and the fused path really ran (no bf16 intermediate was saved)."""
    from ml_trainer_amd.ops import fp8 as f8
    called = {"f": 0, "b": 0}
    fwd0, bwd0 = f8.Fp8Linear.fwd_gelu_q, f8.Fp8Linear.dgrad_gelu_q

    def fwd_spy(*a, **k):
        r = fwd0(*a, **k)
        called["f"] += r is not None
        return r

    def bwd_spy(*a, **k):
        called["b"] += 1
        return bwd0(*a, **k)

    f8.Fp8Linear.fwd_gelu_q, f8.Fp8Linear.dgrad_gelu_q = staticmethod(fwd_spy), staticmethod(bwd_spy)
    try:
        yf, gf = _ffn_step(dev, True)
    finally:
        f8.Fp8Linear.fwd_gelu_q, f8.Fp8Linear.dgrad_gelu_q = staticmethod(fwd0), staticmethod(bwd0)
    assert called["f"] == 1 and called["b"] == 1, called  # second pass only (first initialises scales)
    yu, gu = _ffn_step(dev, False)
    assert ((yf - yu).norm() / yu.norm()).item() < 3e-2
    for name, a, b in zip(("x", "w1", "b1", "w2", "b2"), gf, gu):
        r = ((a - b).norm() / (b.norm() + 1e-12)).item()
        assert r < 6e-2, (name, r)


@pytest.mark.parametrize("D", [768, 1024])
@pytest.mark.parametrize("rows", [480, 4096, 20480])  # 20480: > 512 blocks x 32 rows, chunks grid-stride
def test_ln_bwd_q8_matches_ln_bwd_plus_cast(dev, D, rows):
    """C.ln_bwd_q8 (LayerNorm backward + e5m2 quantisation of dx): Y8, Y8^T and amax are bit for bit
    the separate cast-transpose of the dx it wrote; that dx matches C.ln_bwd to one bf16 rounding
    (the two kernels' fp32 expressions may contract differently), dgamma / dbeta / column sums of dx
    to fp32 rounding (partials over other row sets)."""
    C = require_native()
    g = torch.Generator().manual_seed(rows + D)
    x = (torch.randn(rows, D, generator=g) * 2 + 0.3).to(torch.bfloat16).to(dev)
    dy = (torch.randn(rows, D, generator=g) * 0.01).to(torch.bfloat16).to(dev)
    gamma = (1 + 0.1 * torch.randn(D, generator=g)).to(dev)
    beta = (0.1 * torch.randn(D, generator=g)).to(dev)
    mean = torch.empty(rows, device=dev)
    rstd = torch.empty(rows, device=dev)
    C.ln_fwd(x, gamma, beta, torch.empty_like(x), mean, rstd, 1e-12)
    scale = torch.tensor([512.0], device=dev)
    nb = max(C.ln_partial_blocks(rows), C.ln_q8_partial_blocks(rows))

    def bufs():
        return (torch.empty_like(x), torch.empty(nb * 3 * D, device=dev), *(torch.empty(D, device=dev) for _ in range(3)),
                torch.empty(rows, D, dtype=torch.float8_e5m2, device=dev),
                torch.empty(D, rows, dtype=torch.float8_e5m2, device=dev), torch.zeros(C.FP8_AMAX_SLOTS, device=dev))
    dx, part, dg, db, dxs, y8, yt8, amax = bufs()
    assert C.ln_bwd_q8(dy, x, gamma, mean, rstd, dx, part, dg, db, False, dxs, False, y8, yt8, scale, amax)
    rx, rpart, rdg, rdb, rdxs, ry8, ryt8, ramax = bufs()
    C.ln_bwd(dy, x, gamma, mean, rstd, rx, rpart, rdg, rdb, False, None, dxsum=rdxs, dxsum_acc=False)
    C.fp8_cast_transpose(dx, ry8, ryt8, scale, ramax, 1)  # the cast of the fused kernel's own dx
    assert torch.equal(y8.view(torch.uint8), ry8.view(torch.uint8))
    assert torch.equal(yt8.view(torch.uint8), ryt8.view(torch.uint8))
    assert float(amax.max()) == float(ramax.max())
    torch.testing.assert_close(dx.float(), rx.float(), rtol=8e-3, atol=1e-6)
    assert (dx != rx).float().mean().item() < 0.01
    for a, b in ((dg, rdg), (db, rdb), (dxs, rdxs)):
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-3 * b.abs().max().item())


def test_ln_bwd_q8_declines_uncovered_shapes(dev):
    C = require_native()
    D, rows = 1024, 100  # rows % 32 != 0: the caller keeps ln_bwd + the separate cast
    t = lambda *s, dt=torch.bfloat16: torch.zeros(*s, dtype=dt, device=dev)  # noqa: E731
    f8 = torch.float8_e5m2
    assert not C.ln_bwd_q8(t(rows, D), t(rows, D), t(D, dt=torch.float32), t(rows, dt=torch.float32),
                           t(rows, dt=torch.float32), t(rows, D), t(C.ln_q8_partial_blocks(rows) * 3 * D, dt=torch.float32),
                           t(D, dt=torch.float32), t(D, dt=torch.float32), False, t(D, dt=torch.float32), False,
                           t(rows, D, dt=f8), t(D, rows, dt=f8), t(1, dt=torch.float32) + 1,
                           t(C.FP8_AMAX_SLOTS, dt=torch.float32))


def test_fp8_bert_ln_quantised_dy_matches_separate_cast(dev, monkeypatch):
    """A 768-wide fp8 encoder layer trained a few steps with the LayerNorm backward quantising the
    out-proj / FFN2 dY (Fp8Linear.fuse_ln, opt-in) vs the separate cast-transpose: the fused kernel runs
    (2 calls per layer per step once the scales exist) and the losses agree to fp32 rounding of the
    LayerNorm partial sums."""
    import torch.nn.functional as F
    from ml_trainer_amd.models.bert import BertClassifier, bert_config
    from ml_trainer_amd.ops import fp8 as fp8mod
    from ml_trainer_amd.ops.optim import FusedAdamW
    C = require_native()
    calls = []
    real = C.ln_bwd_q8

    def counting(*a):
        r = real(*a)
        calls.append(r)
        return r
    monkeypatch.setattr(C, "ln_bwd_q8", counting)
    cfg = bert_config("bert-tiny", fp8=True, hidden=768, heads=12, intermediate=3072, layers=1)
    ids = torch.randint(5, 1000, (4, 128), device=dev)
    y = torch.randint(0, 2, (4,), device=dev)
    losses = {}
    for fuse in (True, False):
        monkeypatch.setattr(fp8mod.Fp8Linear, "fuse_ln", fuse)
        fp8mod._CTX.clear()  # fresh delayed-scaling state for each run
        torch.manual_seed(0)
        m = BertClassifier(cfg).to(dev)
        opt = FusedAdamW(m.parameters(), lr=1e-4)
        ls = []
        for _ in range(4):
            opt.zero_grad()
            loss = F.cross_entropy(m(ids), y)
            loss.backward()
            opt.step()
            ls.append(float(loss))
        losses[fuse] = ls
    assert calls and all(calls), calls
    for a, b in zip(losses[True], losses[False]):
        assert abs(a - b) <= 2e-3 * abs(b) + 1e-4, losses


@pytest.mark.parametrize("B,S,H,use_lens", [(2, 512, 3, False), (2, 256, 2, True), (3, 128, 2, True)])
@pytest.mark.parametrize("grp", ["1", "2"])
def test_attn_bwd_q8_matches_bf16_plus_cast(dev, B, S, H, use_lens, grp, monkeypatch):
    """attn_bwd with q8 outputs (fp8 training): the e5m2 dQKV, its transpose and amax written by the
    dQ / dK-dV ring kernels are bit for bit fp8_cast_transpose of the bf16 dQKV the same kernels
    write without them (incl. fully masked key blocks), and the bias column sums are the same."""
    C = require_native()
    monkeypatch.setenv("MLT_ATTN_DKDV_GROUPS", grp)
    monkeypatch.setenv("MLT_ATTN_DQ_GROUPS", grp)
    g = torch.Generator().manual_seed(S + H + B)
    D = H * 64
    qkv = torch.randn(B * S, 3 * D, generator=g).to(torch.bfloat16).to(dev)
    dout = (torch.randn(B * S, D, generator=g) * 0.1).to(torch.bfloat16).to(dev)
    lens = torch.tensor([7, S, 100][:B], dtype=torch.int32).to(dev) if use_lens else None
    scale = 0.125
    out = torch.empty(B * S, D, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B * H * S, device=dev)
    C.attn_fwd(qkv, out, lse, lens, B, S, H, scale)
    qscale = torch.tensor([2048.0], device=dev)
    dqkv = torch.empty_like(qkv)
    delta = torch.empty(B * S * H, device=dev)
    cs = torch.empty(3 * D, device=dev)
    C.attn_bwd(qkv, out, dout, lse, delta, lens, dqkv, B, S, H, scale, colsum_out=cs)
    ry8 = torch.empty(B * S, 3 * D, dtype=torch.float8_e5m2, device=dev)
    ryt8 = torch.empty(3 * D, B * S, dtype=torch.float8_e5m2, device=dev)
    ramax = torch.zeros(C.FP8_AMAX_SLOTS, device=dev)
    C.fp8_cast_transpose(dqkv, ry8, ryt8, qscale, ramax, 1)
    y8 = torch.empty_like(ry8)
    yt8 = torch.empty_like(ryt8)
    amax = torch.zeros_like(ramax)
    cs8 = torch.empty_like(cs)
    C.attn_bwd(qkv, out, dout, lse, torch.empty_like(delta), lens, torch.empty_like(qkv), B, S, H, scale,
               colsum_out=cs8, q8_y=y8, q8_yt=yt8, q8_scale=qscale, q8_amax=amax)
    assert torch.equal(y8.view(torch.uint8), ry8.view(torch.uint8))
    assert torch.equal(yt8.view(torch.uint8), ryt8.view(torch.uint8))
    assert float(amax.max()) == float(ramax.max()) > 0
    assert torch.equal(cs8, cs)


def test_fp8_bert_attn_quantised_dy_matches_separate_cast(dev, monkeypatch):
    """A 768-wide fp8 encoder layer trained a few steps with the attention backward writing the QKV
    projection's e5m2 dY (Fp8Linear.fuse_attn, default) vs the bf16 dQKV + separate cast-transpose:
    the q8 path runs once the scales exist, and the runs agree to the rounding of the QKV bias
    gradient (column sums of the fp32 values in the kernels vs of the bf16 dQKV in the cast; the
    e5m2 operands themselves are bitwise equal, test above)."""
    import torch.nn.functional as F
    from ml_trainer_amd.models.bert import BertClassifier, bert_config
    from ml_trainer_amd.ops import fp8 as fp8mod
    from ml_trainer_amd.ops.optim import FusedAdamW
    C = require_native()
    calls = []
    real = C.attn_bwd

    def counting(*a, **k):
        calls.append(k.get("q8_y") is not None)
        return real(*a, **k)
    monkeypatch.setattr(C, "attn_bwd", counting)
    cfg = bert_config("bert-tiny", fp8=True, hidden=768, heads=12, intermediate=3072, layers=1)
    ids = torch.randint(5, 1000, (4, 128), generator=torch.Generator().manual_seed(1)).to(dev)
    y = torch.tensor([0, 1, 1, 0], device=dev)
    res = {}
    for fuse in (True, False):
        monkeypatch.setattr(fp8mod.Fp8Linear, "fuse_attn", fuse)
        fp8mod._CTX.clear()
        calls.clear()
        torch.manual_seed(0)
        m = BertClassifier(cfg).to(dev)
        opt = FusedAdamW(m.parameters(), lr=1e-4)
        losses = []
        for _ in range(4):
            opt.zero_grad(set_to_none=False)
            loss = F.cross_entropy(m(ids), y)
            loss.backward()
            opt.step()
            losses.append(float(loss))
        res[fuse] = (losses, [p.detach().clone() for p in m.parameters()], list(calls))
    assert any(res[True][2]) and not any(res[False][2])
    assert res[True][0][0] == res[False][0][0]  # (step 1: the scales did not exist yet, same path)
    torch.testing.assert_close(torch.tensor(res[True][0]), torch.tensor(res[False][0]), rtol=1e-3, atol=1e-4)
    # (Adam turns rounding-level gradient differences on near-zero gradients into +-lr steps, so
    # elementwise closeness is the wrong yardstick: the tensors' relative distance is)
    # (the zero-initialised biases, 4 Adam steps from zero, are left out: there a rounding-level
    # gradient difference is a +-lr step of its own; the weights carry the comparison)
    for a, b in zip(res[True][1], res[False][1]):
        if b.float().norm().item() < 0.05:
            continue
        d = a.float() - b.float()
        rel = (d.norm() / b.float().norm()).item()
        assert rel < 2e-3, rel
