"""FP8 (OCP e4m3 / e5m2) kernels: quantisation (fp8.hip) and the MX-scaled MFMA GEMM
(gemm_tile.hip, F8 variant) vs plain torch fp32 references."""
import pytest
import torch

from ml_trainer_amd.ops._ext import require_native

pytestmark = pytest.mark.gpu

F8 = {0: torch.float8_e4m3fn, 1: torch.float8_e5m2}
FMAX = {0: 448.0, 1: 57344.0}


def _rand_f8(shape, fmt, g, dev, scale=1.0):
    x = torch.randn(*shape, generator=g) * scale
    return x.clamp(-FMAX[fmt], FMAX[fmt]).to(F8[fmt]).to(dev)


@pytest.mark.parametrize("fmt", [0, 1])
@pytest.mark.parametrize("src", [torch.bfloat16, torch.float32])
def test_cast_fp8_matches_torch(dev, fmt, src):
    C = require_native()
    g = torch.Generator().manual_seed(fmt)
    x = (torch.randn(4096 + 64, generator=g) * 30).to(src).to(dev)
    x[5] = 1e6  # saturates
    scale = torch.tensor([0.75], device=dev)
    amax = torch.zeros(C.FP8_AMAX_SLOTS, device=dev)
    y = torch.empty(x.numel(), dtype=F8[fmt], device=dev)
    C.fp8_cast(x, y, scale, amax, fmt)
    ref = (x.float() * 0.75).clamp(-FMAX[fmt], FMAX[fmt]).to(F8[fmt])
    mism = (y.float() != ref.float()).float().mean().item()
    assert mism < 1e-3, mism
    assert float(y[5].float()) == FMAX[fmt]
    torch.testing.assert_close(amax.max().view(1), x.float().abs().max().view(1))


def test_cast_transpose_and_scale_update(dev):
    C = require_native()
    g = torch.Generator().manual_seed(3)
    w = torch.randn(192, 320, generator=g).to(dev)
    y = torch.empty(192, 320, dtype=torch.float8_e4m3fn, device=dev)
    yt = torch.empty(320, 192, dtype=torch.float8_e4m3fn, device=dev)
    scale = torch.tensor([4.0], device=dev)
    amax = torch.zeros(1, C.FP8_AMAX_SLOTS, device=dev)
    C.fp8_cast_transpose(w, y, yt, scale, amax[0], 0)
    ref = (w * 4.0).clamp(-448, 448).to(torch.float8_e4m3fn)
    assert (y.float() != ref.float()).float().mean().item() < 1e-3
    assert torch.equal(yt.view(torch.uint8), y.view(torch.uint8).t().contiguous())
    torch.testing.assert_close(amax.max().view(1), w.abs().max().view(1))
    hist = torch.zeros(1, 4, device=dev)
    inv = torch.ones(1, device=dev)
    fmax = torch.tensor([448.0], device=dev)
    C.fp8_update_scale(hist, amax, scale, inv, fmax, 0, 0)
    torch.testing.assert_close(scale, 448.0 / w.abs().max().view(1))
    torch.testing.assert_close(inv * scale, torch.ones(1, device=dev))
    assert float(amax.abs().sum()) == 0.0
    # history window: a smaller amax later does not lower the scale until it falls out
    amax[0, 3 * 32] = 1.0  # slot 3 (slots are 32 floats apart)
    C.fp8_update_scale(hist, amax, scale, inv, fmax, 1, 1)
    torch.testing.assert_close(scale, 448.0 / (w.abs().max().view(1) * 2))


@pytest.mark.parametrize("cfg,splits", [(1, 1), (2, 1), (3, 1), (4, 1), (5, 1), (6, 1), (1, 2), (4, 3), (5, 3)])
@pytest.mark.parametrize("fmts", [(0, 0), (1, 0), (0, 1)])
def test_gemm_f8(dev, cfg, splits, fmts):
    C = require_native()
    fa, fb = fmts
    M, N, K = 320, 200, 1024
    g = torch.Generator().manual_seed(cfg * 10 + splits + 100 * fa + 7 * fb)
    A = _rand_f8((M, K), fa, g, dev, 4.0)
    B = _rand_f8((N, K), fb, g, dev, 4.0)
    isa = torch.tensor([0.5], device=dev)
    isb = torch.tensor([0.25], device=dev)
    ref = (A.float() @ B.float().t()) * 0.125
    out = torch.empty(M, N, dtype=torch.float32, device=dev)
    C.gemm_f8(A, B, out, fa, fb, isa, isb, cfg=cfg, splits=splits)
    # the fp8 MFMA's internal accumulation of 128-deep products is not a plain fp32 fma chain:
    # compare relative to the output magnitude
    torch.testing.assert_close(out, ref, rtol=2e-3, atol=2e-4 * ref.abs().max().item())
    bias = torch.randn(N, device=dev)
    res = torch.randn(M, N, device=dev).to(torch.bfloat16)
    ob = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    C.gemm_f8(A, B, ob, fa, fb, isa, isb, bias=bias, res=res, cfg=cfg, splits=splits)
    torch.testing.assert_close(ob.float(), ref + bias + res.float(), rtol=1e-2, atol=0.5)


def test_gemm_f8_identity_asymmetric(dev):
    C = require_native()
    M = 128
    A = torch.eye(M, 256).to(torch.float8_e4m3fn).to(dev)                            # [M][K]
    B = ((torch.arange(64 * 256).view(64, 256) % 13) - 6).float().to(torch.float8_e4m3fn).to(dev)  # [N][K]
    one = torch.ones(1, device=dev)
    for cfg in (1, 6):  # 6: persistent kernel with swapped MFMA operands (C^T fragments)
        out = torch.empty(M, 64, dtype=torch.float32, device=dev)
        C.gemm_f8(A, B, out, 0, 0, one, one, cfg=cfg)
        torch.testing.assert_close(out, B.float()[:, :M].t())


def _tiny_fp8_pair(dev):
    from ml_trainer_amd.models.bert import BertClassifier, bert_config
    torch.manual_seed(0)
    m8 = BertClassifier(bert_config("bert-tiny", fp8=True)).to(dev)
    m16 = BertClassifier(bert_config("bert-tiny")).to(dev)
    m16.load_state_dict(m8.state_dict())
    return m8, m16


def test_fp8_bert_close_to_bf16(dev):
    import torch.nn.functional as F
    m8, m16 = _tiny_fp8_pair(dev)
    ids = torch.randint(5, 1000, (4, 128), device=dev)
    y = torch.randint(0, 2, (4,), device=dev)
    o8, o16 = m8(ids), m16(ids)
    rel = (o8 - o16).norm() / o16.norm()
    assert rel < 0.1, rel
    F.cross_entropy(o8, y).backward()
    F.cross_entropy(o16, y).backward()
    for (n, p8), p16 in zip(m8.named_parameters(), m16.parameters()):
        r = (p8.grad - p16.grad).norm() / (p16.grad.norm() + 1e-12)
        assert r < 0.25, (n, float(r))


def test_fp8_bert_trains(dev):
    import torch.nn.functional as F
    from ml_trainer_amd.ops.optim import FusedAdamW
    m8, _ = _tiny_fp8_pair(dev)
    opt = FusedAdamW(m8.parameters(), lr=3e-4)
    ids = torch.randint(5, 1000, (8, 128), device=dev)
    y = torch.randint(0, 2, (8,), device=dev)
    ids[y == 1, 7] = 3
    losses = []
    for _ in range(30):
        opt.zero_grad()
        loss = F.cross_entropy(m8(ids), y)
        loss.backward()
        opt.step()
        losses.append(float(loss))
    assert losses[-1] < 0.5 * losses[0], losses
    from ml_trainer_amd.ops.fp8 import context
    ctx = context(ids.device)
    assert ctx.n > 0 and torch.isfinite(ctx.scale[:ctx.n]).all() and (ctx.scale[:ctx.n] > 0).all()


@pytest.mark.parametrize("fmt", [0, 1])
@pytest.mark.parametrize("shape", [(256, 192), (384, 512), (1024, 3072)])  # 64x64 kernel / 128x128 wide kernel
def test_cast_transpose_bf16_input(dev, fmt, shape):
    C = require_native()
    R, Cc = shape
    g = torch.Generator().manual_seed(5 + fmt)
    x = torch.randn(R, Cc, generator=g).to(dev).to(torch.bfloat16)
    dt = torch.float8_e4m3fn if fmt == 0 else torch.float8_e5m2
    y = torch.empty(R, Cc, dtype=dt, device=dev)
    yt = torch.empty(Cc, R, dtype=dt, device=dev)
    scale = torch.tensor([2.0], device=dev)
    amax = torch.zeros(C.FP8_AMAX_SLOTS, device=dev)
    C.fp8_cast_transpose(x, y, yt, scale, amax, fmt)
    fm = 448.0 if fmt == 0 else 57344.0
    ref = (x.float() * 2.0).clamp(-fm, fm).to(dt)
    assert (y.float() != ref.float()).float().mean().item() < 1e-3
    assert torch.equal(yt.view(torch.uint8), y.view(torch.uint8).t().contiguous())
    assert float(amax.max()) == float(x.float().abs().max())


@pytest.mark.parametrize("shape", [(256, 192), (384, 512), (1024, 3072)])
@pytest.mark.parametrize("acc", [False, True])
def test_cast_transpose_fused_colsum(dev, shape, acc):
    """Bias-gradient column sums from the dY cast (wide kernel partials + fixed-order reduce, or
    the separate colsum on the 64x64 path) vs an fp32 torch reduction; casts are unchanged."""
    C = require_native()
    R, Cc = shape
    g = torch.Generator().manual_seed(11)
    x = torch.randn(R, Cc, generator=g).to(dev).to(torch.bfloat16)
    y = torch.empty(R, Cc, dtype=torch.float8_e5m2, device=dev)
    yt = torch.empty(Cc, R, dtype=torch.float8_e5m2, device=dev)
    y2, yt2 = torch.empty_like(y), torch.empty_like(yt)
    scale = torch.tensor([4.0], device=dev)
    amax = torch.zeros(C.FP8_AMAX_SLOTS, device=dev)
    base = torch.randn(Cc, generator=g).to(dev)
    out = base.clone() if acc else torch.full((Cc,), float("nan"), device=dev)
    C.fp8_cast_transpose(x, y, yt, scale, amax, 1, colsum_out=out, colsum_accumulate=acc)
    C.fp8_cast_transpose(x, y2, yt2, scale, None, 1)
    assert torch.equal(y.view(torch.uint8), y2.view(torch.uint8)) and torch.equal(yt.view(torch.uint8), yt2.view(torch.uint8))
    ref = x.float().sum(0) + (base if acc else 0.0)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-3)
    out2 = base.clone() if acc else torch.empty(Cc, device=dev)
    C.fp8_cast_transpose(x, y2, yt2, scale, None, 1, colsum_out=out2, colsum_accumulate=acc)
    assert torch.equal(out, out2)  # deterministic


def test_fp8_weight_gradient_path(dev):
    """Fp8Linear: forward caches X^T (e4m3), wgrad casts dY with its transpose (e5m2), runs
    dY^T . X^T in fp8 and hands the e5m2 dY to the dgrad that follows."""
    from ml_trainer_amd.ops.fp8 import FP8, context
    g = torch.Generator().manual_seed(9)
    T, I, O = 512, 256, 384
    x = (torch.randn(T, I, generator=g) * 0.5).to(dev).to(torch.bfloat16)
    w = torch.nn.Parameter((torch.randn(O, I, generator=g) * 0.05).to(dev))
    dy = (torch.randn(T, O, generator=g) * 0.1).to(dev).to(torch.bfloat16)
    ctx = context(x.device)
    for _ in range(3):  # delayed scaling settles after the first steps
        FP8.fwd(x, w)
        st = w._mlt_f8
        assert st.xt is not None and st.xt[0] == x.data_ptr()
        dw = FP8.wgrad(w, dy, x, None)
        assert dw is not None and st.xt is None and st.dy8 is not None
        out = torch.empty(T, I, dtype=torch.bfloat16, device=dev)
        FP8.dgrad(dy, w, out)
        assert st.dy8 is None
        ctx.update()
    ref_dw = dy.float().t() @ x.float()
    rel = (dw - ref_dw).norm() / ref_dw.norm()
    assert rel < 0.1, float(rel)
    ref_dx = dy.float() @ w.detach().float()
    rel = (out.float() - ref_dx).norm() / ref_dx.norm()
    assert rel < 0.1, float(rel)
    # accumulate form
    acc = torch.ones(O, I, device=dev)
    FP8.fwd(x, w)
    assert FP8.wgrad(w, dy, x, acc) is acc
    assert ((acc - 1 - ref_dw).norm() / ref_dw.norm()) < 0.1


def test_fp8_bert_uses_fp8_weight_gradients(dev):
    """Through the autograd blocks (grad mode is off inside Function.forward) the forward still
    keeps X^T and the backward consumes it: no weight is left with an unused transpose."""
    import torch.nn.functional as F
    m8, _ = _tiny_fp8_pair(dev)
    ids = torch.randint(5, 1000, (2, 128), device=dev)
    out = m8(ids)
    lin = [p for n, p in m8.named_parameters() if p.dim() == 2 and hasattr(p, "_mlt_f8")]
    assert lin and all(p._mlt_f8.xt is not None for p in lin)
    F.cross_entropy(out, torch.zeros(2, dtype=torch.long, device=dev)).backward()
    assert all(p._mlt_f8.xt is None for p in lin)
    with torch.no_grad():
        m8(ids)
    assert all(p._mlt_f8.xt is None for p in lin)  # inference keeps no transposes


def test_fp8_wgrad_bias_fused_and_fallback(dev):
    """_Grads.wgrad_bias with the fp8 impl: the bias gradient comes out of the dY cast when the
    forward kept X^T, and from the separate colsum when it did not -- same values either way."""
    from ml_trainer_amd.ops.fp8 import FP8
    from ml_trainer_amd.ops.transformer import _Grads
    g = torch.Generator().manual_seed(13)
    T, I, O = 512, 256, 384
    x = (torch.randn(T, I, generator=g) * 0.5).to(dev).to(torch.bfloat16)
    w = torch.nn.Parameter((torch.randn(O, I, generator=g) * 0.05).to(dev))
    b = torch.nn.Parameter(torch.zeros(O, device=dev))
    dy = (torch.randn(T, O, generator=g) * 0.1).to(dev).to(torch.bfloat16)
    ref_db = dy.float().sum(0)
    FP8.fwd(x, w, b)
    G = _Grads()
    dw, db = G.wgrad_bias(w, b, dy, x, FP8)  # fused: X^T cached by the forward
    assert dw is not None and w._mlt_f8.xt is None
    torch.testing.assert_close(db, ref_db, rtol=1e-5, atol=1e-3)
    dw2, db2 = G.wgrad_bias(w, b, dy, x, FP8)  # no cached X^T: bf16 wgrad + separate colsum
    torch.testing.assert_close(db2, ref_db, rtol=1e-5, atol=1e-3)
    ref_dw = dy.float().t() @ x.float()
    assert ((dw2 - ref_dw).norm() / ref_dw.norm()) < 0.02 and ((dw - ref_dw).norm() / ref_dw.norm()) < 0.1


@pytest.mark.parametrize("fmts", [(0, 0), (1, 0), (0, 1)])
def test_gemm_f8_w4_asm(dev, fmts):
    """Config 7 in fp8 (4-wave tile, generated-asm loop on v_mfma_scale_f32_16x16x128_f8f6f4 with unit
    scales, A double-buffered / B column-refilled fragments): fp32 and bf16 outputs, bias + residual,
    GELU with the pre-activation, dGELU; the planner picks it for 256-multiple shapes."""
    C = require_native()
    fa, fb = fmts
    M, N, K = 1024, 768, 1536  # 12 tiles; 12 K-tiles of 128 (6 pairs: peeled + loop + last)
    g = torch.Generator().manual_seed(300 + 10 * fa + fb)
    A = _rand_f8((M, K), fa, g, dev, 4.0)
    B = _rand_f8((N, K), fb, g, dev, 4.0)
    # the planner takes cfg 7 when the tiles fill the chip, split-K tiles for few-tile long-K shapes
    assert C.gemm_f8_plan(65536, 1024, 1024)[0] == 7
    plan = C.gemm_f8_plan(1024, 1024, 262144)  # few tiles, long K: split-K partials (ext reduce)
    assert plan[0] == 7 and plan[1] > 1 and plan[4] == 1, plan
    isa = torch.tensor([0.5], device=dev)
    isb = torch.tensor([0.25], device=dev)
    ref = (A.float() @ B.float().t()) * 0.125
    out = torch.empty(M, N, dtype=torch.float32, device=dev)
    C.gemm_f8(A, B, out, fa, fb, isa, isb, cfg=7)
    torch.testing.assert_close(out, ref, rtol=2e-3, atol=2e-4 * ref.abs().max().item())
    out5 = torch.empty_like(out)
    C.gemm_f8(A, B, out5, fa, fb, isa, isb, cfg=5)
    torch.testing.assert_close(out, out5, rtol=1e-5, atol=1e-5 * ref.abs().max().item())
    bias = torch.randn(N, device=dev)
    res = torch.randn(M, N, device=dev).to(torch.bfloat16)
    ob = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    C.gemm_f8(A, B, ob, fa, fb, isa, isb, bias=bias, res=res, cfg=7)
    torch.testing.assert_close(ob.float(), ref + bias + res.float(), rtol=1e-2, atol=0.5)
    aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    C.gemm_f8(A, B, ob, fa, fb, isa, isb, bias=bias, aux=aux, mode=1, cfg=7)
    torch.testing.assert_close(aux.float(), ref + bias, rtol=1e-2, atol=0.5)
    torch.testing.assert_close(ob.float(), torch.nn.functional.gelu(aux.float()), rtol=1e-2, atol=0.05)


def test_gemm_f8_w4_identity_asymmetric(dev):
    """Operand roles / fragment layout of the fp8 asm loop: A = I picks rows of B exactly."""
    C = require_native()
    M, N, K = 256, 256, 512
    A = torch.eye(M, K).to(torch.float8_e4m3fn).to(dev)
    B = ((torch.arange(N * K).view(N, K) % 13) - 6).float().to(torch.float8_e4m3fn).to(dev)
    one = torch.ones(1, device=dev)
    out = torch.empty(M, N, dtype=torch.float32, device=dev)
    C.gemm_f8(A, B, out, 0, 0, one, one, cfg=7)
    torch.testing.assert_close(out, B.float()[:, :M].t())


def test_gemm_f8_w4_split_k(dev):
    """cfg 7 fp8 with split-K raw partials and the external reduce (the fp8 weight-gradient path):
    inverse scales, bias, fp32 accumulate and bf16 outputs against an fp32 reference."""
    C = require_native()
    M, N, K = 512, 768, 16384
    plan = C.gemm_f8_plan(M, N, K)
    assert plan[0] == 7 and plan[1] > 1 and plan[4] == 1, plan
    g = torch.Generator().manual_seed(410)
    A = _rand_f8((M, K), 1, g, dev, 2.0)
    B = _rand_f8((N, K), 0, g, dev, 2.0)
    isa = torch.tensor([0.5], device=dev)
    isb = torch.tensor([0.25], device=dev)
    ref = (A.float() @ B.float().t()) * 0.125
    acc = torch.full((M, N), 0.5, device=dev)
    C.gemm_f8(A, B, acc, 1, 0, isa, isb, accumulate=True)
    torch.testing.assert_close(acc, ref + 0.5, rtol=2e-3, atol=2e-4 * ref.abs().max().item())
    bias = torch.randn(N, device=dev)
    ob = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    C.gemm_f8(A, B, ob, 1, 0, isa, isb, bias=bias)
    torch.testing.assert_close(ob.float(), ref + bias, rtol=1e-2, atol=0.5)
