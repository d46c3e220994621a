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
    amax = torch.zeros(1, device=dev)
    y = torch.empty(x.numel(), dtype=F8[fmt], device=dev)
    C.fp8_cast(x, y, scale, amax, fmt)
    ref = (x.float() * 0.75).clamp(-FMAX[fmt], FMAX[fmt]).to(F8[fmt])
    mism = (y.float() != ref.float()).float().mean().item()
    assert mism < 1e-3, mism
    assert float(y[5].float()) == FMAX[fmt]
    torch.testing.assert_close(amax, x.float().abs().max().view(1))


def test_cast_transpose_and_scale_update(dev):
    C = require_native()
    g = torch.Generator().manual_seed(3)
    w = torch.randn(192, 320, generator=g).to(dev)
    y = torch.empty(192, 320, dtype=torch.float8_e4m3fn, device=dev)
    yt = torch.empty(320, 192, dtype=torch.float8_e4m3fn, device=dev)
    scale = torch.tensor([4.0], device=dev)
    amax = torch.zeros(1, device=dev)
    C.fp8_cast_transpose(w, y, yt, scale, amax, 0)
    ref = (w * 4.0).clamp(-448, 448).to(torch.float8_e4m3fn)
    assert (y.float() != ref.float()).float().mean().item() < 1e-3
    assert torch.equal(yt.view(torch.uint8), y.view(torch.uint8).t().contiguous())
    torch.testing.assert_close(amax, w.abs().max().view(1))
    hist = torch.zeros(4, device=dev)
    inv = torch.ones(1, device=dev)
    step = torch.zeros(1, dtype=torch.int64, device=dev)
    C.fp8_update_scale(hist, amax, scale, inv, step, 0, 0)
    torch.testing.assert_close(scale, 448.0 / w.abs().max().view(1))
    torch.testing.assert_close(inv * scale, torch.ones(1, device=dev))
    assert float(amax) == 0.0 and int(step) == 1


@pytest.mark.parametrize("cfg,splits", [(1, 1), (2, 1), (3, 1), (4, 1), (1, 2), (4, 3)])
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
    out = torch.empty(M, 64, dtype=torch.float32, device=dev)
    C.gemm_f8(A, B, out, 0, 0, one, one, cfg=1)
    torch.testing.assert_close(out, B.float()[:, :M].t())
