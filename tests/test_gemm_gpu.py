"""bf16 MFMA GEMM (csrc/kernels/gemm.hip) vs a plain torch fp32 reference of the same op."""
import math

import pytest
import torch

from ml_trainer_amd.ops._ext import require_native

pytestmark = pytest.mark.gpu


def _mk(shape, dev, g):
    return (torch.randn(*shape, generator=g, device="cpu") * 0.5).to(torch.bfloat16).to(dev)


def _ref(A, B, a_mn, b_mn):
    a = A.float().t() if a_mn else A.float()
    b = B.float() if b_mn else B.float().t()
    return a @ b


@pytest.mark.parametrize("a_mn,b_mn", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (256, 384, 192), (136, 72, 40), (8, 8, 8), (520, 264, 1000)])
@pytest.mark.parametrize("out", [torch.bfloat16, torch.float32])
def test_gemm_layouts(dev, a_mn, b_mn, M, N, K, out):
    C = require_native()
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K)
    A = _mk((K, M) if a_mn else (M, K), dev, g)
    B = _mk((K, N) if b_mn else (N, K), dev, g)
    Cm = torch.empty(M, N, dtype=out, device=dev)
    C.gemm(A, B, Cm, bool(a_mn), bool(b_mn))
    ref = _ref(A, B, a_mn, b_mn)
    tol = 2e-2 if out == torch.bfloat16 else 2e-3
    torch.testing.assert_close(Cm.float(), ref, rtol=tol, atol=tol * max(1.0, (K ** 0.5) * 0.25))


def test_identity_asymmetric(dev):
    """A = I with an asymmetric B catches any transposed C write (guide §3)."""
    C = require_native()
    M = 128
    A = torch.eye(M, dtype=torch.bfloat16, device=dev)
    B = (torch.arange(M * 64, device=dev).view(64, M) % 251).to(torch.bfloat16)  # B stored [N=64][K=128]
    out = torch.empty(M, 64, dtype=torch.float32, device=dev)
    C.gemm(A, B, out, False, False)
    torch.testing.assert_close(out, B.float().t())


def test_epilogues(dev):
    C = require_native()
    g = torch.Generator().manual_seed(0)
    M, N, K = 256, 192, 128
    A, B = _mk((M, K), dev, g), _mk((N, K), dev, g)
    bias = torch.randn(N, device=dev)
    res = _mk((M, N), dev, g)
    ref = A.float() @ B.float().t()
    # bias + residual + alpha
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    C.gemm(A, B, out, False, False, bias=bias, res=res, alpha=0.5)
    torch.testing.assert_close(out.float(), 0.5 * ref + bias + res.float(), rtol=2e-2, atol=3e-2)
    # GELU: pre-activation saved to aux
    aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    C.gemm(A, B, out, False, False, bias=bias, aux=aux, mode=1)
    pre = ref + bias
    torch.testing.assert_close(aux.float(), pre, rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(out.float(), torch.nn.functional.gelu(aux.float()), rtol=2e-2, atol=3e-2)
    # dGELU: result * gelu'(aux)
    x = aux.float().requires_grad_(True)
    torch.nn.functional.gelu(x).backward(torch.ones_like(x))
    C.gemm(A, B, out, False, False, aux=aux, mode=2)
    torch.testing.assert_close(out.float(), ref * x.grad, rtol=3e-2, atol=5e-2)
    # fp32 accumulate
    acc = torch.ones(M, N, device=dev)
    C.gemm(A, B, acc, False, False, accumulate=True)
    torch.testing.assert_close(acc, ref + 1, rtol=2e-3, atol=2e-3)


def test_colsum(dev):
    C = require_native()
    X = torch.randn(1000, 304, device=dev).to(torch.bfloat16)
    out = torch.zeros(304, device=dev)
    C.colsum(X, out, False)
    torch.testing.assert_close(out, X.float().sum(0), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("cfg,splits", [(1, 1), (2, 1), (3, 1), (4, 1), (5, 1), (1, 3), (2, 4), (3, 2), (4, 2),
                                        (5, 3), (5, 5)])
@pytest.mark.parametrize("a_mn,b_mn", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_tile_kernels(dev, cfg, splits, a_mn, b_mn):
    """256-wide global_load_lds kernels (gemm_tile.hip), forced config / split-K, with M/N tails
    and a strided leading dimension, vs the fp32 reference; epilogues on the split-K path."""
    C = require_native()
    M, N, K = 328, 264, 768
    g = torch.Generator().manual_seed(cfg * 100 + splits * 10 + a_mn * 2 + b_mn)
    A = _mk((K, M + 8) if a_mn else (M, K + 64), dev, g)
    A = A[:, :M] if a_mn else A[:, :K]
    B = _mk((K, N) if b_mn else (N, K), dev, g)
    ref = _ref(A, B, a_mn, b_mn)
    plan = C.gemm_plan(bool(a_mn), bool(b_mn), M, N, K, cfg, splits)
    assert plan[0] == cfg and plan[1] == splits
    for out_dtype in (torch.bfloat16, torch.float32):
        out = torch.empty(M, N, dtype=out_dtype, device=dev)
        C.gemm(A, B, out, bool(a_mn), bool(b_mn), cfg=cfg, splits=splits)
        tol = 2e-2 if out_dtype == torch.bfloat16 else 2e-3
        torch.testing.assert_close(out.float(), ref, rtol=tol, atol=tol * 8)
    bias = torch.randn(N, device=dev)
    res = _mk((M, N), dev, g)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    C.gemm(A, B, out, bool(a_mn), bool(b_mn), bias=bias, aux=aux, mode=1, cfg=cfg, splits=splits)
    torch.testing.assert_close(aux.float(), ref + bias, rtol=2e-2, atol=0.15)
    torch.testing.assert_close(out.float(), torch.nn.functional.gelu(aux.float()), rtol=2e-2, atol=0.15)
    C.gemm(A, B, out, bool(a_mn), bool(b_mn), res=res, alpha=0.5, cfg=cfg, splits=splits)
    torch.testing.assert_close(out.float(), 0.5 * ref + res.float(), rtol=2e-2, atol=0.15)
    acc = torch.ones(M, N, device=dev)
    C.gemm(A, B, acc, bool(a_mn), bool(b_mn), accumulate=True, cfg=cfg, splits=splits)
    torch.testing.assert_close(acc, ref + 1, rtol=2e-3, atol=2e-2)
    # dGELU epilogue (interior tile takes the prefetched side-operand path, tails the general one)
    pre = _mk((M, N), dev, g)
    C.gemm(A, B, out, bool(a_mn), bool(b_mn), aux=pre, mode=2, cfg=cfg, splits=splits)
    x = pre.float()
    dg = 0.5 * (1 + torch.erf(x * 0.7071067811865476)) + x * torch.exp(-0.5 * x * x) * 0.3989422804014327
    torch.testing.assert_close(out.float(), ref * dg, rtol=2e-2, atol=0.15)


def test_tile_split_k_deterministic(dev):
    C = require_native()
    g = torch.Generator().manual_seed(7)
    A = _mk((4096, 768), dev, g)   # [K][M]
    B = _mk((4096, 1024), dev, g)  # [K][N]
    outs = []
    for _ in range(3):
        o = torch.empty(768, 1024, device=dev)
        C.gemm(A, B, o, True, True, cfg=1, splits=8)
        outs.append(o)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    torch.testing.assert_close(outs[0], A.float().t() @ B.float(), rtol=2e-3, atol=2e-2)


def test_identity_asymmetric_tile(dev):
    C = require_native()
    M = 256
    A = torch.eye(M, dtype=torch.bfloat16, device=dev)
    B = (torch.arange(M * 128, device=dev).view(128, M) % 251).to(torch.bfloat16)
    for cfg in (1, 2, 3, 4, 5, 6):
        out = torch.empty(M, 128, dtype=torch.float32, device=dev)
        C.gemm(A, B, out, False, False, cfg=cfg)
        torch.testing.assert_close(out, B.float().t())


@pytest.mark.parametrize("K", [64, 128, 704, 832])
@pytest.mark.parametrize("a_mn,b_mn", [(0, 0), (1, 1)])
def test_pingpong_odd_and_short_k(dev, K, a_mn, b_mn):
    """Config 5 (ping-pong, 2 K-tiles per iteration): odd K-tile counts, 1-2 K-tiles, tails."""
    C = require_native()
    M, N = 296, 520
    g = torch.Generator().manual_seed(K + a_mn)
    A = _mk((K, M) if a_mn else (M, K), dev, g)
    B = _mk((K, N) if b_mn else (N, K), dev, g)
    out = torch.empty(M, N, device=dev)
    C.gemm(A, B, out, bool(a_mn), bool(b_mn), cfg=5)
    torch.testing.assert_close(out, _ref(A, B, a_mn, b_mn), rtol=2e-3, atol=2e-2)


@pytest.mark.parametrize("a_mn,b_mn", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_pingpong_matches_tile_kernel_bitwise(dev, a_mn, b_mn):
    """Race screen: the ping-pong schedule (DMAs in flight across barriers, staggered wave
    groups) must give bit-identical fp32 results to the 2-phase 256x256 kernel, which
    accumulates the same products in the same order -- repeated, on a full-chip grid."""
    C = require_native()
    M = N = 2048
    K = 2048
    g = torch.Generator().manual_seed(11 + 2 * a_mn + b_mn)
    A = _mk((K, M) if a_mn else (M, K), dev, g)
    B = _mk((K, N) if b_mn else (N, K), dev, g)
    ref = torch.empty(M, N, device=dev)
    C.gemm(A, B, ref, bool(a_mn), bool(b_mn), cfg=1)
    out = torch.empty(M, N, device=dev)
    for _ in range(10):
        out.fill_(float("nan"))
        C.gemm(A, B, out, bool(a_mn), bool(b_mn), cfg=5)
        assert torch.equal(out, ref)


@pytest.mark.parametrize("cfg", [1, 4, 5])
def test_split_k_external_reduce_bitwise(dev, cfg):
    """External split-K combine (row-major partials + grid-wide reduce launch) sums the slabs in
    the same split order as the in-kernel last arriver: identical bits, every epilogue."""
    C = require_native()
    M, N, K = 768, 520, 4096
    g = torch.Generator().manual_seed(cfg)
    A = _mk((K, M), dev, g)
    B = _mk((K, N), dev, g)
    bias = torch.randn(N, device=dev)
    res = _mk((M, N), dev, g)
    outs = {}
    try:
        for mode in (0, 1):
            C.set_gemm_split_mode(mode)
            assert C.gemm_plan(True, True, M, N, K, cfg, 6)[4] == mode
            o32 = torch.full((M, N), 0.25, device=dev)
            C.gemm(A, B, o32, True, True, accumulate=True, cfg=cfg, splits=6)
            o16 = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            C.gemm(A, B, o16, True, True, bias=bias, aux=aux, mode=1, cfg=cfg, splits=6)
            o16r = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            C.gemm(A, B, o16r, True, True, res=res, alpha=0.5, cfg=cfg, splits=6)
            outs[mode] = (o32, o16, aux, o16r)
    finally:
        C.set_gemm_split_mode(-1)
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    torch.testing.assert_close(outs[1][0], A.float().t() @ B.float() + 0.25, rtol=2e-3, atol=2e-2)


@pytest.mark.parametrize("b_mn", [0, 1])
def test_persistent_kernel(dev, b_mn):
    """Config 6 (persistent tile loop, next tile's first K-step staged under the current tile's
    last MFMAs, register epilogue from swapped-operand C^T fragments): more tiles than CUs (every
    workgroup walks several), M / N tails, a strided A, every epilogue, bf16 and fp32 outputs."""
    C = require_native()
    M, N, K = 8200, 2312, 256  # 33 x 10 = 330 tiles > 256 workgroups; tails in M and N; 4 K-tiles
    g = torch.Generator().manual_seed(50 + b_mn)
    A = _mk((M, K + 64), dev, g)[:, :K]
    B = _mk((K, N) if b_mn else (N, K), dev, g)
    ref = _ref(A, B, 0, b_mn)
    assert C.gemm_plan(False, bool(b_mn), M, N, K, 6, 0)[0] == 6
    for out_dtype in (torch.bfloat16, torch.float32):
        out = torch.empty(M, N, dtype=out_dtype, device=dev)
        C.gemm(A, B, out, False, bool(b_mn), cfg=6)
        tol = 2e-2 if out_dtype == torch.bfloat16 else 2e-3
        torch.testing.assert_close(out.float(), ref, rtol=tol, atol=tol * 8)
    bias = torch.randn(N, device=dev)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    C.gemm(A, B, out, False, bool(b_mn), bias=bias, aux=aux, mode=1, cfg=6)
    torch.testing.assert_close(aux.float(), ref + bias, rtol=2e-2, atol=0.15)
    torch.testing.assert_close(out.float(), torch.nn.functional.gelu(aux.float()), rtol=2e-2, atol=0.15)
    res = _mk((M, N), dev, g)
    C.gemm(A, B, out, False, bool(b_mn), res=res, alpha=0.5, cfg=6)
    torch.testing.assert_close(out.float(), 0.5 * ref + res.float(), rtol=2e-2, atol=0.15)
    acc = torch.ones(M, N, device=dev)
    C.gemm(A, B, acc, False, bool(b_mn), accumulate=True, cfg=6)
    torch.testing.assert_close(acc, ref + 1, rtol=2e-3, atol=2e-2)
    pre = _mk((M, N), dev, g)
    C.gemm(A, B, out, False, bool(b_mn), aux=pre, mode=2, cfg=6)
    x = pre.float()
    dg = 0.5 * (1 + torch.erf(x * 0.7071067811865476)) + x * torch.exp(-0.5 * x * x) * 0.3989422804014327
    torch.testing.assert_close(out.float(), ref * dg, rtol=2e-2, atol=0.15)


def test_persistent_kernel_repeatable_full_chip(dev):
    """Race screen for the cross-tile pipeline: repeated full-chip runs are bit-identical, and
    agree with the one-tile-per-workgroup kernel to fp32 rounding."""
    C = require_native()
    M, N, K = 8192, 2304, 768
    g = torch.Generator().manual_seed(77)
    A = _mk((M, K), dev, g)
    B = _mk((N, K), dev, g)
    ref = torch.empty(M, N, device=dev)
    C.gemm(A, B, ref, False, False, cfg=1)
    first = None
    for _ in range(6):
        out = torch.full((M, N), float("nan"), device=dev)
        C.gemm(A, B, out, False, False, cfg=6)
        if first is None:
            first = out.clone()
        assert torch.equal(out, first)
    torch.testing.assert_close(first, ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("b_mn", [0, 1])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 320), (1024, 512, 768),
                                   (16384, 3072, 768)])  # the last: the 4-wave kernel's epilogue (cfg 7)
def test_dgelu_colsum_fused(dev, b_mn, M, N, K):
    """dGELU epilogue with fused column sums (the bias gradient of the layer before the GELU):
    output and sums vs fp32 torch; set and accumulate modes."""
    C = require_native()
    g = torch.Generator().manual_seed(M + N + K + b_mn)
    A = _mk((M, K), dev, g)
    B = _mk((K, N) if b_mn else (N, K), dev, g)
    aux = (torch.randn(M, N, generator=g) * 2).to(torch.bfloat16).to(dev)
    x = aux.float().requires_grad_(True)
    torch.nn.functional.gelu(x).backward(torch.ones_like(x))
    ref = _ref(A, B, 0, b_mn) * x.grad
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    cs = torch.full((N,), 3.0, device=dev)
    C.gemm(A, B, out, False, bool(b_mn), aux=aux, mode=2, colsum_out=cs)
    torch.testing.assert_close(out.float(), ref, rtol=3e-2, atol=5e-2)
    scale = ref.abs().sum(0).max().item()
    torch.testing.assert_close(cs, ref.sum(0), rtol=1e-3, atol=1e-4 * scale)
    C.gemm(A, B, out, False, bool(b_mn), aux=aux, mode=2, colsum_out=cs, colsum_accumulate=True)
    torch.testing.assert_close(cs, 2 * ref.sum(0), rtol=1e-3, atol=2e-4 * scale)
    with pytest.raises(RuntimeError):  # edge tiles cannot fuse the sums
        C.gemm(A[:M - 8], B, out[:M - 8], False, bool(b_mn), aux=aux[:M - 8], mode=2, colsum_out=cs)


@pytest.mark.parametrize("b_mn", [0, 1])
def test_w4_asm_kernel(dev, b_mn):
    """Config 7 (4-wave 256x256x64 tile, generated-asm main loop, AGPR accumulators, LDS-staged
    epilogue; B k-contiguous or n-contiguous through transposed LDS reads): every epilogue, bf16 and
    fp32 outputs, a strided A (and B), more tiles than CUs; a shape outside its domain (N tail) falls
    back to the ping-pong kernel."""
    C = require_native()
    M, N, K = 4096, 2304, 768  # 16 x 9 = 144 tiles, 6 K-tile pairs
    g = torch.Generator().manual_seed(71 + b_mn)
    A = _mk((M, K + 64), dev, g)[:, :K]
    B = _mk((K, N + 128), dev, g)[:, :N] if b_mn else _mk((N, K), dev, g)
    ref = _ref(A, B, 0, b_mn)
    assert C.gemm_plan(False, bool(b_mn), 65536, N, K)[0] == 7  # planner: tiles fill the chip
    assert C.gemm_plan(False, bool(b_mn), 1024, 1024, 65536)[0] != 7  # few tiles, long K: split-K
    for out_dtype in (torch.bfloat16, torch.float32):
        out = torch.empty(M, N, dtype=out_dtype, device=dev)
        C.gemm(A, B, out, False, bool(b_mn), cfg=7)
        tol = 2e-2 if out_dtype == torch.bfloat16 else 2e-3
        torch.testing.assert_close(out.float(), ref, rtol=tol, atol=tol * 8)
    bias = torch.randn(N, device=dev)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    C.gemm(A, B, out, False, bool(b_mn), bias=bias, aux=aux, mode=1, cfg=7)
    torch.testing.assert_close(aux.float(), ref + bias, rtol=2e-2, atol=0.15)
    torch.testing.assert_close(out.float(), torch.nn.functional.gelu(aux.float()), rtol=2e-2, atol=0.15)
    res = _mk((M, N), dev, g)
    C.gemm(A, B, out, False, bool(b_mn), res=res, alpha=0.5, cfg=7)
    torch.testing.assert_close(out.float(), 0.5 * ref + res.float(), rtol=2e-2, atol=0.15)
    pre = _mk((M, N), dev, g)
    C.gemm(A, B, out, False, bool(b_mn), aux=pre, mode=2, cfg=7)
    x = pre.float()
    dg = 0.5 * (1 + torch.erf(x * 0.7071067811865476)) + x * torch.exp(-0.5 * x * x) * 0.3989422804014327
    torch.testing.assert_close(out.float(), ref * dg, rtol=2e-2, atol=0.15)
    # outside the 256-multiple domain -> the ping-pong fallback, same numbers
    Bt = B[:, : N - 40] if b_mn else B[: N - 40]
    out = torch.empty(M, N - 40, dtype=torch.float32, device=dev)
    C.gemm(A, Bt, out, False, bool(b_mn), cfg=7)
    torch.testing.assert_close(out, ref[:, : N - 40], rtol=2e-3, atol=2e-2)


@pytest.mark.parametrize("b_mn", [0, 1])
def test_w4_asm_kernel_repeatable_full_chip(dev, b_mn):
    """Repeated full-chip runs of config 7 are bit-identical and agree with config 1 to fp32 rounding
    (K = 3072: 24 K-tiles through both LDS stages many times)."""
    C = require_native()
    M, N, K = 8192, 2304, 3072
    g = torch.Generator().manual_seed(78 + b_mn)
    A = _mk((M, K), dev, g)
    B = _mk((K, N) if b_mn else (N, K), dev, g)
    ref = torch.empty(M, N, device=dev)
    C.gemm(A, B, ref, False, bool(b_mn), cfg=1)
    first = None
    for _ in range(4):
        out = torch.full((M, N), float("nan"), device=dev)
        C.gemm(A, B, out, False, bool(b_mn), cfg=7)
        if first is None:
            first = out.clone()
        assert torch.equal(out, first)
    torch.testing.assert_close(first, ref, rtol=1e-4, atol=1e-3)


def test_w4_asm_wgrad_split_k(dev):
    """Config 7 in the weight-gradient layout (A [K][M], B [K][N], both through transposed LDS reads)
    with split-K raw partials + the external reduce (the planner's pick for few-tile long-K shapes),
    fp32 accumulate and bf16 + bias outputs; a forced single split runs the epilogue in-kernel."""
    C = require_native()
    M, N, K = 768, 2304, 16384
    g = torch.Generator().manual_seed(90)
    A = _mk((K, M), dev, g)
    B = _mk((K, N), dev, g)
    ref = A.float().t() @ B.float()
    plan = C.gemm_plan(True, True, M, N, K)
    assert plan[0] == 7 and plan[1] > 1 and plan[4] == 1, plan
    acc = torch.full((M, N), 0.25, device=dev)
    C.gemm(A, B, acc, True, True, accumulate=True)
    torch.testing.assert_close(acc, ref + 0.25, rtol=1e-4, atol=2e-3)
    bias = torch.randn(N, device=dev)
    o16 = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    C.gemm(A, B, o16, True, True, bias=bias)
    torch.testing.assert_close(o16.float(), ref + bias, rtol=2e-2, atol=0.2)
    one = torch.empty(M, N, device=dev)
    C.gemm(A, B, one, True, True, cfg=7)
    torch.testing.assert_close(one, ref, rtol=1e-4, atol=2e-3)
    ref1 = torch.empty(M, N, device=dev)
    C.gemm(A, B, ref1, True, True, cfg=1)
    torch.testing.assert_close(acc - 0.25, ref1, rtol=1e-5, atol=1e-3)


def test_w4_wgrad_accumulate_plan(dev):
    """An ACCUMULATING weight gradient (A [K][M], B [K][N]) on a shape the 4-wave kernel would take
    with a single split: that kernel's in-kernel epilogue cannot accumulate, so the planner (told
    `accumulate`) picks the fitted split-K tile plan instead of handing the launch a cfg-7 plan; the
    result is C + A^T B against fp32 torch. Multi-split cfg-7 plans keep accumulating in their reduce."""
    C = require_native()
    M, N, K = 2048, 2048, 512
    assert C.gemm_plan(True, True, M, N, K)[:2] == (7, 1)
    plan = C.gemm_plan(True, True, M, N, K, accumulate=True)
    assert plan[0] != 7, plan
    g = torch.Generator().manual_seed(91)
    A = _mk((K, M), dev, g)
    B = _mk((K, N), dev, g)
    ref = A.float().t() @ B.float()
    acc = torch.full((M, N), -0.5, device=dev)
    C.gemm(A, B, acc, True, True, accumulate=True)
    torch.testing.assert_close(acc, ref - 0.5, rtol=1e-4, atol=2e-3)
    M2, N2, K2 = 768, 3072, 4096  # cfg 7 with split-K partials: accumulates in the external reduce
    assert C.gemm_plan(True, True, M2, N2, K2, accumulate=True)[:2][0] == 7
    A2 = _mk((K2, M2), dev, g)
    B2 = _mk((K2, N2), dev, g)
    acc2 = torch.full((M2, N2), 1.5, device=dev)
    C.gemm(A2, B2, acc2, True, True, accumulate=True)
    torch.testing.assert_close(acc2, A2.float().t() @ B2.float() + 1.5, rtol=1e-4, atol=4e-3)


@pytest.mark.parametrize("mode", [1, 2])
def test_gelu_epilogues_same_bits_on_every_kernel(dev, mode):
    """Every GEMM kernel's GELU (mode 1) / dGELU (mode 2) epilogue multiplies by the same exact table
    entry (csrc/include/mlt_gelu_table.inc; LDS copy in the 4-wave kernel, global memory elsewhere):
    with operands whose products and sums are exact in fp32 (so every kernel reaches the same
    pre-activation whatever its accumulation order), the 4-wave, ping-pong, tile, persistent and
    general kernels and the split-K reduce all write identical bits, which also match torch's erf
    GELU within bf16 rounding."""
    C = require_native()
    M, N, K = 4096, 2304, 256
    g = torch.Generator().manual_seed(5 + mode)
    # entries in {-1, 0, 1} / 4: every partial sum is a multiple of 1/16 below 16 -> exact in fp32
    A = (torch.randint(-1, 2, (M, K), generator=g).float() / 4).to(torch.bfloat16).to(dev)
    B = (torch.randint(-1, 2, (N, K), generator=g).float() / 4).to(torch.bfloat16).to(dev)
    bias = (torch.randn(N, generator=g) * 2).to(dev)
    pre = (torch.randn(M, N, generator=g) * 2).to(torch.bfloat16).to(dev)
    outs = {}
    for cfg, splits in ((7, 0), (5, 0), (1, 0), (6, 0), (0, 0), (1, 2)):
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        if mode == 1:
            aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            C.gemm(A, B, out, False, False, bias=bias, aux=aux, mode=1, cfg=cfg, splits=splits)
            outs[(cfg, splits)] = (out, aux)
        else:
            C.gemm(A, B, out, False, False, aux=pre, mode=2, cfg=cfg, splits=splits)
            outs[(cfg, splits)] = (out, pre)
    ref_out, ref_aux = outs[(7, 0)]
    for key, (out, aux) in outs.items():
        assert torch.equal(aux, ref_aux), key
        assert torch.equal(out, ref_out), key
    x = ref_aux.float()
    acc = A.float() @ B.float().t()
    if mode == 1:
        torch.testing.assert_close(x, acc + bias, rtol=1e-2, atol=1e-2)
        torch.testing.assert_close(ref_out.float(), torch.nn.functional.gelu(x.double()).float(), rtol=8e-3, atol=1e-6)
    else:
        xd = x.double()
        dg = 0.5 * torch.erfc(-xd / math.sqrt(2.0)) + xd * torch.exp(-0.5 * xd * xd) / math.sqrt(2.0 * math.pi)
        torch.testing.assert_close(ref_out.float(), (acc.double() * dg).float(), rtol=8e-3, atol=1e-6)
