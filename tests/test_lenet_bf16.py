"""bf16 MFMA LeNet engine (csrc/kernels/lenet_mfma.hip; BASELINE.json configs 2/3 "default config
bf16") vs a plain-torch reference that rounds to bf16 at exactly the kernel's MFMA operands
(ml_trainer_amd/models/lenet_bf16_ref.py), plus the engine invariants: graph == eager, staged
next-step inputs == gathered inputs (bitwise), the data-parallel (REDUCE) step == the fused step."""
import copy

import pytest
import torch
import torch.nn.functional as F

from ml_trainer_amd.models.lenet import MLModel
from ml_trainer_amd.models.lenet_bf16_ref import lenet_bf16_grads


def _mk(config="default", seed=0):
    torch.manual_seed(seed)
    return MLModel(config)


# ----------------------------------------------------------------------------- CPU: the reference
@pytest.mark.parametrize("config", ["default", "tiny"])
def test_reference_without_rounding_is_autograd(config):
    """With identity rounding the hand-written backward of the reference IS the fp32 model's
    autograd backward (pins unpool / transposed-conv / wgrad index math without a GPU)."""
    m = _mk(config, 1).double()
    x = torch.randn(6, 3, 32, 32, dtype=torch.float64)
    y = torch.randint(0, 10, (6,))
    loss = F.cross_entropy(m.forward_reference(x), y)
    loss.backward()
    l2, _, g = lenet_bf16_grads(dict(m.named_parameters()), x, y, rnd=lambda t: t)
    assert abs(l2 - loss.item()) < 1e-12
    for n, p in m.named_parameters():
        torch.testing.assert_close(g[n], p.grad, rtol=1e-9, atol=1e-12, msg=lambda s: f"{n}: {s}")


def _cos(a, b):
    a, b = a.double().cpu().flatten(), b.double().cpu().flatten()
    return (a @ b / (a.norm() * b.norm()).clamp_min(1e-30)).item()


def test_reference_bf16_close_to_fp32():
    """bf16 operands flip a few ReLU / max-pool decisions near their thresholds (random init, a
    small batch), so bf16 and fp32 gradients differ by a few percent in norm but point the same
    way."""
    m = _mk("default", 2)
    x = torch.randn(32, 3, 32, 32)
    y = torch.randint(0, 10, (32,))
    _, _, g32 = lenet_bf16_grads(dict(m.named_parameters()), x, y, rnd=lambda t: t)
    _, _, g16 = lenet_bf16_grads(dict(m.named_parameters()), x, y)
    for n in g32:
        assert _cos(g16[n], g32[n]) > 0.97, (n, _cos(g16[n], g32[n]))


# ----------------------------------------------------------------------------- GPU: the kernels
def _engine(m, opt="sgd", max_batch=32, lr=1e-2, precision="bf16", wd=0.0):
    from ml_trainer_amd.models.lenet_engine import LeNetStepEngine
    from ml_trainer_amd.ops.optim import build_optimizer
    from ml_trainer_amd.utils.flat import FlatParams
    flat = FlatParams(m.parameters())
    o = build_optimizer(opt, m.parameters(), lr=lr, momentum=0.9, weight_decay=wd, flat=flat)
    return LeNetStepEngine(m, flat, max_batch=max_batch, optimizer=o, precision=precision), flat


def _rel(a, b):
    return ((a.double().cpu() - b.double().cpu()).norm() / b.double().cpu().norm().clamp_min(1e-30)).item()


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["default", "tiny"])
@pytest.mark.parametrize("B", [1, 5, 32, 64])
def test_bf16_step_grads_match_reference(dev, config, B):
    m = _mk(config, 3).to(dev)
    p0 = {n: p.detach().clone() for n, p in m.named_parameters()}
    eng, flat = _engine(m, max_batch=max(B, 8))
    x = torch.randn(B, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (B,), device=dev)
    eng.reset_stats()
    eng.step_from_tensors(x, y, train=True)
    loss, acc = eng.read_stats(1)
    rl, racc, g = lenet_bf16_grads(p0, x, y)
    assert abs(loss - rl) < 2e-4 * max(1.0, rl), (loss, rl)
    assert abs(acc - racc) < 1e-9, (acc, racc)
    for n, p in m.named_parameters():
        o, k = flat.segment(p)
        gk = flat.grad[o:o + k].view_as(p)
        assert torch.isfinite(gk).all(), n
        assert _rel(gk, g[n]) < 1e-2, (n, _rel(gk, g[n]))
        # SGD first step (momentum buffer = g): p1 = p0 - lr * g with the kernel's own gradient
        torch.testing.assert_close(p.detach(), p0[n] - 1e-2 * gk, rtol=1e-6, atol=1e-7, msg=lambda s: f"{n}: {s}")


@pytest.mark.gpu
def test_bf16_step_close_to_fp32_autograd(dev):
    m = _mk("default", 4).to(dev)
    ref = copy.deepcopy(m)
    eng, flat = _engine(m)
    x = torch.randn(32, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (32,), device=dev)
    eng.step_from_tensors(x, y, train=True)
    F.cross_entropy(ref.forward_reference(x), y).backward()
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        o, k = flat.segment(p)
        assert _cos(flat.grad[o:o + k].view_as(q), q.grad) > 0.97, n


@pytest.mark.gpu
@pytest.mark.parametrize("opt", ["adam", "adamw", "adagrad", "adamax"])
def test_bf16_engine_optimizers(dev, opt):
    """The fused update of KW (every optimizer) == torch.optim applied to the kernel's gradient."""
    m = _mk("default", 5).to(dev)
    ref = copy.deepcopy(m)
    eng, flat = _engine(m, opt, lr=1e-3, wd=1e-3)
    ro = {"adam": torch.optim.Adam, "adamw": torch.optim.AdamW, "adagrad": torch.optim.Adagrad,
          "adamax": torch.optim.Adamax}[opt](ref.parameters(), lr=1e-3, weight_decay=1e-3)
    for i in range(3):
        x = torch.randn(16, 3, 32, 32, device=dev)
        y = torch.randint(0, 10, (16,), device=dev)
        eng.step_from_tensors(x, y, train=True)
        for p, q in zip(m.parameters(), ref.parameters()):
            o, k = flat.segment(p)
            q.grad = flat.grad[o:o + k].view_as(q).clone()
        ro.step()
        for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
            torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-5, atol=1e-6, msg=lambda s: f"{n} {i}: {s}")


def _toy_data(N, seed=0):
    g = torch.Generator().manual_seed(seed)
    targets = torch.randint(0, 10, (N,), generator=g)
    base = (targets.view(N, 1, 1, 1).float() * 25).expand(N, 32, 32, 3)
    data = (base + torch.randint(0, 30, (N, 32, 32, 3), generator=g).float()).clamp(0, 255).to(torch.uint8)
    return data, targets


@pytest.mark.gpu
def test_bf16_graph_equals_eager_bitwise(dev):
    data, targets = _toy_data(512)
    runs = []
    for use_graph in (False, True):
        m = _mk("default", 6).to(dev)
        eng, flat = _engine(m, "adam", max_batch=64, lr=1e-3)
        eng.set_dataset(data, targets, batch_size=64)
        eng.start_epoch(torch.arange(512))
        eng.train_steps(64, 8, use_graph=use_graph, steps_per_graph=4)
        torch.cuda.synchronize()
        runs.append((flat.data.clone(), eng.stats.clone(), eng.ctrl.clone()))
    assert torch.equal(runs[0][0], runs[1][0])
    assert torch.equal(runs[0][1], runs[1][1])
    assert runs[1][2].tolist() == [8, 8]


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_bf16_prewarm_is_a_bitwise_noop(dev, precision):
    """engine.prewarm launches the graphs of the next steps once and restores every tensor they
    wrote: all engine buffers, weights, gradients, optimizer state and counters are bitwise what
    they were, and training after it == training without it, bit for bit (adam: state + step)."""
    data, targets = _toy_data(300, 5)
    runs = []
    for pre in (False, True):
        m = _mk("default", 4).to(dev)
        eng, flat = _engine(m, "adam", max_batch=32, lr=1e-3, precision=precision)
        eng.set_dataset(data, targets, batch_size=32)
        eng.start_epoch(torch.randperm(300, generator=torch.Generator().manual_seed(3)))
        eng.train_steps(32, 2, use_graph=True, steps_per_graph=2)
        if pre:
            torch.cuda.synchronize()
            state = eng._state_tensors()
            assert any(t.data_ptr() == flat.data.data_ptr() for t in state)
            assert len([t for t in state if t.dtype == torch.float32]) >= 4  # (+ adam's two moments)
            before = [t.clone() for t in state]
            assert eng.can_prewarm()
            assert eng.prewarm(32, 6, steps_per_graph=3) == 1
            torch.cuda.synchronize()
            for i, (a, b) in enumerate(zip(state, before)):  # bitwise (scratch may hold NaN patterns)
                assert torch.equal(a.reshape(-1).view(torch.uint8), b.reshape(-1).view(torch.uint8)), i
        eng.train_steps(32, 6, use_graph=True, steps_per_graph=3)
        torch.cuda.synchronize()
        runs.append((flat.data.clone(), eng.stats.clone(), eng.ctrl.clone()))
    assert torch.equal(runs[0][0], runs[1][0])
    assert torch.equal(runs[0][1], runs[1][1])
    assert runs[1][2].tolist() == [8, 8]


@pytest.mark.gpu
def test_bf16_staging_bitwise(dev):
    """The batch-reduction kernel's prep blocks augment the next step's inputs (pixels + tags);
    a step uses them only on a tag match. Training with prepared inputs (graphs, two epochs, a
    partial last batch) == training with every tag invalidated before each step (the per-sample
    kernel then gathers and augments itself), bit for bit."""
    data, targets = _toy_data(300, 7)
    runs = []
    for staged in (True, False):
        m = _mk("default", 8).to(dev)
        eng, flat = _engine(m, "sgd", max_batch=32, lr=1e-2)
        eng.set_dataset(data, targets, batch_size=32)
        for ep in range(2):
            perm = torch.randperm(300, generator=torch.Generator().manual_seed(10 + ep))
            eng.start_epoch(perm)
            if staged:
                eng.train_steps(32, 9, use_graph=True, steps_per_graph=3)
                torch.cuda.synchronize()
                meta = eng.bufs["pmeta"].view(-1, 4)[:12].cpu()
                # the 9th step's (in-epoch index 8) batch-reduction kernel prepared in-epoch step 9
                # (positions 288 + b): global step, position, target
                assert meta[:, 0].tolist() == [ep * 10 + 9] * 12, meta
                assert meta[:, 1].tolist() == list(range(288, 300)), meta
                assert meta[:, 2].tolist() == targets[perm[288:]].tolist()
                # ... from the raw images the 9th step's per-sample kernel staged for them (meta2:
                # step, position, dataset row, target)
                m2 = eng.bufs["meta2"].view(-1, 4)[:12].cpu()
                assert m2[:, 0].tolist() == [ep * 10 + 9] * 12, m2
                assert m2[:, 2].tolist() == perm[288:].tolist(), m2
                assert m2[:, 3].tolist() == targets[perm[288:]].tolist(), m2
            else:
                for _ in range(9):
                    eng._reset_staging()
                    eng.train_steps(32, 1, use_graph=False)
                eng._reset_staging()
            eng.train_steps(300 - 9 * 32, 1, use_graph=staged, steps_per_graph=1)  # partial batch of 12
        torch.cuda.synchronize()
        runs.append((flat.data.clone(), eng.stats.clone()))
    assert torch.equal(runs[0][0], runs[1][0])
    assert torch.equal(runs[0][1], runs[1][1])


@pytest.mark.gpu
def test_bf16_aug_path_matches_reference(dev):
    """HBM dataset + on-GPU augmentation through the bf16 step == CPU-augmented batches through
    the bf16 reference (first step: exact inputs; gradients within accumulation noise)."""
    from tests.test_lenet_native import _cpu_augment
    data, targets = _toy_data(64, 3)
    m = _mk("default", 9).to(dev)
    p0 = {n: p.detach().clone() for n, p in m.named_parameters()}
    eng, flat = _engine(m, "sgd")
    eng.set_dataset(data, targets, batch_size=32)
    perm = torch.randperm(64, generator=torch.Generator().manual_seed(2))
    eng.start_epoch(perm)
    eng.train_steps(32, 1, use_graph=False)
    mean, std = [0.4914, 0.4822, 0.4465], [0.2023, 0.1994, 0.2010]
    x = _cpu_augment(data, perm.to(torch.int32), 0, 0, 32, eng.seed, 4, True, mean, std)
    y = targets[perm[:32]]
    _, _, g = lenet_bf16_grads(p0, x, y)
    for n, p in m.named_parameters():
        o, k = flat.segment(p)
        assert _rel(flat.grad[o:o + k].view_as(p), g[n]) < 1e-2, n


@pytest.mark.gpu
def test_bf16_graph_training_converges(dev):
    data, targets = _toy_data(2048, 11)
    m = _mk("default", 12).to(dev)
    # lr 1e-2 as the fp32 test (5e-2 is unstable on this toy set)
    eng, flat = _engine(m, "sgd", max_batch=64, lr=1e-2)
    eng.set_dataset(data, targets, batch_size=64)
    losses = []
    for ep in range(4):
        eng.start_epoch(torch.randperm(2048, generator=torch.Generator().manual_seed(ep)))
        eng.reset_stats()
        eng.train_steps(64, 32, use_graph=True, steps_per_graph=16)
        losses.append(eng.read_stats(32)[0])
    assert all(torch.isfinite(torch.tensor(losses))), losses
    assert losses[-1] < 0.6 * losses[0], losses


@pytest.mark.gpu
@pytest.mark.parametrize("opt", ["sgd", "adamw"])
def test_bf16_reduce_mode_matches_fused(dev, opt):
    """The data-parallel step (KS -> KW without the update -> RCCL all-reduce over one rank ->
    flat optimizer -> shadow / fragment-image repack) == the fused single-rank step, bitwise."""
    C = pytest.importorskip("ml_trainer_amd.ops._ext").require_native()
    data, targets = _toy_data(256, 5)
    runs = []
    for dp in (False, True):
        m = _mk("default", 13).to(dev)
        eng, flat = _engine(m, opt, max_batch=32, lr=1e-3)
        if dp:
            eng.use_transport(comm=C.Communicator(C.Communicator.unique_id(), 1, 0, dev.index))
        eng.set_dataset(data, targets, batch_size=32)
        eng.start_epoch(torch.arange(256))
        eng.train_steps(32, 6, use_graph=True, steps_per_graph=3)
        torch.cuda.synchronize()
        runs.append(flat.data.clone())
    assert torch.equal(runs[0], runs[1])


@pytest.mark.gpu
def test_bf16_eval_uses_fp32_forward(dev):
    """Evaluation on a bf16 engine runs the fp32 forward on the fp32 masters."""
    m = _mk("default", 14).to(dev)
    eng, flat = _engine(m)
    x = torch.randn(16, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (16,), device=dev)
    eng.reset_stats()
    eng.step_from_tensors(x, y, train=False)
    loss, _ = eng.read_stats(1)
    ref = F.cross_entropy(m.forward_reference(x), y).item()
    assert abs(loss - ref) < 1e-4 * max(1.0, ref)


@pytest.mark.gpu
def test_bf16_host_change_of_masters_is_packed(dev):
    """A host-side in-place change of the fp32 masters between replays reaches the bf16 shadow /
    fragment images (one pack ahead of the next replay, keyed on the flat buffer's version): the
    graph path then matches the eager path (which packs before every step) bitwise."""
    data, targets = _toy_data(256, 13)
    runs = []
    for use_graph in (True, False):
        m = _mk("default", 21).to(dev)
        eng, flat = _engine(m, "sgd", max_batch=32, lr=1e-2)
        eng.set_dataset(data, targets, batch_size=32)
        eng.start_epoch(torch.arange(256))
        eng.train_steps(32, 2, use_graph=True, steps_per_graph=2)
        with torch.no_grad():
            m.fc1.weight.mul_(0.5)
            m.conv1.weight.mul_(-1.0)
            m.conv2.weight.add_(0.01)
        eng.train_steps(32, 2, use_graph=use_graph, steps_per_graph=2)
        torch.cuda.synchronize()
        runs.append(flat.data.clone())
    assert torch.equal(runs[0], runs[1])


@pytest.mark.gpu
@pytest.mark.parametrize("opt", ["sgd", "adamw"])
def test_bf16_fused_dp_loopback_matches_fused(dev, opt):
    """The two-launch data-parallel step (lenet_mwx: batch reductions -> publish granules into the
    xGMI region -> poll -> rank-ordered sum -> update, one launch) against the loopback transport
    (the only peer is this rank) == the fused single-rank step, bitwise; and the graph holds two
    kernels per step."""
    from ml_trainer_amd.parallel.comm import create_xgmi_loopback
    data, targets = _toy_data(256, 5)
    runs = []
    for dp in (False, True):
        m = _mk("default", 13).to(dev)
        eng, flat = _engine(m, opt, max_batch=32, lr=1e-3)
        if dp:
            x = create_xgmi_loopback(flat.numel, dev)
            eng.use_transport(xgmi=x)
            assert eng.dp_transport == "xgmi-fused" and eng.in_graph_collective
        eng.set_dataset(data, targets, batch_size=32)
        eng.start_epoch(torch.arange(256))
        eng.train_steps(32, 6, use_graph=True, steps_per_graph=3)
        eng.check_transport()
        torch.cuda.synchronize()
        if dp:
            assert x.error() == 0
            assert eng.eng.graph_nodes(eng._train_mode(), 32, 3) == 6  # 2 kernels x 3 steps
        runs.append((flat.data.clone(), flat.grad.clone(), eng.stats.clone(), eng.ctrl.clone()))
    for a, b in zip(runs[0], runs[1]):
        assert torch.equal(a, b)


@pytest.mark.gpu
def test_bf16_fused_dp_loopback_fault_raises(dev):
    """Fault injection on the loopback transport: the withheld blocks time out, the sticky error
    word makes the host raise TransportError, and every later launch publishes and applies nothing."""
    from ml_trainer_amd.models.lenet_engine import TransportError
    from ml_trainer_amd.parallel.comm import create_xgmi_loopback
    data, targets = _toy_data(256, 5)
    m = _mk("default", 13).to(dev)
    eng, flat = _engine(m, "sgd", max_batch=32, lr=1e-3)
    x = create_xgmi_loopback(flat.numel, dev, timeout_ms=200)
    eng.use_transport(xgmi=x)
    eng.set_dataset(data, targets, batch_size=32)
    eng.start_epoch(torch.arange(256))
    eng.train_steps(32, 2, use_graph=True, steps_per_graph=1)
    eng.check_transport()
    x.fault = 1
    eng.use_transport(xgmi=x)  # recapture with the fault live
    with pytest.raises(TransportError):
        eng.train_steps(32, 1, use_graph=True, steps_per_graph=1)
        eng.check_transport()
    torch.cuda.synchronize()
    before = flat.data.clone()
    with pytest.raises(TransportError):  # sticky: nothing is applied any more
        eng.train_steps(32, 2, use_graph=True, steps_per_graph=1)
    torch.cuda.synchronize()
    assert torch.equal(flat.data, before)


def _quality_run(precision, model_dir, epochs=6, n_train=8192):
    from ml_trainer_amd.data.cifar10 import SyntheticCIFAR10
    from ml_trainer_amd.data.transforms import Compose, Normalize, RandomCrop, RandomHorizontalFlip, ToTensor
    from ml_trainer_amd.trainer import Trainer
    norm = Normalize((0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010))
    tr = SyntheticCIFAR10(n_train, True, transform=Compose([RandomCrop(32, padding=4), RandomHorizontalFlip(),
                                                             ToTensor(), norm]), seed=3, learnable="pattern")
    va = SyntheticCIFAR10(2048, False, transform=Compose([ToTensor(), norm]), seed=3, learnable="pattern")
    torch.manual_seed(5)
    t = Trainer(MLModel(), datasets=(tr, va), epochs=epochs, batch_size=32, metric="accuracy", lr=1e-2,
                model_dir=str(model_dir), options={"progress": False, "use_engine": True, "precision": precision})
    t.fit()
    return t.history


@pytest.mark.gpu
def test_bf16_training_quality_matches_fp32(tmp_path):
    """Training quality of the bf16 headline step (BASELINE configs 2/3) against the reference
    dtype over epochs (the reference's only quality evidence is its accuracy trajectory,
    01_ML_Training_local.ipynb:309-409): Trainer.fit() for 6 epochs on a dataset whose accuracy
    climbs gradually (class colour templates under heavy noise, RandomCrop + HFlip), fp32 vs bf16
    engine, same init and data order. Final val accuracy within 1.5 points; per-epoch train loss
    within 5 % or 0.05 nats (the two trajectories separate chaotically once the loss is small:
    measured 0.251 vs 0.281 at epoch 6 with val accuracy 96.8 % vs 97.0 %,
    profiles/r4/lenet_bf16_vs_fp32_quality.jsonl)."""
    h = {p: _quality_run(p, tmp_path / p) for p in ("fp32", "bf16")}
    a32, a16 = h["fp32"]["val_metric"], h["bf16"]["val_metric"]
    assert a32[-1] > 0.5, a32  # it learned something non-trivial
    assert abs(a32[-1] - a16[-1]) <= 0.015, (a32, a16)
    for e, (l32, l16) in enumerate(zip(h["fp32"]["train_loss"], h["bf16"]["train_loss"])):
        assert abs(l32 - l16) <= max(0.05 * l32, 0.05), (e, h["fp32"]["train_loss"], h["bf16"]["train_loss"])

