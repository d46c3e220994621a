"""Sampler partition, transforms, CIFAR readers, device-augment spec recognition, logger format."""
import datetime
import os
import pickle

import numpy as np
import pytest
import torch
from torch.utils.data import DistributedSampler

from ml_trainer_amd.data import transforms as T
from ml_trainer_amd.data.cifar10 import CIFAR10, SyntheticCIFAR10
from ml_trainer_amd.data.loader import Loader, device_dataset_spec
from ml_trainer_amd.parallel.sampler import ShardSampler, shard_indices
from ml_trainer_amd.utils.functions import custom_pre_process_function
from ml_trainer_amd.utils.logging import render


@pytest.mark.parametrize("n", [1, 7, 103, 50000])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_indices_equal_distributed_sampler(n, world):
    ds = range(n)
    for rank in range(world):
        s = DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=True, seed=0)
        s.set_epoch(5)
        assert list(s) == shard_indices(n, world, rank, True, 0, 5)
        ss = ShardSampler(ds, num_replicas=world, rank=rank)
        ss.set_epoch(5)
        assert list(ss) == list(s) and len(ss) == len(s)


def test_reference_transform_semantics():
    tf = custom_pre_process_function()
    img = np.random.default_rng(0).integers(0, 256, (32, 32, 3), dtype=np.uint8)
    out = tf(img)
    assert out.shape == (3, 32, 32) and out.dtype == torch.float32
    # no-crop/no-flip pipeline reduces to ToTensor+Normalize exactly
    base = T.Compose([T.ToTensor(), T.Normalize((0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010))])(img)
    ref = (torch.from_numpy(img).permute(2, 0, 1).float() / 255 - torch.tensor([0.4914, 0.4822, 0.4465]).view(3, 1, 1)) \
        / torch.tensor([0.2023, 0.1994, 0.2010]).view(3, 1, 1)
    torch.testing.assert_close(base, ref)
    # crop content: every output row is a shifted window of the zero-padded image
    crop = T.RandomCrop(32, padding=4)(img)
    padded = np.pad(img, ((4, 4), (4, 4), (0, 0)))
    found = any((padded[i:i + 32, j:j + 32] == crop).all() for i in range(9) for j in range(9))
    assert found


def test_device_augment_spec():
    assert device_augment_spec_is(custom_pre_process_function(), pad=4, flip=True)
    assert T.device_augment_spec(None)["pad"] == 0
    assert T.device_augment_spec(T.Compose([T.RandomHorizontalFlip(0.3), T.ToTensor()])) is None
    assert T.device_augment_spec(T.Compose([T.Normalize((0,) * 3, (1,) * 3)])) is None


def device_augment_spec_is(tf, pad, flip):
    s = T.device_augment_spec(tf)
    return s is not None and s["pad"] == pad and s["flip"] == flip


def _write_cifar_py(root, n_per=10):
    d = os.path.join(root, "cifar-10-batches-py")
    os.makedirs(d)
    rng = np.random.default_rng(0)
    allx, ally = [], []
    for fn in [f"data_batch_{i}" for i in range(1, 6)] + ["test_batch"]:
        x = rng.integers(0, 256, (n_per, 3072), dtype=np.uint8)
        y = rng.integers(0, 10, n_per).tolist()
        with open(os.path.join(d, fn), "wb") as f:
            pickle.dump({"data": x, "labels": y}, f)
        allx.append(x)
        ally.append(y)
    with open(os.path.join(d, "batches.meta"), "wb") as f:
        pickle.dump({"label_names": ["c%d" % i for i in range(10)]}, f)
    return allx, ally


def test_cifar_python_batches(tmp_path):
    xs, ys = _write_cifar_py(str(tmp_path))
    tr = CIFAR10(str(tmp_path), train=True)
    te = CIFAR10(str(tmp_path), train=False)
    assert len(tr) == 50 and len(te) == 10 and tr.classes[3] == "c3"
    assert tr.data.shape == (50, 32, 32, 3)
    np.testing.assert_array_equal(tr.data[0], xs[0][0].reshape(3, 32, 32).transpose(1, 2, 0))
    assert tr.targets[:10] == ys[0]
    x, y = tr[0]
    assert isinstance(x, torch.Tensor) and x.shape == (3, 32, 32)  # B10 fix: tensors without a transform


def test_cifar_rejects_code_in_pickle(tmp_path):
    d = tmp_path / "cifar-10-batches-py"
    d.mkdir()

    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))
    for fn in [f"data_batch_{i}" for i in range(1, 6)]:
        with open(d / fn, "wb") as f:
            pickle.dump({"data": Evil(), "labels": []}, f)
    with pytest.raises(pickle.UnpicklingError):
        CIFAR10(str(tmp_path), train=True)


def test_cifar_binary_batches(tmp_path):
    d = tmp_path / "cifar-10-batches-bin"
    d.mkdir()
    rng = np.random.default_rng(1)
    for fn in [f"data_batch_{i}.bin" for i in range(1, 6)] + ["test_batch.bin"]:
        recs = np.concatenate([rng.integers(0, 10, (4, 1)), rng.integers(0, 256, (4, 3072))], 1).astype(np.uint8)
        recs.tofile(d / fn)
    assert len(CIFAR10(str(tmp_path), train=True)) == 20


def test_download_disabled():
    with pytest.raises(RuntimeError):
        CIFAR10("/nonexistent", download=True)


def test_device_dataset_spec_and_loader():
    ds = SyntheticCIFAR10(16, transform=custom_pre_process_function())
    assert device_dataset_spec(ds)["pad"] == 4
    assert Loader(ds, batch_size=4).device_capable()
    x, y = next(iter(Loader(ds, batch_size=4)))
    assert x.shape == (4, 3, 32, 32)


def test_log_render_format():
    line = render("info", "Config inputs.", {"config": {"lr": 0.1}}, now=datetime.datetime(2023, 2, 3, 15, 21, 11))
    assert line == "2023-02-03 15:21.11 [info     ] Config inputs.                 config={'lr': 0.1}"
