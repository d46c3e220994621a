"""CIFAR-10 datasets without torchvision.

``CIFAR10`` reads the standard ``cifar-10-batches-py`` layout that
``torchvision.datasets.CIFAR10(root, train, download=False)`` reads in the
reference (``main.py:14-28``, ``01_ML_Training_local.ipynb:77-97``): pickled
batch dicts ``{b'data': uint8[N,3072], b'labels': [...]}`` plus
``batches.meta``. The pickles are read with a *restricted* unpickler that only
admits plain containers and numpy array reconstruction, so a malicious file
cannot execute code. The binary ``cifar-10-batches-bin`` layout is also
accepted (fixed 3073-byte records, no pickle at all).

``SyntheticCIFAR10`` has the same attributes (``data`` uint8 [N,32,32,3],
``targets``, ``classes``) filled from a seeded generator -- the benchmark /
test dataset (no network, no real data in this environment).

Both expose ``data``/``targets`` so the Trainer can upload them once to HBM and
run augmentation on the GPU (``Loader.device_capable``).
"""
from __future__ import annotations

import io
import os
import pickle
from typing import Callable, List, Optional, Tuple

import numpy as np

CLASSES = ["airplane", "automobile", "bird", "cat", "deer", "dog", "frog", "horse", "ship", "truck"]

_TRAIN_PY = [f"data_batch_{i}" for i in range(1, 6)]
_TEST_PY = ["test_batch"]
_TRAIN_BIN = [f"data_batch_{i}.bin" for i in range(1, 6)]
_TEST_BIN = ["test_batch.bin"]


class _SafeUnpickler(pickle.Unpickler):
    _ALLOWED = {
        ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
        ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"),
        ("numpy._core.multiarray", "scalar"), ("_codecs", "encode"), ("builtins", "bytearray"),
    }

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from a dataset file")


def _safe_load(path: str):
    with open(path, "rb") as f:
        return _SafeUnpickler(f, encoding="latin1").load()


def _find_dir(root: str, name: str) -> Optional[str]:
    for cand in (os.path.join(root, name), root):
        if os.path.isdir(cand) and any(f.startswith("data_batch") or f.startswith("test_batch")
                                       for f in os.listdir(cand)):
            return cand
    return None


def load_cifar10_arrays(root: str, train: bool = True) -> Tuple[np.ndarray, List[int], List[str]]:
    d = _find_dir(root, "cifar-10-batches-py")
    if d is not None and os.path.exists(os.path.join(d, (_TRAIN_PY if train else _TEST_PY)[0])):
        datas, labels = [], []
        for fn in (_TRAIN_PY if train else _TEST_PY):
            entry = _safe_load(os.path.join(d, fn))
            datas.append(np.asarray(entry["data"], dtype=np.uint8))
            labels.extend(entry["labels"] if "labels" in entry else entry["fine_labels"])
        data = np.vstack(datas).reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1)
        classes = CLASSES
        meta = os.path.join(d, "batches.meta")
        if os.path.exists(meta):
            classes = list(_safe_load(meta)["label_names"])
        return np.ascontiguousarray(data), list(labels), classes
    d = _find_dir(root, "cifar-10-batches-bin")
    if d is not None:
        recs = []
        for fn in (_TRAIN_BIN if train else _TEST_BIN):
            raw = np.fromfile(os.path.join(d, fn), dtype=np.uint8).reshape(-1, 3073)
            recs.append(raw)
        raw = np.vstack(recs)
        labels = raw[:, 0].astype(np.int64).tolist()
        data = raw[:, 1:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1)
        return np.ascontiguousarray(data), labels, CLASSES
    raise FileNotFoundError(f"no CIFAR-10 batches under {root!r} (expected cifar-10-batches-py or -bin); "
                            "download is disabled in this environment")


class _CifarBase:
    data: np.ndarray
    targets: List[int]
    classes: List[str]
    transform: Optional[Callable]
    target_transform: Optional[Callable]
    as_pil = True

    def __len__(self) -> int:
        return len(self.targets)

    def __getitem__(self, index: int):
        img, target = self.data[index], int(self.targets[index])
        if self.transform is not None:
            if self.as_pil:
                try:
                    from PIL import Image
                    img = Image.fromarray(img)
                except ImportError:  # pragma: no cover
                    pass
            img = self.transform(img)
        else:
            # reference B10 fix: without a transform torchvision yields PIL images that
            # default_collate rejects; we yield a ToTensor()-style float tensor instead.
            import torch
            img = torch.from_numpy(np.ascontiguousarray(img)).permute(2, 0, 1).float().div(255)
        if self.target_transform is not None:
            target = self.target_transform(target)
        return img, target

    @property
    def class_to_idx(self):
        return {c: i for i, c in enumerate(self.classes)}


class CIFAR10(_CifarBase):
    def __init__(self, root: str, train: bool = True, transform: Optional[Callable] = None,
                 target_transform: Optional[Callable] = None, download: bool = False):
        if download:
            raise RuntimeError("download=True is not supported (no network); place the batches under root")
        self.root, self.train = root, train
        self.transform, self.target_transform = transform, target_transform
        self.data, self.targets, self.classes = load_cifar10_arrays(root, train)


class SyntheticCIFAR10(_CifarBase):
    """Seeded random CIFAR-10-shaped dataset (50,000 train / 10,000 test by default).

    ``learnable``: False = uniform noise (throughput runs); True = a class-dependent brightness
    offset (fitted within an epoch: plumbing tests); ``"pattern"`` = each class a fixed 4x4-block
    colour template (the same for train and test: ``pattern_seed``) blended 12/88 with uniform
    noise -- the model has to learn spatial colour filters and accuracy climbs over several epochs
    (training-quality comparisons, e.g. bf16 vs fp32)."""

    def __init__(self, n: Optional[int] = None, train: bool = True, transform: Optional[Callable] = None,
                 target_transform: Optional[Callable] = None, seed: int = 0, learnable=False,
                 pattern_seed: int = 1234):
        n = n if n is not None else (50000 if train else 10000)
        rng = np.random.default_rng(seed + (0 if train else 1))
        self.targets = rng.integers(0, 10, size=n).tolist()
        if learnable == "pattern":
            prng = np.random.default_rng(pattern_seed)
            tmpl = prng.integers(0, 256, size=(10, 4, 4, 3)).astype(np.float32)
            tmpl = tmpl.repeat(8, axis=1).repeat(8, axis=2)  # [10, 32, 32, 3]
            t = np.asarray(self.targets)
            noise = rng.integers(0, 256, size=(n, 32, 32, 3)).astype(np.float32)
            self.data = np.clip(0.12 * tmpl[t] + 0.88 * noise, 0, 255).astype(np.uint8)
        elif learnable:
            # class-dependent colour offset so a model can actually fit it (tests)
            t = np.asarray(self.targets, dtype=np.int16).reshape(n, 1, 1, 1)
            noise = rng.integers(0, 40, size=(n, 32, 32, 3), dtype=np.int16)
            self.data = np.clip(t * 20 + noise, 0, 255).astype(np.uint8)
        else:
            self.data = rng.integers(0, 256, size=(n, 32, 32, 3), dtype=np.uint8)
        self.classes = list(CLASSES)
        self.train = train
        self.transform, self.target_transform = transform, target_transform
