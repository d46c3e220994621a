"""Image transforms with torchvision semantics (torchvision is not installed here).

The reference's augmentation (``src/utils/functions.py:5-12``)::

    Compose([RandomCrop(32, padding=4), RandomHorizontalFlip(), ToTensor(),
             Normalize((0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010))])

These classes accept PIL images or HWC uint8 numpy arrays / tensors and
reproduce torchvision's math (zero padding, crop offset uniform in
[0, 2*pad], flip p=0.5, ``/255`` then ``(x-mean)/std``).

:func:`device_augment_spec` recognises any prefix-compatible composition of
these four transforms and returns the parameters of the fused on-GPU
augmentation kernel (``csrc/kernels/lenet.hip`` K1 / ``cifar_augment``), which
applies the same transform to an HBM-resident uint8 dataset.
"""
from __future__ import annotations

import random
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch


def _to_hwc_array(img) -> np.ndarray:
    if isinstance(img, np.ndarray):
        return img
    if isinstance(img, torch.Tensor):
        return img.numpy()
    try:
        from PIL import Image
        if isinstance(img, Image.Image):
            return np.asarray(img)
    except ImportError:  # pragma: no cover
        pass
    raise TypeError(f"unsupported image type {type(img)}")


class Compose:
    def __init__(self, transforms: Sequence[Any]):
        self.transforms = list(transforms)

    def __call__(self, img):
        for t in self.transforms:
            img = t(img)
        return img

    def __repr__(self):
        return "Compose(" + ", ".join(repr(t) for t in self.transforms) + ")"


class RandomCrop:
    def __init__(self, size, padding: int = 0, fill: int = 0):
        self.size = (size, size) if isinstance(size, int) else tuple(size)
        self.padding = int(padding)
        self.fill = fill

    def __call__(self, img):
        a = _to_hwc_array(img)
        p = self.padding
        if p:
            a = np.pad(a, ((p, p), (p, p), (0, 0)) if a.ndim == 3 else ((p, p), (p, p)),
                       mode="constant", constant_values=self.fill)
        h, w = a.shape[:2]
        th, tw = self.size
        i = random.randint(0, h - th)
        j = random.randint(0, w - tw)
        return np.ascontiguousarray(a[i:i + th, j:j + tw])

    def __repr__(self):
        return f"RandomCrop(size={self.size}, padding={self.padding})"


class RandomHorizontalFlip:
    def __init__(self, p: float = 0.5):
        self.p = p

    def __call__(self, img):
        a = _to_hwc_array(img)
        if random.random() < self.p:
            return np.ascontiguousarray(a[:, ::-1])
        return a

    def __repr__(self):
        return f"RandomHorizontalFlip(p={self.p})"


class ToTensor:
    def __call__(self, img):
        a = _to_hwc_array(img)
        if a.ndim == 2:
            a = a[:, :, None]
        t = torch.from_numpy(np.ascontiguousarray(a)).permute(2, 0, 1).contiguous()
        if t.dtype == torch.uint8:
            return t.to(torch.float32).div(255)
        return t.to(torch.float32)

    def __repr__(self):
        return "ToTensor()"


class Normalize:
    def __init__(self, mean: Sequence[float], std: Sequence[float]):
        self.mean = [float(m) for m in mean]
        self.std = [float(s) for s in std]

    def __call__(self, t: torch.Tensor):
        m = torch.tensor(self.mean, dtype=t.dtype).view(-1, 1, 1)
        s = torch.tensor(self.std, dtype=t.dtype).view(-1, 1, 1)
        return (t - m) / s

    def __repr__(self):
        return f"Normalize(mean={self.mean}, std={self.std})"


def device_augment_spec(transform) -> Optional[Dict[str, Any]]:
    """Map a transform to the fused GPU augmentation parameters, or None if it
    contains anything the kernel does not implement.

    ``None`` transform -> ToTensor-only semantics (the reference would crash in
    default_collate on PIL images; we feed tensors instead).
    """
    spec = dict(pad=0, flip=False, mean=(0.0, 0.0, 0.0), std=(1.0, 1.0, 1.0))
    if transform is None:
        return spec
    ts: List[Any] = transform.transforms if isinstance(transform, Compose) else [transform]
    stage = 0  # 0: crop/flip allowed, 1: after ToTensor (normalize allowed), 2: done
    saw_tensor = False
    for t in ts:
        if isinstance(t, RandomCrop) and stage == 0 and not spec["flip"]:
            if t.size != (32, 32) or t.fill != 0 or spec["pad"]:
                return None
            spec["pad"] = t.padding
        elif isinstance(t, RandomHorizontalFlip) and stage == 0:
            if t.p != 0.5:
                return None
            spec["flip"] = True
        elif isinstance(t, ToTensor) and stage == 0:
            stage, saw_tensor = 1, True
        elif isinstance(t, Normalize) and stage == 1:
            if len(t.mean) != 3 or len(t.std) != 3:
                return None
            spec["mean"], spec["std"] = tuple(t.mean), tuple(t.std)
            stage = 2
        else:
            return None
    return spec if saw_tensor else None
