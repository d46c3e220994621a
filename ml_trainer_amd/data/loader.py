"""``Loader`` (reference ``src/dataloader.py``: ``class Loader(DataLoader): pass``)
plus the MI355X input paths.

Three ways a batch reaches the GPU:

1. **HBM-resident dataset** (fast path). Datasets exposing ``data`` (uint8
   ``[N,32,32,3]``) + ``targets`` and a transform the fused augmentation kernel
   implements (see :func:`~ml_trainer_amd.data.transforms.device_augment_spec`)
   are uploaded ONCE (150 MB for CIFAR-10 train: nothing next to 288 GB of
   HBM3E). Each epoch only the sampler's permutation (200 KB) is copied; crop /
   flip / normalise happen inside the first conv kernel (LeNet engine) or in
   ``cifar_augment`` (generic models). No per-step host work, no H2D copies.
2. **Pinned-host prefetch** (generic datasets). A ``DataLoader`` collates on the
   host; :class:`DevicePrefetcher` copies each batch into pinned memory and
   issues the H2D ``hipMemcpyAsync`` on a dedicated copy stream, ``depth``
   batches ahead, with event ordering into the compute stream.
3. Plain iteration (CPU plumbing config).

``Loader`` keeps the ``DataLoader`` signature and attributes (``dataset``,
``sampler``, ``batch_size``, ``__len__``) that the reference Trainer and
notebooks use (``trainer.train_loader`` / ``val_loader``, ``01…ipynb:269,507``).
"""
from __future__ import annotations

from typing import Any, Dict, Iterator, Optional, Tuple

import numpy as np
import torch
from torch.utils.data import DataLoader

from ml_trainer_amd.data.transforms import device_augment_spec


class Loader(DataLoader):
    """DataLoader with the reference name; adds device-path introspection."""

    def device_capable(self) -> bool:
        return device_dataset_spec(self.dataset) is not None


def device_dataset_spec(dataset) -> Optional[Dict[str, Any]]:
    """Return the on-GPU augmentation spec when the dataset can live in HBM, else None."""
    data = getattr(dataset, "data", None)
    targets = getattr(dataset, "targets", None)
    if data is None or targets is None:
        return None
    if getattr(dataset, "target_transform", None) is not None:
        return None
    shape = tuple(getattr(data, "shape", ()))
    if len(shape) != 4 or shape[1:] != (32, 32, 3):
        return None
    dt = getattr(data, "dtype", None)
    if dt not in (np.uint8, torch.uint8):
        return None
    return device_augment_spec(getattr(dataset, "transform", None))


class DeviceDataset:
    """A dataset's uint8 pixels + targets resident in HBM."""

    def __init__(self, dataset, device: torch.device):
        spec = device_dataset_spec(dataset)
        if spec is None:
            raise ValueError("dataset is not device-capable")
        data = dataset.data
        data_t = torch.as_tensor(np.ascontiguousarray(data)) if isinstance(data, np.ndarray) else data
        self.data = data_t.to(device, non_blocking=False).contiguous()
        self.targets = torch.as_tensor(np.asarray(dataset.targets), dtype=torch.int64).to(device)
        self.spec = spec
        self.n = self.data.shape[0]
        self.device = device


class NativePinnedPrefetcher:
    """Batches staged through the native pinned-host ring (csrc/runtime/runtime.cpp
    ``PinnedPrefetcher``): ``depth`` persistent hipHostMalloc slots + device buffers,
    hipMemcpyAsync on a dedicated copy stream. The copy of batch k + depth - 1 waits only for
    the compute that last read its device buffer (batch k - 1's, released when the consumer
    asked for batch k), and the compute stream waits for a batch's copy only where the batch is
    consumed -- so the copies run under the previous batches' kernels. No per-batch pinned
    allocation, no host synchronisation except reusing a host slot whose copy is in flight."""

    def __init__(self, loader: DataLoader, device: torch.device, depth: int = 3):
        from ml_trainer_amd.ops._ext import require_native
        self.C = require_native()
        self.loader = loader
        self.device = device
        self.depth = max(2, int(depth))
        self.pf = None
        self.dev_bufs = []

    def __len__(self) -> int:
        return len(self.loader)

    def _layout(self, x: torch.Tensor, y: torch.Tensor):
        xb = x.numel() * x.element_size()
        yo = (xb + 255) // 256 * 256
        return xb, yo, yo + y.numel() * y.element_size()

    def _ensure(self, nbytes: int) -> None:
        if self.pf is None or self.pf.slot_bytes < nbytes:
            if self.pf is not None:
                torch.cuda.current_stream(self.device).synchronize()  # old buffers may still be read
            self.pf = self.C.PinnedPrefetcher(int(nbytes), self.depth, self.device.index or 0)
            self.dev_bufs = [torch.empty(int(nbytes), dtype=torch.uint8, device=self.device)
                             for _ in range(self.depth)]

    def _stage(self, k: int, batch):
        x, y = batch
        y = y if isinstance(y, torch.Tensor) else torch.as_tensor(y)
        x, y = x.contiguous(), y.contiguous()
        xb, yo, total = self._layout(x, y)
        self._ensure(total)
        self.pf.wait(k)  # the host slot's previous H2D copy must be done before we overwrite it
        slot = self.pf.slot(k)
        slot[:xb].copy_(x.view(-1).view(torch.uint8))
        slot[yo:total].copy_(y.view(-1).view(torch.uint8))
        dev = self.dev_bufs[k]
        self.pf.copy_to_device(k, dev, total)  # after the release of buffer k only
        xd = dev[:xb].view(x.dtype).view(x.shape)
        yd = dev[yo:total].view(y.dtype).view(y.shape)
        return k, xd, yd

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        it = iter(self.loader)
        if self.pf is not None:  # a new pass (or one that was abandoned): everything queued so far
            for i in range(self.depth):  # may still read the buffers
                self.pf.release(i)
        pending = []
        k = 0
        for _ in range(self.depth - 1):
            try:
                pending.append(self._stage(k % self.depth, next(it)))
                k += 1
            except StopIteration:
                break
        last = None
        while pending:
            slot, xd, yd = pending.pop(0)
            if last is not None:
                # the consumer enqueued its work on the previous batch when it asked for this one
                self.pf.release(last)
            try:
                # buffer (k % depth) was last used by the batch just released: its copy follows that
                pending.append(self._stage(k % self.depth, next(it)))
                k += 1
            except StopIteration:
                pass
            self.pf.acquire(slot)  # the compute stream waits for this batch's copy here
            last = slot
            yield xd, yd
        if last is not None:
            self.pf.release(last)


class DevicePrefetcher:
    """Iterate a host ``DataLoader`` with batches staged ``depth`` ahead through
    pinned memory and copied on a side stream (torch streams are HIP streams).
    On a GPU with the native extension this delegates to NativePinnedPrefetcher
    (``MLT_NATIVE_PREFETCH=0`` keeps the torch pinned-memory path)."""

    def __new__(cls, loader: DataLoader, device: torch.device, depth: int = 2):
        import os
        device = torch.device(device)
        if device.type == "cuda" and os.environ.get("MLT_NATIVE_PREFETCH", "1") != "0":
            from ml_trainer_amd.ops._ext import native_available
            if native_available():
                return NativePinnedPrefetcher(loader, device, depth=max(depth, 2) + 1)
        return super().__new__(cls)

    def __init__(self, loader: DataLoader, device: torch.device, depth: int = 2):
        self.loader = loader
        self.device = device
        self.depth = max(1, int(depth))
        self.stream = torch.cuda.Stream(device=device) if device.type == "cuda" else None

    def __len__(self) -> int:
        return len(self.loader)

    def _stage(self, batch):
        x, y = batch
        if self.stream is None:
            return x.to(self.device), y.to(self.device), None
        if not x.is_pinned():
            x = x.pin_memory()
        if isinstance(y, torch.Tensor) and not y.is_pinned():
            y = y.pin_memory()
        with torch.cuda.stream(self.stream):
            xd = x.to(self.device, non_blocking=True)
            yd = y.to(self.device, non_blocking=True) if isinstance(y, torch.Tensor) else torch.as_tensor(
                y, device=self.device)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return xd, yd, ev

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        it = iter(self.loader)
        queue = []
        for _ in range(self.depth):
            try:
                queue.append(self._stage(next(it)))
            except StopIteration:
                break
        while queue:
            xd, yd, ev = queue.pop(0)
            if ev is not None:
                torch.cuda.current_stream(self.device).wait_event(ev)
                # the tensors were allocated on the copy stream: tell the allocator they are used here
                xd.record_stream(torch.cuda.current_stream(self.device))
                yd.record_stream(torch.cuda.current_stream(self.device))
            try:
                queue.append(self._stage(next(it)))
            except StopIteration:
                pass
            yield xd, yd
