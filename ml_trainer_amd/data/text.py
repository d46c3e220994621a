"""Synthetic sequence-classification data for the BERT configs (no network: no
GLUE download). Token ids uniform over the vocabulary (ids >= 5 so special ids
stay free); with ``learnable=True`` the label is decided by whether a marker
token appears in the first half of the sequence, so training curves move."""
from __future__ import annotations

import numpy as np
import torch


class SyntheticTextClassification(torch.utils.data.Dataset):
    def __init__(self, n: int, seq_len: int = 512, vocab_size: int = 30522, num_labels: int = 2, seed: int = 0,
                 learnable: bool = False):
        rng = np.random.default_rng(seed)
        self.ids = torch.from_numpy(rng.integers(5, vocab_size, size=(n, seq_len), dtype=np.int64))
        self.targets = torch.from_numpy(rng.integers(0, num_labels, size=n, dtype=np.int64))
        if learnable:
            marker = 3
            pos = torch.from_numpy(rng.integers(1, max(seq_len // 2, 2), size=n))
            has = self.targets == 1
            self.ids[has, pos[has]] = marker
        self.classes = [str(i) for i in range(num_labels)]
        self.seq_len = seq_len

    def __len__(self) -> int:
        return self.ids.shape[0]

    def __getitem__(self, i):
        return self.ids[i], int(self.targets[i])
