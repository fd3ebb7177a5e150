"""DataLoader over a :class:`~deeprank2_amd.dataset.GraphDataset`.

Replaces ``torch_geometric.loader.DataLoader(dataset, batch_size, shuffle,
num_workers, pin_memory)`` as ``Trainer`` uses it (reference
``deeprank2/trainer.py:541-558,856-861``).  A batch is the list of dataset
positions it covers; its graphs already sit in the dataset's HBM store, so
nothing is collated or copied per step (the fused models read the store via
``Batch.dr_handle``).  ``num_workers`` / ``pin_memory`` are accepted for API
compatibility and have nothing to do here.

``shuffle`` draws a fresh permutation per epoch from a ``numpy`` generator
(seeded by ``generator`` or torch's global RNG, like PyG's sampler).
"""

from __future__ import annotations

import numpy as np
import torch

from deeprank2_amd.data import Batch


class DataLoader:
    def __init__(self, dataset, batch_size: int = 1, shuffle: bool = False, num_workers: int = 0, pin_memory: bool = False, drop_last: bool = False, generator=None, **_kw):  # noqa: ARG002
        if batch_size < 1:
            msg = "batch_size must be >= 1"
            raise ValueError(msg)
        self.dataset = dataset
        self.batch_size = int(batch_size)
        self.shuffle = bool(shuffle)
        self.drop_last = bool(drop_last)
        self.num_workers = num_workers
        self.pin_memory = pin_memory
        self.generator = generator

    def __len__(self):
        n = len(self.dataset)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def _order(self):
        n = len(self.dataset)
        if not self.shuffle:
            return np.arange(n)
        seed = int(torch.randint(0, 2**62, (1,), generator=self.generator).item())
        return np.random.default_rng(seed).permutation(n)

    def batches(self):
        """Lists of dataset positions, one per mini-batch, in this epoch's order."""
        order = self._order()
        out = [order[i:i + self.batch_size] for i in range(0, len(order), self.batch_size)]
        if self.drop_last and out and len(out[-1]) < self.batch_size:
            out.pop()
        return out

    def __iter__(self):
        for idx in self.batches():
            yield Batch(self.dataset, idx)
