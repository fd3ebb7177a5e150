"""DataLoader over a :class:`~deeprank2_amd.dataset.GraphDataset`.

Replaces ``torch_geometric.loader.DataLoader(dataset, batch_size, shuffle,
num_workers, pin_memory)`` as ``Trainer`` uses it (reference
``deeprank2/trainer.py:541-558,856-861``).  A batch is the list of dataset
positions it covers; its graphs already sit in the dataset's HBM store, so
nothing is collated or copied per step (the fused models read the store via
``Batch.dr_handle``).  ``num_workers`` / ``pin_memory`` are accepted for API
compatibility and have nothing to do here.

Epoch order consumes torch's RNG exactly as ``torch.utils.data.DataLoader``
(which PyG's loader subclasses) does with ``num_workers=0``: creating the
iterator draws the base seed (one int64 from ``generator`` or the global
RNG, also without shuffling); with ``shuffle`` the ``RandomSampler`` then
draws one int64 from the global RNG to seed a private generator (or uses
``generator``) and takes ``torch.randperm(n)`` from it.  So under the same
``torch.manual_seed`` the batches and the RNG state after them match the
reference's loader.

Data parallel: with ``process_group`` set, every rank draws the same way (so
RNG states stay in step) and rank 0's order is broadcast, so all ranks walk
the same global batches and shard them (``distributed.shard_contiguous``).
"""

from __future__ import annotations

import numpy as np
import torch

from deeprank2_amd.data import Batch


class DataLoader:
    def __init__(self, dataset, batch_size: int = 1, shuffle: bool = False, num_workers: int = 0, pin_memory: bool = False, drop_last: bool = False, generator=None, process_group=None, **_kw):  # noqa: ARG002
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
        self.process_group = process_group

    def __len__(self):
        n = len(self.dataset)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def _order(self):
        n = len(self.dataset)
        # _BaseDataLoaderIter.__init__: the iterator's base seed (drawn even without shuffle)
        torch.empty((), dtype=torch.int64).random_(generator=self.generator)
        if not self.shuffle:
            return np.arange(n)
        gen = self.generator
        if gen is None:  # RandomSampler.__iter__: a private generator seeded from the global RNG
            seed = int(torch.empty((), dtype=torch.int64).random_().item())
            gen = torch.Generator()
            gen.manual_seed(seed)
        order = torch.randperm(n, generator=gen).numpy()
        pg = self.process_group
        if pg is not None and torch.distributed.get_world_size(pg) > 1:
            box = [order]
            torch.distributed.broadcast_object_list(box, src=torch.distributed.get_global_rank(pg, 0), group=pg)
            order = np.asarray(box[0])
        return order

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
