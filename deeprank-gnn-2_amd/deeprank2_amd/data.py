"""Graph containers with the attribute surface DeepRank2 code uses.

``Data`` is what ``GraphDataset.get`` returns (reference
``deeprank2/dataset.py:1044-1052``: ``x, edge_index, edge_attr, y, pos,
cluster0, cluster1, entry_names``).  ``Batch`` is what the loader yields; it
carries the graph ids of the batch so the fused models read the HBM-resident
store directly, and materialises PyG's collated tensors (``Batch.from_data_list``:
node-offset ``edge_index``, ``batch`` vector, ``ptr``, concatenated ``y``,
``cluster0/1`` concatenated WITHOUT offsets, ``entry_names`` list) only if a
caller reads them.
"""

from __future__ import annotations

import torch

_TENSOR_KEYS = ("x", "edge_index", "edge_attr", "y", "pos", "cluster0", "cluster1")


class Data:
    def __init__(self, x=None, edge_index=None, edge_attr=None, y=None, pos=None, **kw):
        self.x = x
        self.edge_index = edge_index
        self.edge_attr = edge_attr
        self.y = y
        self.pos = pos
        self.cluster0 = None
        self.cluster1 = None
        self.entry_names = None
        for k, v in kw.items():
            setattr(self, k, v)

    @property
    def num_nodes(self):
        if self.x is not None:
            return int(self.x.shape[0])
        return int(self.pos.shape[0]) if self.pos is not None else 0

    @property
    def num_features(self):
        return 0 if self.x is None else (1 if self.x.dim() == 1 else int(self.x.shape[1]))

    num_node_features = num_features

    @property
    def num_edges(self):
        return 0 if self.edge_index is None else int(self.edge_index.shape[1])

    def keys(self):
        return [k for k, v in self.__dict__.items() if v is not None]

    def __contains__(self, key):
        return getattr(self, key, None) is not None

    def clone(self):
        out = Data()
        for k, v in self.__dict__.items():
            setattr(out, k, v.clone() if isinstance(v, torch.Tensor) else v)
        return out

    def to(self, device, non_blocking=False):
        for k, v in list(self.__dict__.items()):
            if isinstance(v, torch.Tensor):
                setattr(self, k, v.to(device, non_blocking=non_blocking))
        return self

    def __repr__(self):
        parts = [f"{k}={list(v.shape)}" for k, v in self.__dict__.items() if isinstance(v, torch.Tensor)]
        return f"Data({', '.join(parts)})"


def collate(datas) -> dict:
    """PyG ``Batch.from_data_list`` for the keys DeepRank2 graphs carry."""
    out = {}
    n = [d.num_nodes for d in datas]
    offs = torch.tensor([0, *n]).cumsum(0)
    out["ptr"] = offs
    out["batch"] = torch.repeat_interleave(torch.arange(len(datas)), torch.tensor(n, dtype=torch.long)) if datas else torch.zeros(0, dtype=torch.long)
    for k in _TENSOR_KEYS:
        vals = [getattr(d, k, None) for d in datas]
        if any(v is None for v in vals):
            out[k] = None
            continue
        if k == "edge_index":
            out[k] = torch.cat([v + offs[i] for i, v in enumerate(vals)], dim=1)
        else:
            out[k] = torch.cat(vals, dim=0)
    out["entry_names"] = [d.entry_names for d in datas]
    return out


class Batch(Data):
    """A mini-batch.  ``dr_handle(device)`` gives the fused models the batch's
    graph ids in the dataset's resident store; tensor attributes are collated
    lazily from ``dataset.get`` when first read."""

    def __init__(self, dataset=None, indices=None, **kw):
        object.__setattr__(self, "_dataset", dataset)
        object.__setattr__(self, "_indices", None if indices is None else [int(i) for i in indices])
        object.__setattr__(self, "_collated", None)
        object.__setattr__(self, "_device", None)
        object.__setattr__(self, "_overrides", {})
        for k, v in kw.items():
            self._overrides[k] = v

    @classmethod
    def from_data_list(cls, datas):
        return cls(**collate(datas))

    # lazy attribute access ---------------------------------------------------
    def _collate(self):
        if self._collated is None:
            datas = [self._dataset.get(i) for i in self._indices]
            c = collate(datas)
            if self._device is not None:
                c = {k: (v.to(self._device) if isinstance(v, torch.Tensor) else v) for k, v in c.items()}
            object.__setattr__(self, "_collated", c)
        return self._collated

    def __getattr__(self, key):
        if key.startswith("__"):
            raise AttributeError(key)
        ov = object.__getattribute__(self, "_overrides")
        if key in ov:
            return ov[key]
        if key == "y" and self._dataset is not None:
            y = self._dataset._targets_of(self._indices)  # noqa: SLF001
            if y is not None and self._device is not None:
                y = y.to(self._device)
            return y
        if key == "entry_names" and self._dataset is not None:
            return [self._dataset.index_entries[i][1] for i in self._indices]
        if key in (*_TENSOR_KEYS, "batch", "ptr"):
            if self._dataset is None:
                return None
            return self._collate()[key]
        raise AttributeError(key)

    def __setattr__(self, key, value):
        self._overrides[key] = value

    @property
    def num_graphs(self):
        if self._indices is not None:
            return len(self._indices)
        p = self._overrides.get("ptr")
        return 0 if p is None else int(p.numel()) - 1

    @property
    def __dict__(self):  # for Data.keys()/clone(): the materialised view
        d = {}
        if self._dataset is not None:
            d.update(self._collate())
        d.update(self._overrides)
        return d

    def clone(self):
        return Batch(**{k: (v.clone() if isinstance(v, torch.Tensor) else v) for k, v in self.__dict__.items()})

    def to(self, device, non_blocking=False):
        object.__setattr__(self, "_device", torch.device(device))
        for k, v in list(self._overrides.items()):
            if isinstance(v, torch.Tensor):
                self._overrides[k] = v.to(device, non_blocking=non_blocking)
        if self._collated is not None:
            object.__setattr__(self, "_collated", {k: (v.to(device) if isinstance(v, torch.Tensor) else v) for k, v in self._collated.items()})
        return self

    def dr_handle(self, device):
        """BatchHandle on the dataset's HBM-resident store (None for a free-standing batch)."""
        if self._dataset is None or not hasattr(self._dataset, "batch_handle"):
            return None
        return self._dataset.batch_handle(self._indices, device)
