"""TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Restatement of ``GraphDataset.load_one_graph`` (reference
``deeprank2/dataset.py:883-1052``) over the ``.npz`` dump written by
``deeprank2_amd/io/h5extract.py`` (h5py is only present in the conda
interpreter, so the reference's own reader cannot run next to torch here).
"""

from __future__ import annotations

import numpy as np
import torch

from oracle import pyg_ops as P


def read_dump(path):
    """{entry_name: {"group/name": array}} in file order."""
    z = np.load(path, allow_pickle=False)
    entries = [s.split("\t", 1)[1] for s in z["__entries__"]]
    out = {e: {} for e in entries}
    for key in z.files:
        if key.startswith("__"):
            continue
        k, name = key.split("|", 1)
        out[entries[int(k)]][name] = z[key]
    return out


def _feature_block(grp, group, feats, transform_cfg, means, devs):
    blocks = []
    for feat in feats:
        if feat.startswith("_"):
            continue
        vals = grp[f"{group}/{feat}"]
        transform = standard = None
        if transform_cfg is not None:  # dataset.py:906-915 precedence
            transform = transform_cfg.get("all", {}).get("transform")
            standard = transform_cfg.get("all", {}).get("standardize")
            if transform is None and feat in transform_cfg:
                transform = transform_cfg.get(feat, {}).get("transform")
            if standard is None and feat in transform_cfg:
                standard = transform_cfg.get(feat, {}).get("standardize")
        if transform:
            vals = transform(vals)
        if vals.ndim == 1:
            vals = vals.reshape(-1, 1)
            if standard:
                vals = (vals - means[feat]) / devs[feat]
        elif standard:
            m = [v for k, v in means.items() if feat in k]
            d = [v for k, v in devs.items() if feat in k]
            vals = (vals - m) / d
        blocks.append(vals)
    return blocks


def load_one_graph(grp, name, node_features, edge_features, target=None, clustering_method=None, features_transform=None, means=None, devs=None, task="regress", target_transform=False):
    nb = _feature_block(grp, "node_features", node_features, features_transform, means, devs)
    x = torch.tensor(np.hstack(nb), dtype=torch.float) if nb else None

    if "edge_features/_index" in grp:
        ind = grp["edge_features/_index"]
        if ind.ndim == 2:  # noqa: PLR2004
            ind = np.vstack((ind, np.flip(ind, 1))).T
        edge_index = torch.tensor(ind, dtype=torch.long).contiguous()
    else:
        edge_index = torch.empty((2, 0), dtype=torch.long)

    eb = _feature_block(grp, "edge_features", edge_features, features_transform, means, devs)
    if eb:
        ed = np.hstack(eb)
        edge_attr = torch.tensor(np.vstack((ed, ed)), dtype=torch.float).contiguous()
    else:
        edge_attr = torch.empty((edge_index.shape[1], 0), dtype=torch.float)

    y = None
    if target is not None and f"target_values/{target}" in grp:
        y = torch.tensor([grp[f"target_values/{target}"][()]], dtype=torch.float)
        if task == "regress" and target_transform:
            y = torch.sigmoid(torch.log(y))

    pos = torch.tensor(grp["node_features/_position"], dtype=torch.float).contiguous()
    c0 = c1 = None
    if clustering_method is not None:
        k0 = f"clustering/{clustering_method}/depth_0"
        k1 = f"clustering/{clustering_method}/depth_1"
        if k0 in grp and k1 in grp:
            c0 = torch.tensor(grp[k0], dtype=torch.long)
            c1 = torch.tensor(grp[k1], dtype=torch.long)
    d = P.Data(x=x, edge_index=edge_index, edge_attr=edge_attr, y=y, pos=pos)
    d.cluster0 = c0
    d.cluster1 = c1
    d.entry_names = name
    return d


def synthetic_to_data(g, name="synthetic"):
    """A ``deeprank2_amd.utils.synthetic`` graph as the ``Data`` load_one_graph would build."""
    ind = g["index"]
    ei = np.vstack((ind, np.flip(ind, 1))).T
    ea = np.vstack((g["edge_attr_half"], g["edge_attr_half"]))
    d = P.Data(
        x=torch.tensor(g["x"], dtype=torch.float),
        edge_index=torch.tensor(ei, dtype=torch.long).contiguous(),
        edge_attr=torch.tensor(ea, dtype=torch.float),
        y=torch.tensor([float(g["y"])], dtype=torch.float),
        pos=torch.tensor(g["pos"], dtype=torch.float),
    )
    d.cluster0 = torch.tensor(g["cluster0"], dtype=torch.long)
    d.cluster1 = torch.tensor(g["cluster1"], dtype=torch.long)
    d.entry_names = name
    return d
