"""GraphDataset / DataLoader / collate (CPU).

* Synthetic DeepRank2-layout HDF5 files written by ``utils.synthetic`` (our own
  writer): items and collated batches equal the generator's arrays, edges
  doubled as ``dataset.py:944-948,994-996``.
* The reference's own fixtures (``tests/data/hdf5``) read IN PLACE when
  /root/reference is present (this container only; never copied into the
  repo): batch tensors equal the ``ginet_1atn`` golden inputs, and the
  assertions of the reference's ``tests/test_dataset.py`` (lengths, target
  filter, doubled edge feature statistics, task/classes) hold.
"""

from __future__ import annotations

import os

import numpy as np
import pytest
import torch

from deeprank2_amd.data import Batch, collate
from deeprank2_amd.dataset import GraphDataset
from deeprank2_amd.loader import DataLoader
from deeprank2_amd.utils import synthetic as S

REF_H5 = "/root/reference/tests/data/hdf5"
needs_ref = pytest.mark.skipif(not os.path.isdir(REF_H5), reason="reference fixtures not present (GPU box)")
DEFAULT_FEATURES = ["res_type", "polarity", "bsa", "res_depth", "hse", "info_content", "pssm"]  # reference tests/test_trainer.py:31-39


@pytest.fixture(scope="module")
def synth_file(tmp_path_factory):
    graphs = S.make_dataset(7, seed=31, n_lo=20, n_hi=45, mean_degree=6.0)
    path = str(tmp_path_factory.mktemp("h5") / "synth.hdf5")
    names = S.write_hdf5(path, graphs)
    return path, graphs, names


def _ds(path, **kw):
    kw.setdefault("node_features", S.SYNTH_NODE_FEATURES)
    kw.setdefault("edge_features", S.SYNTH_EDGE_FEATURES)
    kw.setdefault("target", "irmsd")
    kw.setdefault("clustering_method", "mcl")
    return GraphDataset(path, **kw)


def test_items_equal_generator_arrays(synth_file):
    path, graphs, names = synth_file
    ds = _ds(path)
    assert len(ds) == ds.len() == 7
    assert [e for _, e in ds.index_entries] == names
    for i, g in enumerate(graphs):
        d = ds.get(i)
        ei, ea = S.doubled_edges(g)
        np.testing.assert_array_equal(d.x.numpy(), g["x"])
        np.testing.assert_array_equal(d.edge_index.numpy(), ei)
        np.testing.assert_array_equal(d.edge_attr.numpy(), ea)
        np.testing.assert_array_equal(d.cluster0.numpy(), g["cluster0"])
        np.testing.assert_array_equal(d.cluster1.numpy(), g["cluster1"])
        assert d.y.dtype == torch.float32 and float(d.y) == pytest.approx(float(g["y"]))
        assert d.entry_names == names[i]
        assert d.num_features == 30


def test_all_features_in_file_order(synth_file):
    ds = _ds(synth_file[0], node_features="all", edge_features="all")
    assert ds.node_features == sorted(S.SYNTH_NODE_FEATURES)  # HDF5 groups iterate by name
    assert ds.edge_features == sorted(S.SYNTH_EDGE_FEATURES)
    assert ds.get(0).x.shape[1] == 30


def test_loader_batches_collate_like_pyg(synth_file):
    path, graphs, _ = synth_file
    ds = _ds(path)
    loader = DataLoader(ds, batch_size=3, shuffle=False)
    batches = list(loader)
    assert len(loader) == len(batches) == 3
    b = batches[1]
    datas = [ds.get(i) for i in (3, 4, 5)]
    n = [d.num_nodes for d in datas]
    np.testing.assert_array_equal(b.ptr.numpy(), np.cumsum([0, *n]))
    np.testing.assert_array_equal(b.batch.numpy(), np.repeat(np.arange(3), n))
    np.testing.assert_array_equal(b.edge_index.numpy(), np.concatenate([d.edge_index.numpy() + o for d, o in zip(datas, np.cumsum([0, *n[:-1]]))], 1))
    np.testing.assert_array_equal(b.cluster1.numpy(), np.concatenate([d.cluster1.numpy() for d in datas]))  # no offsets
    np.testing.assert_allclose(b.y.numpy(), [float(graphs[i]["y"]) for i in (3, 4, 5)], rtol=1e-6)
    assert b.entry_names == [ds.index_entries[i][1] for i in (3, 4, 5)]
    assert b.num_graphs == 3


def test_shuffle_covers_every_graph_once(synth_file):
    ds = _ds(synth_file[0])
    torch.manual_seed(0)
    seen = np.concatenate(DataLoader(ds, batch_size=2, shuffle=True).batches())
    assert sorted(seen.tolist()) == list(range(7))
    assert len(DataLoader(ds, batch_size=2, drop_last=True)) == 3


class _Range:
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


@pytest.mark.parametrize("shuffle", [True, False])
@pytest.mark.parametrize(("n", "bs"), [(7, 2), (64, 8), (1, 4)])
def test_loader_rng_consumption_matches_torch_dataloader(n, bs, shuffle):
    """Same batches and the same torch RNG state afterwards as
    torch.utils.data.DataLoader (which PyG's loader subclasses,
    trainer.py:541-547) under one torch.manual_seed, two epochs in a row."""
    torch.manual_seed(1234)
    ref = torch.utils.data.DataLoader(list(range(n)), batch_size=bs, shuffle=shuffle)
    want = [[b.tolist() for b in ref] for _ in range(2)]
    state = torch.random.get_rng_state()
    torch.manual_seed(1234)
    dl = DataLoader(_Range(n), batch_size=bs, shuffle=shuffle)
    got = [[list(map(int, b)) for b in dl.batches()] for _ in range(2)]
    assert got == want
    assert torch.equal(torch.random.get_rng_state(), state)


def test_subset_order_and_target_filter(synth_file):
    path, graphs, names = synth_file
    ds = _ds(path, subset=[names[5], names[1], "missing"])
    assert [e for _, e in ds.index_entries] == [names[5], names[1]]
    ys = np.array([float(g["y"]) for g in graphs])
    thr = float(np.median(ys))
    ds = _ds(path, target_filter={"irmsd": f">{thr}"})
    assert len(ds) == int((ys.astype(np.float64) > thr).sum())
    with pytest.raises(IndexError):
        _ds(path, target_filter={"irmsd": "<-1"})


def test_target_errors(synth_file):
    with pytest.raises(ValueError, match="Please set the target"):
        GraphDataset(synth_file[0], clustering_method="mcl")
    with pytest.raises(ValueError, match="not present"):
        GraphDataset(synth_file[0], target="dockq", task="regress")
    with pytest.raises(ValueError, match="Not all features"):
        _ds(synth_file[0], node_features=["nope"])


def test_standardize_and_transform_with_train_source(synth_file):
    path = synth_file[0]
    ft = {"bsa": {"transform": lambda t: np.log(t + 10), "standardize": True}, "res_depth": {"standardize": True}}
    tr = _ds(path, features_transform=ft)
    raw = np.concatenate([np.asarray(tr._entry(p, e)["node_features/bsa"]) for p, e in tr.index_entries])  # noqa: SLF001
    assert tr.means["bsa"] == round(float(np.nanmean(np.log(raw + 10))), 1)
    assert tr.devs["bsa"] == round(float(np.nanstd(np.log(raw + 10))), 1)
    col = 24  # res_type (20) and polarity (4) columns come first
    x = tr.get(0).x.numpy()
    bsa0 = np.asarray(tr._entry(*tr.index_entries[0])["node_features/bsa"])  # noqa: SLF001
    np.testing.assert_allclose(x[:, col], ((np.log(bsa0 + 10) - tr.means["bsa"]) / tr.devs["bsa"]).astype(np.float32), rtol=1e-6)
    va = GraphDataset(path, train_source=tr, clustering_method="mcl")
    assert va.node_features == tr.node_features and va.target == "irmsd" and va.means == tr.means
    np.testing.assert_array_equal(va.get(0).x.numpy(), x)


def test_classification_task_and_classes(synth_file):
    ds = GraphDataset(synth_file[0], target="irmsd", task="classif", classes=[0, 1, 2])
    assert ds.task == "classif"  # an explicit task is kept (dataset.py:157-162)
    assert ds.classes_to_index == {0: 0, 1: 1, 2: 2}
    ds = GraphDataset(synth_file[0], target="irmsd")
    assert ds.task == "regress" and ds.classes is None


def test_collate_free_standing_batch():
    d1 = S.make_dataset(2, seed=3, n_lo=10, n_hi=12)
    from deeprank2_amd.data import Data

    datas = []
    for g in d1:
        ei, ea = S.doubled_edges(g)
        datas.append(Data(x=torch.from_numpy(g["x"]), edge_index=torch.from_numpy(ei), edge_attr=torch.from_numpy(ea), y=torch.tensor([1.0])))
    b = Batch.from_data_list(datas)
    c = collate(datas)
    assert torch.equal(b.edge_index, c["edge_index"]) and b.num_graphs == 2


# ---- the reference's fixtures, read in place -------------------------------


@needs_ref
def test_1atn_batch_equals_golden_inputs(golden):
    z = golden("ginet_1atn")
    ds = GraphDataset(f"{REF_H5}/1ATN_ppi.hdf5", node_features=DEFAULT_FEATURES, edge_features=["distance"], target="irmsd", clustering_method="mcl")
    b = next(iter(DataLoader(ds, batch_size=4)))
    for k in ("x", "edge_index", "edge_attr", "batch", "cluster0", "cluster1", "y"):
        np.testing.assert_array_equal(getattr(b, k).numpy(), z[f"in/{k}"], err_msg=k)


@needs_ref
def test_reference_dataset_assertions():
    """Reference tests/test_dataset.py:178-197, 348-368, 520-550."""
    p = f"{REF_H5}/1ATN_ppi.hdf5"
    ds = GraphDataset(p, node_features=DEFAULT_FEATURES, edge_features=["distance"], target="irmsd")
    assert len(ds) == 4 and ds[0] is not None
    with pytest.raises(IndexError):
        GraphDataset(p, node_features=DEFAULT_FEATURES, edge_features=["distance"], target="irmsd", target_filter={"irmsd": "<10"})
    assert len(GraphDataset(p, node_features=DEFAULT_FEATURES, edge_features=["distance"], target="irmsd", target_filter={"irmsd": ">15"})) == 3
    ds = GraphDataset(p, target="binary", node_features="all", edge_features="all")
    df = ds.hdf5_to_pandas()
    for j, feat in enumerate(ds.edge_features):
        vals = np.concatenate([ds.get(i).edge_attr[:, j].numpy() for i in range(len(ds))])
        ref = np.concatenate(df[feat].values)
        assert np.float32(round(vals.mean(), 2)) == np.float32(round(ref.mean(), 2)), feat
        assert np.float32(round(vals.std(), 2)) == np.float32(round(ref.std(), 2)), feat
    assert ds.task == "classif" and ds.classes == [0, 1]


@needs_ref
def test_test_hdf5_matches_foutnet_golden_inputs(golden):
    z = golden("foutnet_testhdf5")
    ds = GraphDataset(f"{REF_H5}/test.hdf5", node_features=DEFAULT_FEATURES, edge_features=["distance"], target="binary", clustering_method="mcl")
    b = next(iter(DataLoader(ds, batch_size=len(ds))))
    for k in ("x", "edge_index", "cluster0", "cluster1"):
        np.testing.assert_array_equal(getattr(b, k).numpy(), z[f"in/{k}"], err_msg=k)
