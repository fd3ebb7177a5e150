"""Trainer host logic on CPU (no kernels run): construction, task/loss rules,
dataset splitting, early stopping, checkpoint format."""

from __future__ import annotations

import numpy as np
import pytest
import torch
from torch import nn

from deeprank2_amd.dataset import GraphDataset
from deeprank2_amd.exporters import MemoryOutputExporter
from deeprank2_amd.neuralnets.gnn.foutnet import FoutNet
from deeprank2_amd.neuralnets.gnn.ginet import GINet
from deeprank2_amd.trainer import Trainer, _divide_dataset
from deeprank2_amd.utils import synthetic as S
from deeprank2_amd.utils.earlystopping import EarlyStopping


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    d = tmp_path_factory.mktemp("tr")
    tr, va = str(d / "train.hdf5"), str(d / "valid.hdf5")
    S.write_hdf5(tr, S.make_dataset(12, seed=1, n_lo=20, n_hi=30, mean_degree=6.0), prefix="tr")
    S.write_hdf5(va, S.make_dataset(4, seed=2, n_lo=20, n_hi=30, mean_degree=6.0), prefix="va")
    return tr, va


def _sets(files, target="irmsd", **kw):
    tr = GraphDataset(files[0], node_features=S.SYNTH_NODE_FEATURES, edge_features=S.SYNTH_EDGE_FEATURES, target=target, clustering_method="mcl", **kw)
    va = GraphDataset(files[1], train_source=tr, clustering_method="mcl")
    return tr, va


def test_builds_model_like_the_reference(files):
    tr, va = _sets(files)
    t = Trainer(GINet, tr, va, output_exporters=[MemoryOutputExporter()])
    assert isinstance(t.model, GINet) and t.output_shape == 1
    assert t.model.conv1.fc.weight.shape == (16, 30) and t.model.conv1.fc_edge_attr.weight.shape == (3, 3)  # neuralnet(F, out, Fe)
    assert isinstance(t.optimizer, torch.optim.Adam) and isinstance(t.lossfunction, nn.MSELoss)
    assert t.lr == 0.001 and t.weight_decay == 1e-05


def test_loss_rules(files):
    tr, va = _sets(files)
    t = Trainer(FoutNet, tr, va, output_exporters=[MemoryOutputExporter()])
    with pytest.raises(ValueError, match="not appropriate"):
        t.set_lossfunction(nn.CrossEntropyLoss)
    t.set_lossfunction(nn.L1Loss)
    with pytest.raises(ValueError, match="not appropriate"):
        t.set_lossfunction(nn.CTCLoss)
    t.set_lossfunction(nn.CTCLoss, override_invalid=True)


def test_requires_train_source_and_target(files):
    tr, _ = _sets(files)
    loose = GraphDataset(files[1], node_features=S.SYNTH_NODE_FEATURES, edge_features=S.SYNTH_EDGE_FEATURES, target="irmsd", clustering_method="mcl")
    with pytest.raises(ValueError, match="train_source"):
        Trainer(GINet, tr, loose)
    with pytest.raises(ValueError, match="at least a train or test"):
        Trainer(GINet)


def test_divide_dataset(files):
    tr, _ = _sets(files)
    a, b = _divide_dataset(tr, 0.25)
    assert len(a) == 9 and len(b) == 3
    assert sorted(a.index_entries + b.index_entries) == sorted(tr.index_entries)
    with pytest.raises(ValueError):
        _divide_dataset(tr, 12)
    t = Trainer(GINet, tr, output_exporters=[MemoryOutputExporter()])  # no validation set: 25 % split off
    assert len(t.dataset_val) == 3 and len(t.dataset_train) == 9


def test_classification_output_shape(files):
    tr = GraphDataset(files[0], node_features=S.SYNTH_NODE_FEATURES, edge_features=S.SYNTH_EDGE_FEATURES, target="irmsd", task="classif", classes=[0, 1, 2], clustering_method="mcl")
    t = Trainer(GINet, tr, val_size=3, output_exporters=[MemoryOutputExporter()])
    assert t.output_shape == 3 and isinstance(t.lossfunction, nn.CrossEntropyLoss)


def test_checkpoint_is_weights_only_loadable(files, tmp_path):
    tr, va = _sets(files, features_transform={"bsa": {"transform": lambda t: np.log(t + 10), "standardize": True}})
    t = Trainer(GINet, tr, va, output_exporters=[MemoryOutputExporter()])
    t.epoch_saved_model = 0
    ck = t._save_model()  # noqa: SLF001
    assert ck["features_transform"]["bsa"]["transform"].startswith("lambda t: np.log(t + 10)")
    path = str(tmp_path / "m.pth.tar")
    torch.save(ck, path)
    state = torch.load(path, weights_only=True)
    assert state["optimizer"] == "Adam" and state["lossfunction"] == "MSELoss" and state["data_type"] == "GraphDataset"
    test_set = GraphDataset(files[1], train_source=path, clustering_method="mcl")
    assert test_set.node_features == tr.node_features and test_set.means == tr.means
    t2 = Trainer(GINet, dataset_test=test_set, pretrained_model=path, output_exporters=[MemoryOutputExporter()])
    for k, v in t.model.state_dict().items():
        assert torch.equal(t2.model.state_dict()[k].cpu(), v.cpu()), k


def test_early_stopping_rules():
    es = EarlyStopping(patience=2, verbose=False, trace_func=lambda *_: None)
    for e, v in enumerate([1.0, 0.9, 0.95, 0.96], 1):
        es(e, v)
    assert es.early_stop
    es = EarlyStopping(patience=10, maxgap=0.1, min_epoch=1, trace_func=lambda *_: None)
    es(1, 1.0, 0.5)
    assert not es.early_stop
    es(2, 1.0, 0.5)
    assert es.early_stop


def _stop_epoch(**kw):
    """Known answers of the reference's tests/utils/test_earlystopping.py
    (its loss sequences; min_epoch=0)."""
    val = [3, 2, 1, 2, 0.5, 2, 3, 4, 5, 6, 7]
    train = [3, 2, 1, 2, 0.5, 2, 3, 4, 5, 1, 7]
    es = EarlyStopping(min_epoch=0, trace_func=lambda *_: None, **kw)
    for ep, v in enumerate(val):
        es(ep, v, train[ep])
        if es.early_stop:
            return ep
    return None


def test_early_stopping_reference_known_answers():
    assert _stop_epoch(patience=3) == 7
    assert _stop_epoch(patience=3, delta=1) == 5
    assert _stop_epoch(maxgap=1) == 9


def test_early_stopping_nan_loss_as_reference():
    """A NaN validation loss (reference earlystopping.py:47-70 on the negated
    score): not a stall, resets the run, best_score becomes NaN, and the next
    finite epoch counts as progress whatever its value."""
    es = EarlyStopping(patience=2, verbose=False, trace_func=lambda *_: None)
    es(1, 1.0)
    es(2, 2.0)
    assert es.counter == 1
    es(3, float("nan"))
    assert es.counter == 0 and es.best_score != es.best_score and es.val_loss_min == 1.0
    es(4, 5.0)  # worse than 1.0, still progress after the NaN epoch
    assert es.counter == 0 and es.best_score == -5.0 and es.val_loss_min == 5.0
    es(5, 6.0)
    es(6, 7.0)
    assert es.early_stop
    es = EarlyStopping(patience=2, verbose=False, trace_func=lambda *_: None)
    es(1, float("nan"))  # a NaN first epoch
    es(2, 3.0)
    assert es.counter == 0 and es.val_loss_min == 3.0
