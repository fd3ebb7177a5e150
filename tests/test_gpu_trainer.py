"""Trainer end to end on the GPU against an oracle replay of the reference's
training loop (trainer.py:503-724): same batches, same Adam/SGD, same losses."""

from __future__ import annotations

import numpy as np
import pytest
import torch
from torch import nn

from deeprank2_amd.dataset import GraphDataset
from deeprank2_amd.exporters import MemoryOutputExporter
from deeprank2_amd.neuralnets.gnn.foutnet import FoutNet
from deeprank2_amd.neuralnets.gnn.ginet import GINet
from deeprank2_amd.neuralnets.gnn.ginet_nocluster import GINet as GINetNoCluster
from deeprank2_amd.neuralnets.gnn.sgat import SGAT
from deeprank2_amd.trainer import Trainer
from deeprank2_amd.utils import synthetic as S
from oracle import gnn_ref
from oracle import pyg_ops as P

pytestmark = pytest.mark.gpu


def _connected_clusters(n, seed):
    """Graphs whose every depth-0 cluster has a pooled edge (FoutNet's conv2
    turns an isolated pooled node into NaN, foutnet.py:58; keep those out of a
    loss-trajectory comparison)."""
    out, s = [], seed
    while len(out) < n:
        for g in S.make_dataset(4 * n, seed=s, n_lo=25, n_hi=60, mean_degree=8.0):
            c = g["cluster0"][g["index"]]
            cross = c[:, 0] != c[:, 1]
            if np.unique(c[cross]).size == int(g["cluster0"].max()) + 1 and len(out) < n:
                out.append(g)
        s += 1000
    return out


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    d = tmp_path_factory.mktemp("trg")
    tr, va = str(d / "train.hdf5"), str(d / "valid.hdf5")
    S.write_hdf5(tr, _connected_clusters(24, 11), prefix="tr")
    S.write_hdf5(va, _connected_clusters(8, 12), prefix="va")
    ctr, cva = str(d / "ctrain.hdf5"), str(d / "cvalid.hdf5")
    S.write_hdf5(ctr, S.make_dataset(24, seed=13, n_lo=25, n_hi=60, task="classif"), prefix="ctr", target="binary")
    S.write_hdf5(cva, S.make_dataset(8, seed=14, n_lo=25, n_hi=60, task="classif"), prefix="cva", target="binary")
    return tr, va, ctr, cva


def _sets(tr_path, va_path, target="irmsd", edge_features=S.SYNTH_EDGE_FEATURES):
    tr = GraphDataset(tr_path, node_features=S.SYNTH_NODE_FEATURES, edge_features=edge_features, target=target, clustering_method="mcl")
    return tr, GraphDataset(va_path, train_source=tr, clustering_method="mcl")


def _oracle_batch(ds, idx):
    datas = []
    for i in idx:
        d = ds.get(i)
        o = P.Data(x=d.x, edge_index=d.edge_index, edge_attr=d.edge_attr, y=d.y, pos=d.pos)
        o.cluster0, o.cluster1 = d.cluster0, d.cluster1
        datas.append(o)
    return P.Batch.from_data_list(datas)


def _losses(mem, phase):
    return [r["loss"] for r in mem.records if r["phase"] == phase]


def _replay(model_o, opt, tr, va, nepoch, bs):
    """The reference loop on the oracle: epoch-0 evals, then train/validate per epoch."""
    losses = {"training": [], "validation": []}

    def ev(ds):
        model_o.eval()
        tot, n = 0.0, 0
        with torch.no_grad():
            for s in range(0, len(ds), bs):
                b = _oracle_batch(ds, range(s, min(s + bs, len(ds))))
                out = model_o(b).reshape(-1)
                tot += float(nn.functional.mse_loss(out, b.y)) * out.shape[0]
                n += out.shape[0]
        return tot / n

    losses["training"].append(ev(tr))
    losses["validation"].append(ev(va))
    for _ in range(nepoch):
        model_o.train()
        tot, n = 0.0, 0
        for s in range(0, len(tr), bs):
            b = _oracle_batch(tr, range(s, min(s + bs, len(tr))))
            opt.zero_grad()
            out = model_o(b).reshape(-1)
            loss = nn.functional.mse_loss(out, b.y)
            loss.backward()
            opt.step()
            tot += float(loss.detach()) * out.shape[0]
            n += out.shape[0]
        losses["training"].append(tot / n)
        losses["validation"].append(ev(va))
    return losses


def test_foutnet_trainer_adam_matches_oracle_replay(files):
    tr, va = _sets(files[0], files[1])
    mem = MemoryOutputExporter()
    torch.manual_seed(4)
    t = Trainer(FoutNet, tr, va, cuda=True, output_exporters=[mem], precluster=False)  # keep the connected k-means clusters
    model_o = gnn_ref.FoutNet(30, 1)
    model_o.load_state_dict({k: v.cpu() for k, v in t.model.state_dict().items()})
    t.train(nepoch=3, batch_size=8, shuffle=False, validate=True, best_model=False, filename=None)
    assert t._fused  # noqa: SLF001  (the fused path ran)
    assert np.isfinite(_losses(mem, "training")).all()
    ref = _replay(model_o, torch.optim.Adam(model_o.parameters(), lr=1e-3, weight_decay=1e-5), tr, va, 3, 8)
    np.testing.assert_allclose(_losses(mem, "training"), ref["training"], rtol=2e-4)
    np.testing.assert_allclose(_losses(mem, "validation"), ref["validation"], rtol=2e-4)
    for n, p in model_o.named_parameters():
        mine = t.model.state_dict()[n].cpu().numpy()
        assert np.mean(np.abs(mine - p.detach().numpy()) < 1e-5) > 0.97, n
    # checkpoint optimizer state is torch Adam's
    sd = t.optimizer.state_dict()
    assert int(float(sd["state"][0]["step"])) == 9


def test_foutnet_trainer_sgd_generic_path_matches_oracle(files):
    tr, va = _sets(files[0], files[1])
    mem = MemoryOutputExporter()
    torch.manual_seed(5)
    t = Trainer(FoutNet, tr, va, cuda=True, output_exporters=[mem], precluster=False)  # keep the connected k-means clusters
    t.configure_optimizers(torch.optim.SGD, lr=0.01, weight_decay=0.0)
    model_o = gnn_ref.FoutNet(30, 1)
    model_o.load_state_dict({k: v.cpu() for k, v in t.model.state_dict().items()})
    t.train(nepoch=2, batch_size=8, shuffle=False, validate=True, best_model=False, filename=None)
    assert not t._fused  # noqa: SLF001
    ref = _replay(model_o, torch.optim.SGD(model_o.parameters(), lr=0.01, weight_decay=0.0), tr, va, 2, 8)
    np.testing.assert_allclose(_losses(mem, "training"), ref["training"], rtol=2e-4)
    for n, p in model_o.named_parameters():
        np.testing.assert_allclose(t.model.state_dict()[n].cpu().numpy(), p.detach().numpy(), rtol=1e-4, atol=1e-5, err_msg=n)


def test_ginet_classification_class_weights_checkpoint_and_test(files, tmp_path):
    tr, va = _sets(files[2], files[3], target="binary")
    mem = MemoryOutputExporter()
    t = Trainer(GINet, tr, va, class_weights=True, cuda=True, output_exporters=[mem])
    path = str(tmp_path / "ginet.pth.tar")
    t.train(nepoch=3, batch_size=8, validate=True, filename=path)
    assert t._fused and t.weights is not None  # noqa: SLF001
    tl = _losses(mem, "training")
    assert len(tl) == 4 and all(np.isfinite(tl))
    last = [r for r in mem.records if r["phase"] == "training"][-1]
    np.testing.assert_allclose(np.array(last["output"]).sum(1), 1.0, rtol=1e-5)
    state = torch.load(path, weights_only=True)
    # as in the reference (trainer.py:628-631) the snapshot is taken before
    # epoch_saved_model is updated, so the file holds the previous best epoch
    # (None when the kept model is the first one saved)
    assert set(state["model_state"]) == set(t.model.state_dict())
    vl = [r["loss"] for r in mem.records if r["phase"] == "validation"][1:]
    saves = [e for e in range(1, len(vl) + 1) if min(vl[:e]) == vl[e - 1]]
    assert state["epoch_saved_model"] == (saves[-2] if len(saves) > 1 else None)
    assert t.epoch_saved_model == saves[-1]
    te = GraphDataset(files[3], train_source=path, clustering_method="mcl")
    mem2 = MemoryOutputExporter()
    t2 = Trainer(GINet, dataset_test=te, pretrained_model=path, cuda=True, output_exporters=[mem2])
    t2.test(batch_size=4)
    t.dataset_test = va
    mem.records.clear()
    t.test(batch_size=8)
    np.testing.assert_allclose(np.array(mem2.records[0]["output"]), np.array(mem.records[0]["output"]), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize(("model_cls", "acc"), [(GINet, False), (FoutNet, False), (SGAT, False), (GINetNoCluster, False), (GINet, True)])
def test_captured_epochs_bit_identical_to_per_batch_steps(files, model_cls, acc):
    """Trainer epochs replayed from one captured HIP graph (epoch.py) against
    the per-batch loop: the same epoch losses, exported outputs and final
    parameters, bit for bit (shuffled batches, a last partial batch, GINet's
    in-kernel dropout).  acc: every step on the accumulating pass over 2
    workgroups (what batches past the CU count take), prefetch layout on."""
    from deeprank2_amd import trainer as trainer_mod
    from deeprank2_amd.engine import FusedTrainStep

    res = []
    for captured in (True, False):
        # SGAT multiplies its one edge feature into every channel (sgat.py:71)
        tr, va = _sets(files[0], files[1], edge_features=S.SYNTH_EDGE_FEATURES[:1] if model_cls is SGAT else S.SYNTH_EDGE_FEATURES)
        mem = MemoryOutputExporter()
        torch.manual_seed(21)
        trainer_mod.Trainer.capture_epochs = captured
        if acc:
            FusedTrainStep.acc_default, FusedTrainStep.acc_groups_default = True, 2
        try:
            t = Trainer(model_cls, tr, va, cuda=True, output_exporters=[mem], precluster=False)
            t.train(nepoch=3, batch_size=5, shuffle=True, validate=True, best_model=False, filename=None)
        finally:
            trainer_mod.Trainer.capture_epochs = True
            FusedTrainStep.acc_default = FusedTrainStep.acc_groups_default = None
        assert t._fused  # noqa: SLF001
        assert bool(t._runners) == captured  # noqa: SLF001  (the captured path ran)
        assert (t._fused._acc_slab is not None) == acc  # noqa: SLF001  (the accumulating pass ran)
        res.append((mem.records, {k: v.detach().cpu() for k, v in t.model.state_dict().items()}))
    (ra, pa), (rb, pb) = res
    assert [r["loss"] for r in ra] == [r["loss"] for r in rb]
    assert [r["output"] for r in ra] == [r["output"] for r in rb]
    assert [r["entry"] for r in ra] == [r["entry"] for r in rb]
    for k in pa:
        assert torch.equal(pa[k], pb[k]), k
