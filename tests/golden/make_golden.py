"""Generate the golden vectors in ``tests/golden/*.npz`` from the REFERENCE itself.

Runs only in the build container (it needs ``/root/reference`` and the conda
interpreter with h5py); the fixtures it writes are plain data and travel with
the repo.  Nothing else in the repo imports the reference.

What it does:

1. dumps the reference HDF5 fixtures (``tests/data/hdf5/{1ATN_ppi,test}.hdf5``)
   to ``.npz`` with ``deeprank2_amd/io/h5extract.py`` under
   ``/opt/conda/bin/python3.9`` (h5py is only installed there);
2. imports ``deeprank2.neuralnets.gnn.{ginet,foutnet,vanilla_gnn}`` and
   ``deeprank2.utils.community_pooling`` from ``/root/reference`` with the
   stand-ins in ``tests/golden/refshim`` for the absent PyG / torch_scatter
   (they forward to ``oracle/pyg_ops.py``: that boundary stays unpinned);
3. runs the reference modules forward (eval, and train with a fixed dropout
   mask) and backward (MSE / CE losses) on seeded weights and stores inputs,
   weights, outputs, losses and every parameter gradient.

Usage: ``python tests/golden/make_golden.py [siblings|nonfinite|pretrained]``
(from the repo root; ``siblings`` regenerates only the SGAT / ginet_nocluster
fixtures, ``nonfinite`` only the non-finite-input GINet fixtures,
``pretrained`` only the reference's pre-trained VanillaNetwork on test.hdf5).
"""

from __future__ import annotations

import os
import subprocess
import sys
import tempfile

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = "/root/reference"
HERE = os.path.join(ROOT, "tests", "golden")
sys.path[:0] = [ROOT, os.path.join(ROOT, "deeprank-gnn-2_amd"), os.path.join(HERE, "refshim"), REF]

from deeprank2.neuralnets.gnn import foutnet as ref_fout  # noqa: E402
from deeprank2.neuralnets.gnn import ginet as ref_ginet  # noqa: E402
from deeprank2.neuralnets.gnn import ginet_nocluster as ref_ginet_nc  # noqa: E402
from deeprank2.neuralnets.gnn import sgat as ref_sgat  # noqa: E402
from deeprank2.neuralnets.gnn import vanilla_gnn as ref_vanilla  # noqa: E402
from deeprank2.utils import community_pooling as ref_cp  # noqa: E402

from deeprank2_amd.utils.synthetic import make_dataset  # noqa: E402
from oracle import data_ref  # noqa: E402
from oracle import pyg_ops as P  # noqa: E402

DEFAULT_FEATURES = ["res_type", "polarity", "bsa", "res_depth", "hse", "info_content", "pssm"]  # tests/test_trainer.py:31-39


def dump_hdf5(name):
    out = os.path.join(tempfile.gettempdir(), f"golden_{name}.npz")
    script = os.path.join(ROOT, "deeprank-gnn-2_amd", "deeprank2_amd", "io", "h5extract.py")
    subprocess.run(["/opt/conda/bin/python3.9", script, out, f"{REF}/tests/data/hdf5/{name}.hdf5"], check=True)
    return data_ref.read_dump(out)


def batch_to_arrays(batch, prefix="in/"):
    out = {}
    for k in ("x", "edge_index", "edge_attr", "batch", "cluster0", "cluster1", "y", "pos"):
        v = getattr(batch, k, None)
        if isinstance(v, torch.Tensor):
            out[prefix + k] = v.detach().numpy()
    out[prefix + "ptr"] = batch.ptr.numpy()
    return out


def fixed_dropout(mask):
    def _drop(x, p, training):
        if not training:
            return x
        return x * mask / (1.0 - p)

    return _drop


def run_model(model, batch, loss_kind, mask=None, module=None):
    """eval output, then train output + loss + grads with a fixed dropout mask."""
    rec = {}
    model.eval()
    with torch.no_grad():
        rec["out/eval"] = model(batch.clone()).numpy()
    model.train()
    if mask is not None:
        module.dropout = fixed_dropout(mask)
    model.zero_grad()
    out = model(batch.clone())
    if loss_kind == "mse":
        loss = torch.nn.functional.mse_loss(out.reshape(-1), batch.y)
    else:
        loss = torch.nn.functional.cross_entropy(out, batch.y.long())
    loss.backward()
    rec["out/train"] = out.detach().numpy()
    rec["loss"] = np.array(loss.item(), dtype=np.float64)
    for n, p in model.named_parameters():
        rec["param/" + n] = p.detach().numpy().copy()
        rec["grad/" + n] = (p.grad if p.grad is not None else torch.zeros_like(p)).numpy().copy()
        rec["hasgrad/" + n] = np.array(p.grad is not None)
    return rec


def save(name, rec, meta):
    for k, v in meta.items():
        rec["meta/" + k] = np.array(v)
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **rec)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB)")


def synthetic_batch(n, seed, **kw):
    graphs = make_dataset(n, seed=seed, **kw)
    return [data_ref.synthetic_to_data(g, f"syn{seed}_{i}") for i, g in enumerate(graphs)]


def twist_clusters(datas):
    """Exercise the cluster paths the fixtures never hit: non-consecutive
    depth-0 ids and a depth-1 level with more than one cluster."""
    d = datas[0]
    ids = torch.unique(d.cluster0)
    remap = {int(v): 3 * i for i, v in enumerate(ids)}  # 0,3,6,...
    d.cluster0 = torch.tensor([remap[int(v)] for v in d.cluster0])
    k = len(ids)
    d.cluster1 = torch.tensor([i % 2 for i in range(k)], dtype=torch.long)
    if len(datas) > 2:
        e = datas[2]
        k2 = len(e.cluster1)
        e.cluster1 = torch.tensor([(i * 7) % 3 for i in range(k2)], dtype=torch.long)
        e.cluster1 = torch.unique(e.cluster1, return_inverse=True)[1]
    return datas


def isolate_node(d, node):
    keep = (d.edge_index[0] != node) & (d.edge_index[1] != node)
    d.edge_index = d.edge_index[:, keep]
    d.edge_attr = d.edge_attr[keep]
    return d


def main():  # noqa: PLR0915
    torch.set_num_threads(4)
    dump = dump_hdf5("1ATN_ppi")
    names = list(dump)

    def atn_data(idx, node_features=DEFAULT_FEATURES):
        return [data_ref.load_one_graph(dump[names[i]], names[i], node_features, ["distance"], target="irmsd", clustering_method="mcl") for i in idx]

    # ---- GINet on the reference fixture (config 1 of BASELINE.json) ----
    torch.manual_seed(1234)
    model = ref_ginet.GINet(50, 1, 1)
    b4 = P.Batch.from_data_list(atn_data(range(4)))
    g = torch.Generator().manual_seed(7)
    mask = (torch.rand(4, 128, generator=g) >= 0.4).float()
    rec = batch_to_arrays(b4)
    rec.update(run_model(model, b4, "mse", mask, ref_ginet))
    rec["mask"] = mask.numpy()
    with torch.no_grad():
        model.eval()
        rec["out/eval_b1"] = np.concatenate([model(P.Batch.from_data_list(atn_data([i]))).numpy() for i in range(4)])
    save("ginet_1atn", rec, {"F": 50, "Fe": 1, "out": 1, "loss": "mse", "source": "tests/data/hdf5/1ATN_ppi.hdf5 default_features+distance, mcl"})

    # ---- GINet on a synthetic batch with twisted clusters / isolated node ----
    for tag, out_dim, loss in (("regress", 1, "mse"), ("classif", 2, "ce")):
        torch.manual_seed(99 if tag == "regress" else 98)
        datas = twist_clusters(synthetic_batch(5, seed=3 if tag == "regress" else 4, n_lo=40, n_hi=70, mean_degree=10.0))
        isolate_node(datas[1], 5)
        if tag == "classif":
            for i, d in enumerate(datas):
                d.y = torch.tensor([float(i % 2)])
        bat = P.Batch.from_data_list(datas)
        model = ref_ginet.GINet(30, out_dim, 3)
        mask = (torch.rand(5, 128, generator=torch.Generator().manual_seed(11)) >= 0.4).float()
        rec = batch_to_arrays(bat)
        rec.update(run_model(model, bat, loss, mask, ref_ginet))
        rec["mask"] = mask.numpy()
        save(f"ginet_synth_{tag}", rec, {"F": 30, "Fe": 3, "out": out_dim, "loss": loss, "source": "deeprank2_amd.utils.synthetic, twisted clusters, node 5 of graph 1 isolated"})

    # ---- GINetConvLayer alone on an arbitrary (asymmetric, self-loop, duplicate) edge list ----
    torch.manual_seed(5)
    layer = ref_ginet.GINetConvLayer(12, 16, 2)
    gen = torch.Generator().manual_seed(5)
    x = torch.randn(37, 12, generator=gen, requires_grad=True)
    ei = torch.randint(0, 37, (2, 300), generator=gen)
    ei[:, :5] = torch.tensor([[3, 3, 3, 9, 9], [3, 3, 4, 9, 1]])  # self loops + duplicates
    ea = torch.randn(300, 2, generator=gen)
    z = layer(x, ei, ea)
    gz = torch.randn(z.shape, generator=gen)
    (z * gz).sum().backward()
    rec = {"in/x": x.detach().numpy(), "in/edge_index": ei.numpy(), "in/edge_attr": ea.numpy(), "in/gz": gz.numpy(), "out/z": z.detach().numpy(), "grad/x": x.grad.numpy()}
    for n, p in layer.named_parameters():
        rec["param/" + n] = p.detach().numpy().copy()
        rec["grad/" + n] = (p.grad if p.grad is not None else torch.zeros_like(p)).numpy().copy()
    save("ginet_conv_layer", rec, {"in": 12, "out": 16, "Fe": 2})

    # ---- community_pooling + get_preloaded_cluster on the 1ATN batch ----
    b = P.Batch.from_data_list(atn_data(range(4)))
    c = ref_cp.get_preloaded_cluster(b.cluster0.clone(), b.batch)
    pooled = ref_cp.community_pooling(c, b)
    rec = batch_to_arrays(b)
    rec.update({"out/cluster_offset": c.numpy(), "out/x": pooled.x.numpy(), "out/edge_index": pooled.edge_index.numpy(), "out/edge_attr": pooled.edge_attr.numpy(), "out/batch": pooled.batch.numpy(), "out/pos": pooled.pos.numpy()})
    save("community_pooling_1atn", rec, {"source": "1ATN_ppi mcl depth_0"})

    # ---- FoutNet: synthetic (finite) and the reference's test.hdf5 (NaN rows) ----
    torch.manual_seed(21)
    model = ref_fout.FoutNet(30, 1)
    bat = P.Batch.from_data_list(twist_clusters(synthetic_batch(3, seed=8, n_lo=26, n_hi=36, mean_degree=8.0)))
    rec = batch_to_arrays(bat)
    rec.update(run_model(model, bat, "mse"))
    save("foutnet_synth", rec, {"F": 30, "out": 1, "loss": "mse"})

    dump_t = dump_hdf5("test")
    tn = list(dump_t)
    datas = [data_ref.load_one_graph(dump_t[n], n, DEFAULT_FEATURES, ["distance"], target="binary", clustering_method="mcl", task="classif") for n in tn]
    bat = P.Batch.from_data_list(datas)
    torch.manual_seed(22)
    model = ref_fout.FoutNet(50, 2)
    model.eval()
    rec = batch_to_arrays(bat)
    with torch.no_grad():
        rec["out/eval"] = model(bat.clone()).numpy()
    for n, p in model.named_parameters():
        rec["param/" + n] = p.detach().numpy().copy()
    save("foutnet_testhdf5", rec, {"F": 50, "out": 2, "source": "tests/data/hdf5/test.hdf5 (1 cluster/graph: NaN path)"})

    # ---- VanillaNetwork ----
    torch.manual_seed(31)
    model = ref_vanilla.VanillaNetwork(30, 1, 3)
    bat = P.Batch.from_data_list(synthetic_batch(3, seed=9, n_lo=40, n_hi=60, mean_degree=10.0))
    rec = batch_to_arrays(bat)
    rec.update(run_model(model, bat, "mse"))
    save("vanilla_synth", rec, {"F": 30, "Fe": 3, "out": 1, "loss": "mse"})


PRETRAINED = f"{REF}/tests/data/pretrained/testing_graph_model.pth.tar"


def main_pretrained():
    """The reference's pre-trained VanillaNetwork (tests/data/pretrained/
    testing_graph_model.pth.tar, read with the inert opcode reader of
    deeprank2_amd.io.checkpoint: nothing from the file runs) on the reference's
    test.hdf5, the graphs loaded as GraphDataset(test.hdf5, train_source=<that
    checkpoint>) loads them (dataset.py:85-131 inheritance: its node / edge
    features, transforms and the stored means / devs; load_one_graph restated in
    oracle/data_ref): eval outputs as Trainer.test() computes them
    (trainer.py:836-872), plus a CE loss and every gradient."""
    from deeprank2_amd.io.checkpoint import load_checkpoint, transform_from_source  # noqa: PLC0415

    st = load_checkpoint(PRETRAINED)
    ft = {k: {"transform": transform_from_source(v["transform"]) if isinstance(v.get("transform"), str) else v.get("transform"), "standardize": v.get("standardize")} for k, v in st["features_transform"].items()}
    means = {k: float(v) for k, v in st["means"].items()}
    devs = {k: float(v) for k, v in st["devs"].items()}
    dump_t = dump_hdf5("test")
    tn = list(dump_t)
    datas = [data_ref.load_one_graph(dump_t[n], n, st["node_features"], st["edge_features"], target=st["target"], features_transform=ft, means=means, devs=devs, task=st["task"]) for n in tn]
    bat = P.Batch.from_data_list(datas)
    f, fe = bat.x.shape[1], bat.edge_attr.shape[1]
    model = ref_vanilla.VanillaNetwork(f, len(st["classes"]), fe)
    model.load_state_dict(st["model_state"])
    rec = batch_to_arrays(bat)
    rec.update(run_model(model, bat, "ce"))
    save("vanilla_pretrained_testhdf5", rec, {"F": f, "Fe": fe, "out": len(st["classes"]), "loss": "ce", "source": "tests/data/pretrained/testing_graph_model.pth.tar on tests/data/hdf5/test.hdf5 (train_source inheritance)", "node_features": st["node_features"], "edge_features": st["edge_features"]})


def main_siblings():
    """SGAT (sgat.py) and ginet_nocluster.GINet goldens."""
    torch.set_num_threads(4)
    dump = dump_hdf5("1ATN_ppi")
    names = list(dump)
    atn = [data_ref.load_one_graph(dump[n], n, DEFAULT_FEATURES, ["distance"], target="irmsd", clustering_method="mcl") for n in names[:4]]

    # ---- SGAT on the reference fixture (Fe = 1: sgat.py:71 broadcasts edge_attr over the channels) ----
    torch.manual_seed(4321)
    model = ref_sgat.SGAT(50, 1)
    bat = P.Batch.from_data_list([d.clone() for d in atn])
    rec = batch_to_arrays(bat)
    rec.update(run_model(model, bat, "mse"))
    save("sgat_1atn", rec, {"F": 50, "Fe": 1, "out": 1, "loss": "mse", "source": "tests/data/hdf5/1ATN_ppi.hdf5 default_features+distance, mcl"})

    # ---- SGAT, synthetic: twisted clusters, an isolated node (empty scatter_mean row), CE ----
    torch.manual_seed(77)
    datas = twist_clusters(synthetic_batch(5, seed=13, n_lo=40, n_hi=70, mean_degree=10.0))
    for d in datas:
        d.edge_attr = d.edge_attr[:, :1].contiguous()
    isolate_node(datas[1], 5)
    for i, d in enumerate(datas):
        d.y = torch.tensor([float(i % 2)])
    bat = P.Batch.from_data_list(datas)
    model = ref_sgat.SGAT(30, 2)
    rec = batch_to_arrays(bat)
    rec.update(run_model(model, bat, "ce"))
    save("sgat_synth", rec, {"F": 30, "Fe": 1, "out": 2, "loss": "ce", "source": "deeprank2_amd.utils.synthetic, edge_attr[:, :1], twisted clusters, node 5 of graph 1 isolated"})

    # ---- SGraphAttentionLayer alone (arbitrary edges; undirected and directed forms) ----
    for tag, undirected in (("", True), ("_directed", False)):
        torch.manual_seed(6)
        layer = ref_sgat.SGraphAttentionLayer(12, 16, undirected=undirected)
        gen = torch.Generator().manual_seed(6)
        x = torch.randn(41, 12, generator=gen, requires_grad=True)
        ei = torch.randint(0, 40, (2, 260), generator=gen)  # node 40 has no edges
        ei[:, :5] = torch.tensor([[3, 3, 3, 9, 9], [3, 3, 4, 9, 1]])
        ea = torch.rand(260, generator=gen) + 0.5  # 1-D: sgat.py:65 unsqueezes
        z = layer(x, ei, ea)
        gz = torch.randn(z.shape, generator=gen)
        (z * gz).sum().backward()
        rec = {"in/x": x.detach().numpy(), "in/edge_index": ei.numpy(), "in/edge_attr": ea.numpy(), "in/gz": gz.numpy(), "out/z": z.detach().numpy(), "grad/x": x.grad.numpy()}
        for n, p in layer.named_parameters():
            rec["param/" + n] = p.detach().numpy().copy()
            rec["grad/" + n] = p.grad.numpy().copy()
        save(f"sgat_layer{tag}", rec, {"in": 12, "out": 16, "undirected": undirected})

    # ---- ginet_nocluster.GINet: 1ATN (MSE, fixed dropout mask) and synthetic CE ----
    torch.manual_seed(555)
    model = ref_ginet_nc.GINet(50, 1, 1)
    bat = P.Batch.from_data_list([d.clone() for d in atn])
    mask = (torch.rand(4, 128, generator=torch.Generator().manual_seed(8)) >= 0.4).float()
    rec = batch_to_arrays(bat)
    rec.update(run_model(model, bat, "mse", mask, ref_ginet_nc))
    rec["mask"] = mask.numpy()
    save("ginet_nocluster_1atn", rec, {"F": 50, "Fe": 1, "out": 1, "loss": "mse", "source": "tests/data/hdf5/1ATN_ppi.hdf5 default_features+distance"})
    torch.manual_seed(556)
    datas = synthetic_batch(5, seed=17, n_lo=40, n_hi=70, mean_degree=10.0)
    isolate_node(datas[2], 3)
    for i, d in enumerate(datas):
        d.y = torch.tensor([float(i % 3)])
    bat = P.Batch.from_data_list(datas)
    model = ref_ginet_nc.GINet(30, 3, 3)
    mask = (torch.rand(5, 128, generator=torch.Generator().manual_seed(9)) >= 0.4).float()
    rec = batch_to_arrays(bat)
    rec.update(run_model(model, bat, "ce", mask, ref_ginet_nc))
    rec["mask"] = mask.numpy()
    save("ginet_nocluster_synth", rec, {"F": 30, "Fe": 3, "out": 3, "loss": "ce", "source": "deeprank2_amd.utils.synthetic, node 3 of graph 2 isolated"})


def poison_edge(d, cross):
    """Set edge_attr to +inf on both directions of one residue pair whose ends
    lie in different (cross=True) or the same depth-0 cluster."""
    ei, c0 = d.edge_index, d.cluster0
    same = c0[ei[0]] == c0[ei[1]]
    pick = int(torch.nonzero(~same if cross else (same & (ei[0] != ei[1])))[0])
    i, j = int(ei[0, pick]), int(ei[1, pick])
    both = ((ei[0] == i) & (ei[1] == j)) | ((ei[0] == j) & (ei[1] == i))
    d.edge_attr = d.edge_attr.clone()
    d.edge_attr[both, 0] = float("inf")
    return d


def main_nonfinite():
    """GINet / ginet_nocluster / GINetConvLayer with non-finite inputs: the
    reference's singleton softmax turns a non-finite attention logit into NaN
    (ginet.py:48-54); which outputs and gradients end up NaN is decided by the
    depth-0 scatter_max (drops NaN rows) and max_pool_x (propagates them)."""
    torch.set_num_threads(4)
    datas = synthetic_batch(5, seed=23, n_lo=40, n_hi=70, mean_degree=10.0)
    poison_edge(datas[0], cross=True)  # pooled edge inf -> conv2 row NaN -> graph 0 output NaN
    poison_edge(datas[1], cross=False)  # intra-cluster: conv1 rows NaN, dropped by scatter_max
    datas[2].x = datas[2].x.clone()
    datas[2].x[7, 3] = float("nan")  # node 7 and the rows that gather it
    for tag, sel in (("all", [0, 1, 2, 3, 4]), ("conv1", [1, 2, 3, 4])):
        torch.manual_seed(71)
        model = ref_ginet.GINet(30, 1, 3)
        bat = P.Batch.from_data_list([datas[i].clone() for i in sel])
        mask = (torch.rand(len(sel), 128, generator=torch.Generator().manual_seed(12)) >= 0.4).float()
        rec = batch_to_arrays(bat)
        rec.update(run_model(model, bat, "mse", mask, ref_ginet))
        rec["mask"] = mask.numpy()
        save(f"ginet_nonfinite_{tag}", rec, {"F": 30, "Fe": 3, "out": 1, "loss": "mse", "source": f"synthetic seed 23 graphs {sel}: inf edge_attr across clusters (g0), within a cluster (g1), NaN x (g2)"})
    torch.manual_seed(72)
    model = ref_ginet_nc.GINet(30, 1, 3)
    bat = P.Batch.from_data_list([datas[i].clone() for i in (2, 3)])
    mask = (torch.rand(2, 128, generator=torch.Generator().manual_seed(13)) >= 0.4).float()
    rec = batch_to_arrays(bat)
    rec.update(run_model(model, bat, "mse", mask, ref_ginet_nc))
    rec["mask"] = mask.numpy()
    save("ginet_nocluster_nonfinite", rec, {"F": 30, "Fe": 3, "out": 1, "loss": "mse", "source": "synthetic seed 23 graphs [2, 3]: NaN x on node 7 of the first"})
    torch.manual_seed(73)
    layer = ref_ginet.GINetConvLayer(12, 16, 2)
    gen = torch.Generator().manual_seed(14)
    x = torch.randn(30, 12, generator=gen, requires_grad=True)
    ei = torch.randint(0, 30, (2, 200), generator=gen)
    ea = torch.randn(200, 2, generator=gen)
    ea[17, 1] = float("-inf")
    z = layer(x, ei, ea)
    gz = torch.randn(z.shape, generator=gen)
    (z * gz).sum().backward()
    rec = {"in/x": x.detach().numpy(), "in/edge_index": ei.numpy(), "in/edge_attr": ea.numpy(), "in/gz": gz.numpy(), "out/z": z.detach().numpy(), "grad/x": x.grad.numpy()}
    for n, p in layer.named_parameters():
        rec["param/" + n] = p.detach().numpy().copy()
        rec["grad/" + n] = p.grad.numpy().copy()
    save("ginet_conv_layer_nonfinite", rec, {"in": 12, "out": 16, "Fe": 2})


if __name__ == "__main__":
    if sys.argv[1:] == ["siblings"]:
        main_siblings()
    elif sys.argv[1:] == ["pretrained"]:
        main_pretrained()
    elif sys.argv[1:] == ["nonfinite"]:
        main_nonfinite()
    else:
        main()
        main_siblings()
        main_nonfinite()
