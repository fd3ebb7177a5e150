"""Data-parallel path on CPU (gloo, world size 2): sharding helpers and the
gradient algebra FusedTrainStep relies on — per-rank loss scaled by
1/B_global + SUM all-reduce == the single-process step on the whole batch."""

from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from deeprank2_amd.distributed import plan_shards, shard_by_edges, shard_contiguous


def test_shard_contiguous_covers_in_order():
    g = np.arange(10, 27)
    parts = [shard_contiguous(g, r, 4) for r in range(4)]
    np.testing.assert_array_equal(np.concatenate(parts), g)
    assert max(p.size for p in parts) - min(p.size for p in parts) <= 1
    with pytest.raises(ValueError):
        shard_contiguous(g, 4, 4)


def test_shard_by_edges_balances_and_restores_order():
    rng = np.random.default_rng(0)
    gids = rng.permutation(200).astype(np.int32)
    edges = np.where(rng.random(200) < 0.2, rng.integers(40000, 60000, 200), rng.integers(150, 3500, 200))
    shards, perm = shard_by_edges(gids, edges, 8)
    np.testing.assert_array_equal(np.concatenate(shards)[perm], gids)
    e_of = dict(zip(gids.tolist(), edges.tolist()))
    loads = [sum(e_of[int(x)] for x in s) for s in shards]
    assert max(loads) - min(loads) <= edges.max()  # LPT bound
    assert max(loads) / (sum(loads) / 8) < 1.1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _mixed_graphs():
    """A small config-5-like global batch: residue, SRV-like and (scaled-down)
    large graphs in a shuffled order, so contiguous shards are edge-imbalanced."""
    from deeprank2_amd.utils.synthetic import make_dataset

    fams = [{"n_lo": 20, "n_hi": 40, "mean_degree": 6.0}] * 4 + [{"n_lo": 8, "n_hi": 12, "mean_degree": 3.0, "k_lo": 2, "k_hi": 3}] * 3 + [{"n_lo": 150, "n_hi": 220, "mean_degree": 14.0, "k_lo": 4, "k_hi": 8}] * 2
    order = [8, 0, 1, 7, 4, 2, 5, 3, 6]
    return [make_dataset(1, seed=50 + i, **fams[i])[0] for i in order]


def _rank_main(rank, world, port, model_name, out_path, graphs="small"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from deeprank2_amd.trainer import _gather_rows
    from deeprank2_amd.utils.synthetic import make_dataset
    from oracle import data_ref, gnn_ref
    from oracle import pyg_ops as P

    gs = _mixed_graphs() if graphs == "mixed" else make_dataset(6, seed=2, n_lo=20, n_hi=40, mean_degree=6.0)
    datas = [data_ref.synthetic_to_data(g, f"s{i}") for i, g in enumerate(gs)]
    b = len(datas)
    torch.manual_seed(0)
    model = gnn_ref.GINet(30, 1, 3) if model_name == "ginet" else gnn_ref.FoutNet(30, 1)
    model.eval()  # dropout off: the shards see the same arithmetic as the full batch
    plan = plan_shards([d.edge_index.shape[1] for d in datas], world)
    mine = plan.positions[rank]
    bat = P.Batch.from_data_list([datas[i].clone() for i in mine])
    out = model(bat)
    loss = ((out.reshape(-1) - bat.y) ** 2).sum() / b  # per-rank term of the global MSE mean
    loss.backward()
    flat = torch.cat([p.grad.reshape(-1) for p in model.parameters()] + [loss.detach().reshape(1)])
    dist.all_reduce(flat)
    rows = _gather_rows(out.detach(), plan, dist.group.WORLD)  # the exporter's rows, global order
    if rank == 0:
        full = P.Batch.from_data_list([d.clone() for d in datas])
        model.zero_grad()
        ref_out = model(full)
        ref_loss = torch.nn.functional.mse_loss(ref_out.reshape(-1), full.y)
        ref_loss.backward()
        ref = torch.cat([p.grad.reshape(-1) for p in model.parameters()] + [ref_loss.detach().reshape(1)])
        np.savez(out_path, ddp=flat.numpy(), ref=ref.numpy(), rows=rows.numpy(), ref_rows=ref_out.detach().numpy(), balanced=plan.balanced, loads=np.array(plan.loads))
    dist.destroy_process_group()


@pytest.mark.parametrize("model_name", ["ginet", "foutnet"])
def test_gloo_world2_allreduced_gradients_equal_global_batch(tmp_path, model_name):
    out = str(tmp_path / "g.npz")
    mp.spawn(_rank_main, args=(2, _free_port(), model_name, out), nprocs=2, join=True)
    z = np.load(out)
    assert not z["balanced"]  # equal-sized graphs: contiguous shards
    np.testing.assert_allclose(z["ddp"], z["ref"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(z["rows"], z["ref_rows"], rtol=1e-5, atol=1e-6)


def test_gloo_world2_mixed_batch_edge_balanced(tmp_path):
    """Config 5 on the CPU: a mixed batch is sharded by edge bin packing
    (contiguous shards would leave one rank with both large graphs), the
    all-reduced gradients equal the global batch's, and the gathered
    predictions come back in global-batch order."""
    out = str(tmp_path / "m.npz")
    mp.spawn(_rank_main, args=(2, _free_port(), "ginet", out, "mixed"), nprocs=2, join=True)
    z = np.load(out)
    assert z["balanced"]
    assert max(z["loads"]) < 1.25 * z["loads"].mean()
    np.testing.assert_allclose(z["ddp"], z["ref"], rtol=1e-5, atol=1e-5 * float(np.abs(z["ref"]).max()))
    np.testing.assert_allclose(z["rows"], z["ref_rows"], rtol=1e-5, atol=1e-6)


def test_plan_shards_policy():
    residue = np.full(64, 3000)
    p = plan_shards(residue, 8)
    assert not p.balanced and p.sizes() == [8] * 8
    np.testing.assert_array_equal(np.concatenate(p.positions), np.arange(64))
    rng = np.random.default_rng(1)
    mixed = np.where(rng.random(64) < 0.2, 50000, np.where(rng.random(64) < 0.4, 250, 3000))
    c = plan_shards(mixed, 8, policy="contiguous")
    a = plan_shards(mixed, 8)
    assert max(c.loads) > 1.25 * np.mean(c.loads) and a.balanced
    assert max(a.loads) < max(c.loads)
    np.testing.assert_array_equal(np.concatenate(a.positions)[a.perm], np.arange(64))
    for pos in a.positions:
        assert np.all(np.diff(pos) > 0)  # global order within a rank
    assert plan_shards(mixed, 1).sizes() == [64]
    e = plan_shards(np.array([10, 20]), 4)  # fewer graphs than ranks: empty shards
    assert sorted(e.sizes()) == [0, 0, 1, 1]
    with pytest.raises(ValueError):
        plan_shards(mixed, 2, policy="random")


class _FakeDataset:
    def __init__(self, n, entries=None):
        self.entries = list(range(n)) if entries is None else entries

    def __len__(self):
        return len(self.entries)

    def subset_entries(self, idx):
        return _FakeDataset(0, [self.entries[i] for i in idx])


def _trainer_rank_main(rank, world, port, out_path):
    """Trainer's data-parallel bookkeeping on one rank: the validation split and
    every epoch's order come from rank 0 (the ranks' RNGs are seeded apart on
    purpose), and the contiguous shards of each global batch cover it once."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from deeprank2_amd.loader import DataLoader
    from deeprank2_amd.trainer import _divide_dataset

    pg = dist.group.WORLD
    torch.manual_seed(100 + rank)
    main, split = _divide_dataset(_FakeDataset(23), splitsize=0.25, process_group=pg)
    dl = DataLoader(main, batch_size=4, shuffle=True, process_group=pg)
    epochs = []
    for _ in range(3):
        seen = []
        for idx in dl.batches():
            seen.append(shard_contiguous(np.asarray(idx), rank, world).tolist())
        epochs.append(seen)
    box = [None] * world
    dist.all_gather_object(box, {"main": main.entries, "split": split.entries, "epochs": epochs})
    if rank == 0:
        import json

        with open(out_path, "w") as f:
            json.dump(box, f)
    dist.destroy_process_group()


def test_gloo_world2_trainer_split_and_epoch_order_from_rank0(tmp_path):
    import json

    out = str(tmp_path / "t.json")
    mp.spawn(_trainer_rank_main, args=(2, _free_port(), out), nprocs=2, join=True)
    r0, r1 = json.load(open(out))
    assert r0["main"] == r1["main"] and r0["split"] == r1["split"]
    assert sorted(r0["main"] + r0["split"]) == list(range(23))
    for e0, e1 in zip(r0["epochs"], r1["epochs"]):
        visited = [i for b0, b1 in zip(e0, e1) for i in b0 + b1]
        assert sorted(visited) == list(range(len(r0["main"])))  # every graph once per epoch
    assert r0["epochs"][0] != r0["epochs"][1]  # reshuffled per epoch


class _EpochDS:
    """A dataset stand-in for Trainer._epoch: graph g has loss term g, one edge."""

    def __init__(self, n):
        self.index_entries = [("f", f"g{i}") for i in range(n)]

    def __len__(self):
        return len(self.index_entries)

    def edge_counts(self, idx):
        return np.ones(len(idx), dtype=np.int64)

    def _targets_of(self, idx):
        return torch.zeros(len(idx))

    def targets_host(self):
        return np.zeros(len(self), dtype=np.float32)

    def entry_names(self, idx):
        return [self.index_entries[i][1] for i in idx]

    def batch_handle(self, local, dev):
        return np.asarray(local)


class _StubStep:
    """FusedTrainStep stand-in: a step's loss slot is this rank's share of the
    global batch mean (sum of its graphs' terms / global batch), as the fused
    step's 1/B_global loss scale gives; the all-reduce is a gloo SUM."""

    def __init__(self, pg):
        self.pg = pg

    def step(self, local, global_batch):
        t = torch.tensor([float(np.sum(local)) / global_batch])
        torch.distributed.all_reduce(t, group=self.pg)
        return t, torch.as_tensor(np.asarray(local, dtype=np.float32)).reshape(-1, 1)

    def step_empty(self):
        t = torch.zeros(1)
        torch.distributed.all_reduce(t, group=self.pg)
        return t, torch.zeros(0, 1)

    def check_faults(self):
        pass


class _StubRunner:
    """EpochRunner stand-in: per-step local loss terms into the epoch's vector."""

    def __init__(self, sizes, global_sizes):
        self.sizes, self.global_sizes = sizes, global_sizes

    def run(self, local_batches):
        losses = torch.tensor([float(np.sum(lo)) / g for lo, g in zip(local_batches, self.global_sizes)])
        pred = torch.as_tensor(np.concatenate([np.asarray(lo, dtype=np.float32) for lo in local_batches])).reshape(-1, 1)
        return losses, pred


def _captured_epoch_rank_main(rank, world, port, out_path):
    """Trainer._epoch on one rank of a world-2 gloo group with stub step/runner
    (ADVICE r05): the captured epoch's loss weights each rank-summed step loss
    by the GLOBAL batch size, and a global batch that leaves some rank an
    empty shard sends EVERY rank to the per-batch loop."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import deeprank2_amd.trainer as T

    pg = dist.group.WORLD
    calls = []

    def fake_runner_for(step, store, sizes, cache, global_sizes=None):
        calls.append(list(sizes))
        return _StubRunner(list(sizes), list(global_sizes))

    T.runner_for = fake_runner_for

    class _Exp:
        def process(self, *a):
            self.last = a

    class _Fake:
        _epoch = T.Trainer._epoch
        _epoch_captured = T.Trainer._epoch_captured
        _shard = T.Trainer._shard
        _format_output = T.Trainer._format_output
        _export_pred = T.Trainer._export_pred
        _host_targets = T.Trainer._host_targets
        _shard_epoch = T.Trainer._shard_epoch

    res = {}
    for name, batches in (("captured", [[0, 1, 2, 3, 4], [5, 6, 7]]), ("trailing1", [[0, 1, 2, 3, 4], [5, 6, 7], [8]])):
        f = _Fake()
        f.device, f.task, f.process_group, f.shard_policy = torch.device("cpu"), T.REGRESS, pg, "contiguous"
        f.capture_epochs, f._runners = True, {}
        f.dataset_train = _EpochDS(9)
        f.train_loader = type("L", (), {"batches": staticmethod(lambda b=batches: b)})()
        step = _StubStep(pg)
        f._fused_step = lambda s=step: s
        f._fused = step
        f._targets_for_kernel = lambda ds, dev: None
        f._output_exporters = _Exp()
        calls.clear()
        loss = f._epoch(1, "training")
        res[name] = {"loss": loss, "runner_calls": len(calls), "preds": f._output_exporters.last[3]}
    box = [None] * world
    dist.all_gather_object(box, res)
    if rank == 0:
        import json

        with open(out_path, "w") as fh:
            json.dump(box, fh)
    dist.destroy_process_group()


def test_gloo_world2_captured_epoch_loss_and_eligibility(tmp_path):
    import json

    out = str(tmp_path / "e.json")
    mp.spawn(_captured_epoch_rank_main, args=(2, _free_port(), out), nprocs=2, join=True)
    r0, r1 = json.load(open(out))
    # unequal shards (3/2 and 2/1): the epoch loss is the mean of the 8 graphs' terms on both ranks
    for r in (r0, r1):
        assert r["captured"]["runner_calls"] == 1
        assert r["captured"]["loss"] == pytest.approx(np.mean(np.arange(8)), rel=1e-6)
        assert r["captured"]["preds"] == [float(i) for i in range(8)]
    # a trailing batch of 1 at world 2: no rank captures; the loop gives the same loss on both
    for r in (r0, r1):
        assert r["trailing1"]["runner_calls"] == 0
        assert r["trailing1"]["loss"] == pytest.approx(np.mean(np.arange(9)), rel=1e-6)
        assert r["trailing1"]["preds"] == [float(i) for i in range(9)]
