"""One rank of the data-parallel parity test (tests/test_gpu_distributed.py).

Launched as a child process per rank (RANK / WORLD_SIZE / MASTER_* in the
environment); every rank uses the same GPU over the gloo backend, so the test
fits a one-GPU box while exercising FusedTrainStep's sharded step and its
single all-reduce.  DR_DDP_PG=nccl runs one rank over RCCL instead (the
bench's N>1 launch path on one GPU) and DR_DDP_CAPTURE=1 replays every step
from a captured HIP graph (all-reduce included).  Writes the final parameters
(rank 0).  DR_DDP_EMULATE=n (one process, no group): each global batch's n
shards run one after another, their gradient buffers summed in rank order
(what the all-reduce computes), then one Adam update; for n = 2 the same
bits as two ranks, since a two-operand sum does not depend on the order.
DR_DDP_GRAPHS=mixed: global batches of residue, SRV and atom-level graphs
(config 5), sharded by ``plan_shards`` (edge-balanced); rank 0 also writes the
last step's predictions gathered back into global-batch order (the Trainer's
``_gather_rows``).  DR_DDP_ACC=1: GINet's accumulating pass (3 workgroups)."""

from __future__ import annotations

import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "deeprank-gnn-2_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from deeprank2_amd.distributed import plan_shards  # noqa: E402
from deeprank2_amd.engine import FusedTrainStep  # noqa: E402
from deeprank2_amd.fused import BatchHandle  # noqa: E402
from deeprank2_amd.neuralnets.gnn.foutnet import FoutNet  # noqa: E402
from deeprank2_amd.neuralnets.gnn.ginet import GINet  # noqa: E402
from deeprank2_amd.neuralnets.gnn.vanilla_gnn import VanillaNetwork  # noqa: E402
from deeprank2_amd.store import GraphStore, pack_graphs, records_from_batch  # noqa: E402
from deeprank2_amd.utils.synthetic import make_dataset  # noqa: E402
from oracle import data_ref  # noqa: E402
from oracle import pyg_ops as P  # noqa: E402

B, STEPS = 24, 3


def run(model_name, world, rank, out_path):
    dev = torch.device("cuda:0")
    pg = None
    backend = os.environ.get("DR_DDP_PG", "gloo")
    if world > 1 or backend == "nccl":
        if backend == "nccl":
            torch.cuda.set_device(dev)
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        pg = dist.group.WORLD
    capture = os.environ.get("DR_DDP_CAPTURE") == "1"
    mixed = os.environ.get("DR_DDP_GRAPHS") == "mixed"
    if mixed:  # 2 x B graphs: 12 residue, 7 SRV-like, 5 atom-level per global batch
        fams = [{}] * 12 + [{"n_lo": 26, "n_hi": 36, "mean_degree": 7.4, "k_lo": 2, "k_hi": 3}] * 7 + [{"n_lo": 2700, "n_hi": 3300, "mean_degree": 16.7, "k_lo": 8, "k_hi": 32}] * 5
        order = np.random.default_rng(5).permutation(2 * B)
        graphs = [make_dataset(1, seed=100 + i, **fams[i % B])[0] for i in order]
    else:
        graphs = make_dataset(2 * B, seed=17, n_lo=30, n_hi=80, mean_degree=9.0)
    datas = [data_ref.synthetic_to_data(g, f"s{i}") for i, g in enumerate(graphs)]
    store = GraphStore(pack_graphs(records_from_batch(P.Batch.from_data_list(datas))), dev)
    edges = np.array([d.edge_index.shape[1] for d in datas])
    torch.manual_seed(42)
    model = {"ginet": lambda: GINet(30, 1, 3), "foutnet": lambda: FoutNet(30, 1), "vanilla": lambda: VanillaNetwork(30, 1, 3)}[model_name]().to(dev).train()
    if os.environ.get("DR_DDP_ACC") == "1":  # the accumulating pass on 3 workgroups per shard
        FusedTrainStep.acc_default, FusedTrainStep.acc_groups_default = True, 3
    step = FusedTrainStep(model, process_group=pg)
    emulate = int(os.environ.get("DR_DDP_EMULATE", "0"))
    if emulate:
        step.pg, step.world = "emulated", emulate
        acc = []

        def all_reduce(t, group=None):  # noqa: ARG001
            acc.append(t.clone() if not acc else acc[-1] + t)
            t.copy_(acc[-1])

        dist.all_reduce = all_reduce
        adam = step._adam_after_allreduce  # noqa: SLF001
    losses, loads = [], []
    out_global = None
    for s in range(STEPS):
        gids = np.arange(B) + (s % 2) * B  # global batch, global order
        plan = plan_shards(edges[gids], max(world, emulate), policy="edges" if mixed else "contiguous")
        loads.append(plan.loads)
        if emulate:
            acc.clear()
            out_global = np.zeros((B, 1), np.float32)
            for r in range(emulate):
                step._adam_after_allreduce = adam if r == emulate - 1 else (lambda: None)  # noqa: SLF001
                loss, out = step.step(BatchHandle(store, gids[plan.positions[r]]), global_batch=B, dropout=False)
                out_global[plan.positions[r]] = out.cpu().numpy()
            losses.append(float(loss))
            continue
        h = BatchHandle(store, gids[plan.positions[rank]])
        if capture:
            g = step.capture(h, global_batch=B, dropout=False)
            g.replay()
            loss, out = step.loss_out, step.out[: h.B]
        else:
            loss, out = step.step(h, global_batch=B, dropout=False)
        losses.append(float(loss))
        if pg is not None and world > 1:
            from deeprank2_amd.trainer import _gather_rows  # noqa: PLC0415

            out_global = _gather_rows(out.clone(), plan, pg).cpu().numpy()
        else:
            out_global = out.cpu().numpy()
    torch.cuda.synchronize()
    if rank == 0:
        np.savez(out_path, loss=np.array(losses), grad=step.flat_grad.cpu().numpy(), out=out_global, loads=np.array(loads), **{f"p{i}": p.detach().cpu().numpy() for i, p in enumerate(step.params)})
    if pg is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    run(sys.argv[1], int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), sys.argv[2])
