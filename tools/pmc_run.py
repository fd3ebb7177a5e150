"""Workload for rocprofv3 --pmc passes: eager GINet training steps (config 2).

    rocprofv3 --pmc <counters> -f csv -d <dir> -- python3 tools/pmc_run.py [steps] [ginet|vanilla|foutnet|sgat|ginet_nocluster][_atom|_mixed|_b<B>][_bf16]
"""

from __future__ import annotations

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deeprank-gnn-2_amd")]

from bench import make_graphs, records  # noqa: E402
from deeprank2_amd.engine import GINetTrainStep  # noqa: E402
from deeprank2_amd.neuralnets.gnn.ginet import BatchHandle, GINet  # noqa: E402
from deeprank2_amd.neuralnets.gnn.vanilla_gnn import VanillaNetwork  # noqa: E402
from deeprank2_amd.store import GraphStore, pack_graphs  # noqa: E402
from deeprank2_amd.utils.synthetic import make_dataset  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    dev = torch.device("cuda:0")
    which = sys.argv[2] if len(sys.argv) > 2 else "ginet"
    bf16 = which.endswith("_bf16")  # GINet bf16 compute (BASELINE configs[3]): the tile kernels for every graph
    which = which.removesuffix("_bf16")
    atom = which.endswith("_atom")  # B=32 atom-level graphs (the Vanilla pipeline / large paths)
    mixed = which.endswith("_mixed")  # B=64 configs[4] 50/30/20 residue/SRV/atom mix (bench.py --graphs mixed)
    which = which.removesuffix("_atom").removesuffix("_mixed")
    B, nb = (32, 4) if atom else (64, 4) if mixed else (64, 16)
    if "_b" in which:  # e.g. ginet_b4096: B residue graphs per step, two batches (the accumulating pass past the CU count)
        which, b = which.split("_b")
        B, nb = int(b), 2
    fam = {"n_lo": 2700, "n_hi": 3300, "mean_degree": 16.7, "k_lo": 8, "k_hi": 32} if atom else {}
    graphs = make_graphs("mixed", B * nb, seed=1000) if mixed else make_dataset(B * nb, seed=1000, **fam)
    packed = pack_graphs(records(graphs, 1 if which == "sgat" else 3), require_clusters=which not in ("ginet_nocluster", "vanilla"))
    store = GraphStore(packed, dev, dtype="bf16" if bf16 else "f32")
    order = np.random.default_rng(0).permutation(packed.n_graphs).astype(np.int32)
    hs = [BatchHandle(store, order[i * B:(i + 1) * B]) for i in range(nb)]
    torch.manual_seed(1234)
    if which in ("foutnet", "sgat"):
        from deeprank2_amd.neuralnets.gnn import foutnet, sgat  # noqa: PLC0415

        model = (sgat.SGAT(30, 1, 1) if which == "sgat" else foutnet.FoutNet(30, 1, 3)).to(dev).train()
    elif which == "ginet_nocluster":
        from deeprank2_amd.neuralnets.gnn import ginet_nocluster  # noqa: PLC0415

        model = ginet_nocluster.GINet(30, 1, 3).to(dev).train()
    else:
        model = (VanillaNetwork if which == "vanilla" else GINet)(30, 1, 3).to(dev).train()
    step = GINetTrainStep(model, compute_dtype="bf16" if bf16 else "f32")
    for i in range(steps):
        step.step(hs[i % nb])
    torch.cuda.synchronize()
    print("alg_bytes_per_launch", np.mean([__import__("bench").algorithmic_bytes(packed, h.gids_host, which, 2 if bf16 else 4) for h in hs]))


if __name__ == "__main__":
    main()
