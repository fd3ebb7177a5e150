"""Diagnostic: host-side profile (cProfile) of the drop-in Trainer's captured
training epoch and evaluation (bench.py --trainer's workload, smaller).

    python tools/trainer_profile.py [graphs] [ddp]
"""

from __future__ import annotations

import cProfile
import os
import pstats
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deeprank-gnn-2_amd")]

import torch  # noqa: E402

from bench import _free_port, make_graphs  # noqa: E402
from deeprank2_amd.dataset import GraphDataset  # noqa: E402
from deeprank2_amd.exporters import MemoryOutputExporter  # noqa: E402
from deeprank2_amd.neuralnets.gnn.ginet import GINet  # noqa: E402
from deeprank2_amd.trainer import Trainer  # noqa: E402
from deeprank2_amd.utils import synthetic as S  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    ddp = len(sys.argv) > 2 and sys.argv[2] == "ddp"
    dev = torch.device("cuda:0")
    if ddp:
        torch.cuda.set_device(dev)
        torch.distributed.init_process_group("nccl", device_id=dev, init_method=f"tcp://127.0.0.1:{_free_port()}", world_size=1, rank=0)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "train.hdf5")
        S.write_hdf5(path, make_graphs("residue", n, seed=1000))
        ds = GraphDataset(path, node_features=S.SYNTH_NODE_FEATURES, edge_features=S.SYNTH_EDGE_FEATURES, target="irmsd", clustering_method="mcl")
        torch.manual_seed(1234)
        tr = Trainer(GINet, ds, cuda=True, output_exporters=[MemoryOutputExporter()], precluster=False, ngpu=2 if ddp else 0)
        tr.train(nepoch=1, batch_size=64, shuffle=True, best_model=False, filename=None, validate=True)  # warm-up
        for name, fn in (("epoch", lambda: tr._epoch(1, "training")), ("eval", lambda: tr._eval(tr.valid_loader, 1, "validation"))):  # noqa: SLF001
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(10):
                fn()
            torch.cuda.synchronize()
            print(f"{name}: {(time.perf_counter() - t) / 10 * 1e6:.1f} us per call")
            pr = cProfile.Profile()
            pr.enable()
            for _ in range(10):
                fn()
            torch.cuda.synchronize()
            pr.disable()
            pstats.Stats(pr).sort_stats("tottime").print_stats(25)
    if ddp:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
