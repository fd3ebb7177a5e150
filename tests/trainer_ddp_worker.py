"""One process of the captured data-parallel epoch test
(tests/test_gpu_distributed.py::test_trainer_ddp_captured_epochs_bit_identical).

``Trainer(GINet, ..., ngpu=2)`` on a one-rank RCCL process group (the
``ngpu > 1`` code path on one GPU: shards, the all-reduce per step, the
predictions gathered into global order), trained for 3 epochs with validation.
DR_TRAINER_CAPTURE=1 replays each epoch from one captured HIP graph (the RCCL
all-reduce inside it, the loss vector all-reduced and the predictions gathered
once per epoch); 0 runs the per-batch loop.  Writes the exporter records and the
final parameters to an .npz.

    python tests/trainer_ddp_worker.py <train.hdf5> <valid.hdf5> <out.npz>
"""

from __future__ import annotations

import os
import socket
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "deeprank-gnn-2_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from deeprank2_amd import trainer as trainer_mod  # noqa: E402
from deeprank2_amd.dataset import GraphDataset  # noqa: E402
from deeprank2_amd.exporters import MemoryOutputExporter  # noqa: E402
from deeprank2_amd.neuralnets.gnn.ginet import GINet  # noqa: E402
from deeprank2_amd.utils import synthetic as S  # noqa: E402


def main():
    tr_path, va_path, out = sys.argv[1:4]
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    trainer_mod.Trainer.capture_epochs = os.environ.get("DR_TRAINER_CAPTURE", "1") == "1"
    tr = GraphDataset(tr_path, node_features=S.SYNTH_NODE_FEATURES, edge_features=S.SYNTH_EDGE_FEATURES, target="irmsd", clustering_method="mcl")
    va = GraphDataset(va_path, train_source=tr, clustering_method="mcl")
    mem = MemoryOutputExporter()
    torch.manual_seed(21)
    t = trainer_mod.Trainer(GINet, tr, va, cuda=True, ngpu=2, output_exporters=[mem], precluster=False)
    t.train(nepoch=3, batch_size=5, shuffle=True, validate=True, best_model=False, filename=None)
    assert t.process_group is not None and t._fused  # noqa: SLF001
    kinds = [k[0] == "eval" if isinstance(k, tuple) else False for k in t._runners]  # noqa: SLF001
    res = {
        "captured_train": np.array(any(not k for k in kinds)),
        "captured_eval": np.array(any(kinds)),
        "loss": np.array([r["loss"] for r in mem.records], dtype=np.float64),
        "phase": np.array([r["phase"] for r in mem.records]),
    }
    for i, r in enumerate(mem.records):
        res[f"out{i}"] = np.asarray(r["output"], dtype=np.float64)
        res[f"entry{i}"] = np.asarray(r["entry"])
    for k, v in t.model.state_dict().items():
        res[f"p_{k}"] = v.detach().cpu().numpy()
    np.savez(out, **res)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
