"""Diagnostic: timeline of the pipelined GINet step (dr_ginet_piped_step) from
the stamps build (s_memrealtime, one 100 MHz clock for the whole chip).

    DR_LIB_NAME=libdeeprank2_amd_stamps.so python tools/piped_stamps.py [B] [steps]

Per launch, relative to the earliest block start (us): pass blocks' start, the
first wave's wait start / end (the update it waits for), block end; reducers'
start, reduce-loop end, drained, block end.  Medians over blocks, then over
the last steps.  The stamps build is never used for timing claims.
"""

from __future__ import annotations

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deeprank-gnn-2_amd")]
os.environ.setdefault("DR_LIB_NAME", "libdeeprank2_amd_stamps.so")

from bench import make_graphs, records  # noqa: E402
from deeprank2_amd.engine import FusedTrainStep  # noqa: E402
from deeprank2_amd.fused import BatchHandle  # noqa: E402
from deeprank2_amd.neuralnets.gnn.ginet import GINet  # noqa: E402
from deeprank2_amd.store import GraphStore, pack_graphs  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    dev = torch.device("cuda:0")
    nb = 8
    packed = pack_graphs(records(make_graphs("residue", B * nb, seed=1000)))
    store = GraphStore(packed, dev)
    hs = [BatchHandle(store, np.arange(k * B, (k + 1) * B, dtype=np.int32)) for k in range(nb)]
    torch.manual_seed(1234)
    model = GINet(30, 1, 3).to(dev).train()
    step = FusedTrainStep(model)
    step.piped = True
    nr = step._reduce_nr()  # noqa: SLF001
    stamps = torch.zeros((B + nr) * 32, dtype=torch.int64, device=dev)
    for p in (step._pass, step._pass_nodrop):  # noqa: SLF001
        p.stamps = stamps.data_ptr()
    rows = []
    for i in range(steps):
        stamps.zero_()
        step.step(hs[i % nb])
        torch.cuda.synchronize()
        st = stamps.view(B + nr, 32).cpu().numpy().astype(np.float64)
        t0 = st[:, 24][st[:, 24] > 0].min()
        rel = lambda a: (a - t0) / 100.0  # noqa: E731  (100 MHz ticks -> us)
        pas, red = st[:B], st[B:]
        row = {
            "pass_start": np.median(rel(pas[:, 24])),
            "wait_start": np.median(rel(pas[:, 28])) if (pas[:, 28] > 0).any() else float("nan"),
            "wait_end": np.median(rel(pas[:, 29])) if (pas[:, 29] > 0).any() else float("nan"),
            "pass_end": np.median(rel(pas[:, 27])),
            "pass_end_max": rel(pas[:, 27]).max(),
            "red_start": np.median(rel(red[:, 24])),
            "red_start_max": rel(red[:, 24]).max(),
            "red_loop_end": np.median(rel(red[:, 25])) if (red[:, 25] > 0).any() else float("nan"),
            "red_drained_max": rel(red[:, 26]).max() if (red[:, 26] > 0).any() else float("nan"),
            "red_end_max": rel(red[:, 27]).max(),
        }
        rows.append(row)
    print(f"B={B} reducers={nr}  (us from the first block start; median over blocks, then over the last {steps - 10} steps)")
    for k in rows[0]:
        print(f"  {k:16s} {np.median([r[k] for r in rows[10:]]):8.2f}")


if __name__ == "__main__":
    main()
