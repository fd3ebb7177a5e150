"""Diagnostic: one GINet training step's timeline across its two launches
(stamps build: s_memrealtime, the 100 MHz chip clock, so blocks on different
CUs compare): graph-pass blocks' entry / exit, then the reduce + Adam blocks'
entry, partials summed, barrier, stores issued, stores done.  Steps are
replayed from one captured HIP graph of K steps (as bench.py's timed region);
the stamps show the last step.

    DR_LIB_NAME=libdeeprank2_amd_stamps.so python tools/step_timeline.py [B] [K]
"""

from __future__ import annotations

import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deeprank-gnn-2_amd")]
os.environ.setdefault("DR_LIB_NAME", "libdeeprank2_amd_stamps.so")

from bench import records  # noqa: E402
from deeprank2_amd import _lib  # noqa: E402
from deeprank2_amd.engine import GINetTrainStep  # noqa: E402
from deeprank2_amd.neuralnets.gnn import ginet as amd  # noqa: E402
from deeprank2_amd.store import GraphStore, pack_graphs  # noqa: E402
from deeprank2_amd.utils.synthetic import make_dataset  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    store = GraphStore(pack_graphs(records(make_dataset(B * 4, seed=1000))), dev)
    hs = [amd.BatchHandle(store, np.arange(i * B, (i + 1) * B)) for i in range(4)]
    torch.manual_seed(1234)
    model = amd.GINet(30, 1, 3).to(dev).train()
    step = GINetTrainStep(model)
    st = torch.zeros(B * 32, dtype=torch.int64, device=dev)
    for p in (step._pass, step._pass_nodrop):  # noqa: SLF001
        p.stamps = st.data_ptr()
    lib = _lib.load()
    fn = lib.dr_debug_reduce_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    for i in range(4):
        step.step(hs[i % 4])
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(K):
            step.step(hs[i % 4])
    g.replay()
    torch.cuda.synchronize()
    rows = []
    for _rep in range(20):
        st.zero_()
        g.replay()
        torch.cuda.synchronize()
        s = st.view(B, 32).cpu().numpy()
        nblk = 512
        host = np.zeros(nblk * 8, dtype=np.int64)
        assert fn(host.ctypes.data, host.size) == 0
        r = host.reshape(nblk, 8)
        live = r[:, 0] > 0
        r = r[live]
        t0 = s[:, 30].min()
        ms = lambda v: (v - t0) * 0.01  # noqa: E731  (100 MHz ticks -> us)
        rows.append([ms(s[:, 30].max()), ms(np.median(s[:, 31])), ms(s[:, 31].max()), ms(r[:, 0].min()), ms(np.median(r[:, 0])), ms(r[:, 0].max()), ms(np.median(r[:, 5])), ms(r[:, 5].max()), ms(np.median(r[:, 1])), ms(r[:, 1].max()), ms(r[:, 2].max()), ms(r[:, 3].max()), ms(r[:, 4].max())])
    names = ["pass last block entry", "pass median exit", "pass last exit", "reduce first entry", "reduce median entry", "reduce last entry", "reduce median record in", "reduce last record in", "reduce median partials summed", "reduce last partials summed", "reduce last past barrier", "reduce last stores issued", "reduce last stores done"]
    med = np.median(np.array(rows), 0)
    print(f"B={B}, one HIP graph of {K} steps, the last step's timeline (us from the first pass block's entry; median of {len(rows)} replays):")
    for n, v in zip(names, med):
        print(f"  {n:34s} {v:7.2f}")
    print(f"  reduce blocks: {int(live.sum())}")


if __name__ == "__main__":
    main()
