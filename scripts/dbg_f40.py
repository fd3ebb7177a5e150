import sys, os
sys.path[:0] = ['/root/repo', '/root/repo/deeprank-gnn-2_amd', '/root/repo/tests']
import numpy as np, torch
from deeprank2_amd.engine import FusedTrainStep
from deeprank2_amd.fused import BatchHandle
from deeprank2_amd.neuralnets.gnn import ginet as amd
from deeprank2_amd.store import GraphStore, pack_graphs
from deeprank2_amd.utils.synthetic import make_dataset
from bench import records
DEV = "cuda:0"
f, n = 40, 300
store = GraphStore(pack_graphs(records(make_dataset(max(n, 64), seed=41, n_feat=f))), DEV)
rng = np.random.default_rng(4)
h = BatchHandle(store, rng.permutation(max(n, 64))[:n].astype(np.int32))
res = {}
for rep in range(3):
    for mode in ("acc", "per"):
        torch.manual_seed(5)
        m = amd.GINet(f, 1, 3).to(DEV).train(); m._drop_seed = 777
        st = FusedTrainStep(m, max_batch=64); st.acc = mode == "acc"
        l, o = st.step(h); torch.cuda.synchronize()
        res[(mode, rep)] = o.clone()
for k, v in res.items(): print(os.environ.get("DR_LIB_NAME", "main"), k, float(v.abs().sum()), torch.equal(v, res[("per", 0)]))
