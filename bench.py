"""Benchmark: GINet residue-PPI training step on MI355X (BASELINE.json configs[1]).

One step = one mini-batch of 64 synthetic residue-PPI graphs (~200 nodes,
~3k directed edges, 30 node features, 3 edge features) through forward,
MSE loss, backward and Adam — the loop body of ``Trainer._epoch``
(reference ``deeprank2/trainer.py:682-690``) — with the whole synthetic dataset
already resident in HBM (a mini-batch is a list of graph ids).

    python bench.py [--gpus N --steps K --warmup W]

N>1: one rank per GPU over RCCL, one global batch of 64*N graphs per step
(weak scaling), the same global batch sequence on every rank (same seed), each
rank training on its shard of it (``distributed.plan_shards``: contiguous
shards, or edge-balanced bin packing when that split is imbalanced, as for
config 5's mixed residue/SRV/atom batches) with one gradient all-reduce per
step.  Under
torch.distributed.run (WORLD_SIZE set) this process is one rank; otherwise
``--gpus N`` starts ``torch.distributed.run --nproc-per-node N bench.py ...`` as
a child process before anything touches the GPU and relays its output.
Rank 0 prints one JSON line.
"""

from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deeprank-gnn-2_amd")]

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
B_PER_GPU = 64
B_PER_GPU_FOR = {"residue": 64, "mixed": 64, "atom": 32}  # the default per-GPU batch of each workload (pmc_run.py's)
MODEL_NAMES = ("foutnet", "ginet", "ginet_nocluster", "sgat", "vanilla")
ORACLE_MODELS = {"ginet": "GINet", "foutnet": "FoutNet", "vanilla": "VanillaNetwork", "sgat": "SGAT", "ginet_nocluster": "GINetNoCluster"}
# graph families of SURVEY §8(d): residue-PPI (configs 2/3), atom-level (config 4), SRV-like
FAMILIES = {
    "residue": {},
    "atom": {"n_lo": 2700, "n_hi": 3300, "mean_degree": 16.7, "k_lo": 8, "k_hi": 32},
    "srv": {"n_lo": 26, "n_hi": 36, "mean_degree": 7.4, "k_lo": 2, "k_hi": 3},
}
WORKLOADS = {
    ("ginet", "residue"): "GINet residue-PPI training step, BASELINE.json configs[1]",
    ("foutnet", "residue"): "FoutNet residue-PPI training step, BASELINE.json configs[2]",
    ("ginet", "atom"): "GINet atom-level training step, BASELINE.json configs[3] (per-GPU share: 32 of 256)",
    ("ginet", "mixed"): "GINet mixed residue/SRV/atom batch, BASELINE.json configs[4] shape",
    ("vanilla", "mixed"): "VanillaNetwork (fused gather+edge MLP+scatter) mixed residue/SRV/atom batch, BASELINE.json configs[4]",
    ("vanilla", "residue"): "VanillaNetwork residue-PPI training step, configs[1] graph shape",
    ("foutnet", "mixed"): "FoutNet mixed residue/SRV/atom batch, configs[4] graph mix",
    ("sgat", "residue"): "SGAT residue-PPI training step (1 edge feature), configs[1] graph shape",
    ("ginet_nocluster", "residue"): "ginet_nocluster.GINet residue-PPI training step, configs[1] graph shape",
}
HEADLINE_METRIC = "graphs/sec + edges/sec per training step, GINet residue-PPI, 1/2/4/8 MI355X"


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def relaunch(n, argv):
    """``--gpus N`` outside torch.distributed.run: start N ranks as a child
    process (nothing in this process has touched the GPU; only stdlib modules
    are imported so far), stream its output through, exit with its code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    for line in proc.stdout:
        sys.stdout.write(line)
        sys.stdout.flush()
    return proc.wait()


def make_graphs(kind, n, seed):
    """Synthetic dataset of one family, or config 5's 50/30/20 residue/SRV/atom mix."""
    import numpy as np  # noqa: PLC0415

    from deeprank2_amd.utils.synthetic import make_dataset  # noqa: PLC0415

    if kind != "mixed":
        return make_dataset(n, seed=seed, **FAMILIES[kind])
    from deeprank2_amd.utils.synthetic import connect_clusters  # noqa: PLC0415

    rng = np.random.default_rng(seed)
    fam = rng.choice(["residue", "srv", "atom"], size=n, p=[0.5, 0.3, 0.2])
    # no pooled node without out-edges (FoutNet's NaN rows): the mix trains
    return [connect_clusters(make_dataset(1, seed=int(seed * 7919 + i), **FAMILIES[f])[0]) for i, f in enumerate(fam)]


def records(graphs, edge_features=3):
    from deeprank2_amd.store import GraphRecord  # noqa: PLC0415
    from deeprank2_amd.utils.synthetic import doubled_edges  # noqa: PLC0415

    out = []
    for i, g in enumerate(graphs):
        ei, ea = doubled_edges(g)
        ea = ea[:, :edge_features]
        out.append(GraphRecord(x=g["x"], edge_index=ei, edge_attr=ea, cluster0=g["cluster0"], cluster1=g["cluster1"], y=float(g["y"]), pos=g["pos"], name=f"syn{i}"))
    return out


def algorithmic_bytes(packed, gids, model="ginet", s=4):
    """SURVEY §8(d)'s compulsory bytes for one graph pass over these graphs:
    B_alg(g) = s*N*F (x) + 4*E (int32 CSR sources) + 4*(N+1) (rowptr)
    + 4*N (cluster0) + 4*K0 (cluster1) + 4 (y); s = 4 (fp32) or 2 (bf16).
    VanillaNetwork adds its edge features (s*E*Fe) and reads no clusters;
    SGAT adds its one edge feature (s*E); ginet_nocluster reads no clusters."""
    n, e, k0, _p1, _k1 = (a[gids] for a in packed.sizes())
    f = packed.n_feat
    base = s * n * f + 4 * e + 4 * (n + 1) + 4
    clusters = 4 * n + 4 * k0
    if model == "vanilla":
        fe = 0 if packed.edge_attr is None else packed.edge_attr.shape[1]
        per = base + s * e * fe
    elif model == "ginet_nocluster":
        per = base
    elif model == "sgat":
        per = base + clusters + s * e
    else:
        per = base + clusters
    return int(per.sum())


def design_bytes(packed, gids, model="ginet", out_dim=1):
    """Bytes this design moves beyond §8(d)'s compulsory ones, per graph pass:
    the per-graph gradient slab and head vectors the graph pass writes and the
    reduce kernel reads back (GINet: 4(32F+1024) + 4(320+r4(out)) per graph),
    plus the precomputed pooling structures (depth-0 member lists, pooled CSR,
    depth-1 members) and, for Vanilla, the transposed CSR."""
    n, e, k0, p1, k1 = (a[gids] for a in packed.sizes())
    f = packed.n_feat
    r4 = lambda v: (v + 3) & ~3  # noqa: E731
    if model == "vanilla":
        fe = 0 if packed.edge_attr is None else packed.edge_attr.shape[1]
        part = 4 * 2 * (32 * (2 * f + fe) + 32 + f * (f + 32) + f) + 4 * (r4(f) + 256 + r4(out_dim))
        extra = 4 * (n + 1) + 4 * e
    elif model == "ginet_nocluster":
        part = 4 * (32 * f + 1024) + 4 * (320 + r4(out_dim))
        extra = 4 * (n + 1) + 2 * e
    else:
        pool = 4 * (k0 + 1) + 4 * (k0 + 1) + 4 * p1 + 4 * (k1 + 1)
        if model in ("foutnet", "sgat"):
            part = 4 * (32 * f + 1072) + 4 * (160 + r4(out_dim))
        else:
            part = 4 * (32 * f + 1024) + 4 * (320 + r4(out_dim))
        extra = pool + (8 * p1 if model == "sgat" else 0)
    return int((2 * part + extra).sum())


MFMA_PEAK_TFLOPS = {"f32": 157.3, "bf16": 2500.0}  # dense MFMA peaks (MI355X_MICROARCH.md, chip-level parameters)
MFMA_FLOP_PER_INST = 16 * 16 * 4 * 2  # v_mfma_f32_16x16x4_f32, the only MFMA shape of the fp32 graph kernels
N_SIMDS = 256 * 4


def algorithmic_flops(packed, gids, model="ginet"):
    """Algorithmic FLOPs of one graph pass (fwd + bwd) over these graphs.
    GINet: SURVEY §8(d)'s formula per graph, 3*(2*N*F*32) + 2*E*32 (the conv1
    node GEMM forward and its two backward GEMMs, plus the edge aggregation;
    §8(d) quotes ~0.96 MFLOP/graph, but the formula it states evaluates to
    1.34 MFLOP at N=200, E=3000, F=30 — the formula is what is used here).
    The other models by the same recipe (their dense node GEMMs x3 + one
    multiply-add per aggregated element):
    FoutNet/SGAT 3*(2*N*2F*16) + 2*E*F; ginet_nocluster adds conv2 on the
    full graph, 3*(2*N*32*64) + 2*E*32; VanillaNetwork per layer
    3*(2*N*F*64 + 2*N*(F+32)*F) + 2*E*32*(Fe+2)."""
    n, e, *_ = (a[gids] for a in packed.sizes())
    f = packed.n_feat
    if model == "ginet":
        per = 3 * (2 * n * f * 32) + 2 * e * 32
    elif model in ("foutnet", "sgat"):
        per = 3 * (2 * n * 2 * f * 16) + 2 * e * f
    elif model == "ginet_nocluster":
        per = 3 * (2 * n * f * 32) + 2 * e * 32 + 3 * (2 * n * 32 * 64) + 2 * e * 32
    else:  # vanilla
        fe = 0 if packed.edge_attr is None else packed.edge_attr.shape[1]
        per = 2 * (3 * (2 * n * f * 64 + 2 * n * (f + 32) * f) + 2 * e * 32 * (fe + 2))
    return int(per.sum())


def pmc_mfma(model, kernel_ms, n_wg):
    """MFMA utilisation of the dominant kernel from the newest committed PMC pass
    (profiles/*/pmc_mfma_<model>.txt, scripts/gpu.sh pmc: one rocprofv3
    --pmc run of SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_MFMA, SQ_BUSY_CU_CYCLES,
    GRBM_GUI_ACTIVE, median over dispatches).
    * executed MFMA FLOPs = SQ_INSTS_MFMA x 2048 (16x16x4 f32), priced against
      this run's kernel time and the fp32 MFMA peak;
    * busy fractions: SQ_VALU_MFMA_BUSY_CYCLES (matrix-pipe busy cycles summed
      over SIMDs) / (kernel cycles x SIMDs), kernel cycles = GRBM_GUI_ACTIVE / 8
      (summed over the 8 XCDs; reads high on short dispatches, so the
      fractions are lower bounds), over the whole chip (1024 SIMDs) and over
      the SIMDs of the CUs the launch occupies (one workgroup per CU)."""
    import glob  # noqa: PLC0415

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", f"pmc_mfma_{model}.txt")))
    if not files:
        return None
    vals = {}
    for line in open(files[-1]):
        parts = line.split()
        if len(parts) >= 2:
            try:
                vals[parts[0]] = float(parts[1])
            except ValueError:
                pass
    need = ("SQ_INSTS_MFMA", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE")
    if any(k not in vals for k in need):
        return None
    cyc = vals["GRBM_GUI_ACTIVE"] / 8.0
    busy = vals["SQ_VALU_MFMA_BUSY_CYCLES"]
    exec_flops = vals["SQ_INSTS_MFMA"] * MFMA_FLOP_PER_INST
    tf = exec_flops / (kernel_ms * 1e-3) / 1e12
    return {
        "source": os.path.relpath(files[-1], ROOT),
        "insts_per_launch": vals["SQ_INSTS_MFMA"],
        "executed_flops_per_launch": exec_flops,
        "executed_tflops": round(tf, 4),
        "executed_frac_of_peak": round(tf / MFMA_PEAK_TFLOPS["f32"], 6),
        "busy_cycles": busy,
        "kernel_cycles_grbm": cyc,
        "mfma_busy_frac": round(busy / (cyc * N_SIMDS), 6),
        "mfma_busy_frac_active_simds": round(busy / (cyc * 4 * min(256, n_wg)), 6),
        "active_cus": min(256, n_wg),
    }


PMC_FILES = {"ginet": "pmc_ginet_graph_kernel.txt", "foutnet": "pmc_foutnet_graph_kernel.txt", "sgat": "pmc_sgat_graph_kernel.txt", "vanilla": "pmc_vanilla_graph_kernel.txt", "ginet_nocluster": "pmc_ginet_nocluster_graph_kernel.txt"}


def pmc_traffic_bytes(model="ginet"):
    """HBM bytes per graph-kernel launch from the newest committed PMC pass
    (profiles/*/pmc_<model>_graph_kernel.txt, collected by scripts/gpu.sh's pmc
    section with FETCH_SIZE and WRITE_SIZE in separate passes).  gfx950 correction
    (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts half the bytes of wide
    coalesced reads, so bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024."""
    import glob  # noqa: PLC0415

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", PMC_FILES[model])))
    if not files:
        return None, None
    vals = {}
    for line in open(files[-1]):
        parts = line.split()
        if len(parts) >= 2 and parts[0] in ("FETCH_SIZE", "WRITE_SIZE"):
            vals[parts[0]] = float(parts[1])
    if len(vals) != 2:
        return None, None
    return int((2 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024), os.path.relpath(files[-1], ROOT)


def newest_profile(stem):
    """Newest committed ``profiles/r<NN>/<stem>[_final<k>].txt``: the highest
    round first, then the highest ``_final`` suffix (r04 committed its HEAD
    tables as ``_final2``); ``_baseline`` / ``_not_kept`` files never match."""
    import glob  # noqa: PLC0415
    import re  # noqa: PLC0415

    pat = re.compile(re.escape(stem) + r"(?:_final(\d*))?\.txt")
    best = None
    for path in glob.glob(os.path.join(ROOT, "profiles", "r*", f"{stem}*.txt")):
        m = pat.fullmatch(os.path.basename(path))
        if not m:
            continue
        # the canonical name is a round's own HEAD table; among _final<k>, the highest k
        rank = 1000 if m.group(1) is None and not os.path.basename(path).endswith("_final.txt") else int(m.group(1) or 0)
        key = (os.path.basename(os.path.dirname(path)), rank)
        if best is None or key > best[0]:
            best = (key, path)
    return None if best is None else best[1]


def pmc_traffic_step(model, graphs, dtype="f32"):
    """HBM bytes per step of the model's graph-pass kernels from the newest
    committed per-kernel PMC table (profiles/*/pmc_per_kernel_<model>_<graphs>[_bf16].txt,
    tools/pmc_per_kernel.py over FETCH_SIZE / WRITE_SIZE passes of
    tools/pmc_run.py): for the multi-kernel paths (the Vanilla pipeline, the
    GINet tile + tail kernels), whose "graph pass" is a chain of launches
    (same gfx950 correction as pmc_traffic_bytes)."""
    path = newest_profile(f"pmc_per_kernel_{model}_{graphs}" + ("_bf16" if dtype == "bf16" else ""))
    if path is None:
        return None, None
    for line in open(path):
        if line.startswith("per step (graph pass kernels):"):
            mb = float(line.split(",")[1].split("MB")[0])
            return int(mb * 1e6), os.path.relpath(path, ROOT)
    return None, None


def stream_copy_gbs(dev, mib=1024, reps=5):
    """Achievable HBM bandwidth on this GPU: a device-to-device copy of ``mib``
    MiB timed with HIP events (bytes read + written), best of ``reps``."""
    import torch  # noqa: PLC0415

    n = mib * (1 << 20) // 4
    src = torch.ones(n, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    dst.copy_(src)
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        dst.copy_(src)
        e1.record()
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    del src, dst
    torch.cuda.empty_cache()
    return 2 * n * 4 / (best * 1e-3) / 1e9


def host_cores():
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    used = min(aff, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else aff
    return used, aff


def idlest_cpus(cands, k, dt=0.25):
    """The k CPUs of ``cands`` that were idle longest over ``dt`` seconds
    (/proc/stat deltas): on a shared host the low-numbered CPUs of the
    affinity set may be busy with another tenant's work."""
    def snap():
        out = {}
        with open("/proc/stat") as f:
            for line in f:
                if line.startswith("cpu") and line[3:4].isdigit():
                    p = line.split()
                    v = [int(x) for x in p[1:]]
                    out[int(p[0][3:])] = (v[3] + v[4], sum(v))  # idle + iowait, total
        return out

    try:
        a = snap()
        time.sleep(dt)
        b = snap()
    except (OSError, ValueError, IndexError):
        return sorted(cands)[:k]

    def idle(c):
        if c not in a or c not in b or b[c][1] <= a[c][1]:
            return 0.0
        return (b[c][0] - a[c][0]) / (b[c][1] - a[c][1])

    return sorted(sorted(cands, key=lambda c: (-idle(c), c))[:k])


def cpu_baseline(graphs, budget_s=15.0, max_steps=60, model_name="ginet"):
    """The CPU oracle (op-for-op restatement of the reference, torch CPU) training
    the same batch: forward, MSE, backward, Adam — on this host's cores
    (``len(os.sched_getaffinity(0))``, or the box's ``OMP_NUM_THREADS`` share)."""
    import numpy as np  # noqa: PLC0415
    import torch  # noqa: PLC0415

    from oracle import data_ref, gnn_ref  # noqa: PLC0415
    from oracle import pyg_ops as P  # noqa: PLC0415

    cores, affinity = host_cores()
    torch.set_num_threads(cores)
    datas = [data_ref.synthetic_to_data(g) for g in graphs]
    torch.manual_seed(1234)
    if model_name == "sgat":
        for d in datas:
            d.edge_attr = d.edge_attr[:, :1].contiguous()
    model = gnn_ref.MODELS[ORACLE_MODELS[model_name]](30, 1, 3).train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-5)

    def one():
        bat = P.Batch.from_data_list([d.clone() for d in datas])
        opt.zero_grad()
        out = model(bat)
        loss = torch.nn.functional.mse_loss(out.reshape(-1), bat.y)
        loss.backward()
        opt.step()

    # a stable denominator: the threads pinned to the `cores` idlest CPUs of
    # the affinity set, 3 warm-up steps, then the fastest of the timed steps
    pinned = idlest_cpus(os.sched_getaffinity(0), cores) if hasattr(os, "sched_getaffinity") else []
    prev = os.sched_getaffinity(0) if pinned else None
    if pinned:
        os.sched_setaffinity(0, pinned)
    try:
        # warm-up: 3 steps, or 1 when one step already takes over a second
        # (FoutNet's per-node loop, foutnet.py:55-58: ~2.7 s per residue batch)
        t1 = time.perf_counter()
        one()
        warm = 1
        t_first = time.perf_counter() - t1
        if t_first > 2.0:  # a bounded sample: two timed steps (stated in "sample")
            max_steps = 2
        if t_first < 1.0:
            one()
            one()
            warm = 3
        times = []
        t0 = time.perf_counter()
        while len(times) < max_steps and (time.perf_counter() - t0 < budget_s or len(times) < 2):
            t1 = time.perf_counter()
            one()
            times.append(time.perf_counter() - t1)
    finally:
        if prev is not None:
            os.sched_setaffinity(0, prev)
    # the fastest timed step: the shared host's other tenants only ever add
    # time (r06 samples on a busy box spread 60 ms - 1.8 s per step), and the
    # median of a 2-step sample is their mean
    dt = float(np.min(times))
    n = len(times)
    name = ORACLE_MODELS[model_name]
    return {"value": round(len(graphs) / dt, 2), "unit": "graphs/s", "cores": cores, "host_affinity_cores": affinity, "kind": "port", "sample": f"fastest of {n} {name}(30,1,3) train steps (fwd+MSE+bwd+Adam) after {warm} warm-up step(s), on one batch of {len(graphs)} of the same synthetic graphs; oracle/gnn_ref.py on torch CPU, {cores} threads pinned to the {len(pinned) or cores} idlest CPUs (host affinity {affinity}); {dt * 1e3:.1f} ms/step (median {float(np.median(times)) * 1e3:.1f}, max {max(times) * 1e3:.1f})"}


def parse_args(argv):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batches", type=int, default=16, help="resident mini-batches per rank")
    ap.add_argument("--batch", type=int, default=None, help="graphs per GPU per step (default 64; 32 for atom-level graphs)")
    ap.add_argument("--model", choices=MODEL_NAMES, default="ginet")
    ap.add_argument("--graphs", choices=["residue", "atom", "mixed", "srv"], default="residue")
    ap.add_argument("--dtype", choices=["f32", "bf16"], default="f32", help="compute dtype of the node GEMMs (bf16: GINet only; fp32 accumulate, fp32 master weights and Adam)")
    ap.add_argument("--force-large", type=int, default=0, help="GINet: run the split tile+tail path with this many nodes per tile (diagnostic)")
    ap.add_argument("--ginet-path", choices=["auto", "split"], default="auto", help="GINet: auto = one workgroup per graph when the batch fits LDS, else the split path; split = tile kernel + tail kernel")
    ap.add_argument("--vanilla-pipeline", action="store_true", help="VanillaNetwork: the batch-wide kernel pipeline even when the per-graph kernel fits (diagnostic)")
    ap.add_argument("--acc", choices=["auto", "on", "off"], default="auto", help="GINet fp32: accumulating pass (dr_ginet_acc_pass: each workgroup sums every R-th graph's gradients on chip, one partial row per workgroup); auto = batches past the CU count")
    ap.add_argument("--no-acc-prefetch", action="store_true", help="accumulating pass without the prefetch layout (A/B: each graph stages its own inputs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stream-copy", action="store_true")
    ap.add_argument("--eager", action="store_true", help="launch every step from Python instead of replaying captured HIP graphs")
    ap.add_argument("--eager-ddp", action="store_true", help="N>1: launch steps from Python (default: the RCCL all-reduce is captured in the HIP graph with the kernels)")
    ap.add_argument("--trainer", action="store_true", help="diagnostic: the drop-in path, Trainer(GINet, GraphDataset(HDF5)).train(), and the GraphDataset -> GraphStore load rate (one JSON line; not the headline)")
    ap.add_argument("--epochs", type=int, default=3, help="--trainer: timed training epochs")
    ap.add_argument("--validate", action="store_true", help="--trainer: train(validate=True), timing each validation pass")
    ap.add_argument("--shard-policy", choices=["auto", "contiguous", "edges"], default="auto", help="N>1: how each global batch is split over the ranks (distributed.plan_shards)")
    ap.add_argument("--dry-run", action="store_true", help="launcher check without a GPU: each rank joins a gloo group, builds the global batches and its shards, rank 0 prints the JSON skeleton with the per-rank edge loads")
    return ap.parse_args(argv)


def global_batches(args, world, rank):
    """The run's data, identical on every rank: one synthetic set of
    B*world*batches graphs (seed 1000), one global batch of B*world graphs per
    resident mini-batch (a seeded permutation), and this rank's shard of each
    (``plan_shards``).  At world 1 this is the set, order and batches the
    single-GPU bench always used.  Returns (graphs, packed, local batches,
    plans, B)."""
    import numpy as np  # noqa: PLC0415

    from deeprank2_amd.distributed import plan_shards  # noqa: PLC0415
    from deeprank2_amd.store import pack_graphs  # noqa: PLC0415

    B = args.batch or (32 if args.graphs == "atom" else B_PER_GPU)
    if args.graphs in ("atom", "mixed"):
        args.batches = min(args.batches, 4)  # generation time of ~3k-node graphs
    bg = B * world
    graphs = make_graphs(args.graphs, bg * args.batches, seed=1000)
    packed = pack_graphs(records(graphs, 1 if args.model == "sgat" else 3), require_clusters=args.model not in ("ginet_nocluster", "vanilla"))
    order = np.random.default_rng(0).permutation(packed.n_graphs).astype(np.int32)
    edges = np.diff(packed.edge_off)
    local, plans = [], []
    for i in range(args.batches):
        gb = order[i * bg:(i + 1) * bg]
        plan = plan_shards(edges[gb], world, policy=args.shard_policy)
        plans.append(plan)
        local.append(gb[plan.positions[rank]])
    return graphs, packed, local, plans, B


def trainer_bench(args):
    """The drop-in path as a user runs it (reference trainer.py:503-724 over
    dataset.py:883-1052): configs[1]-shape graphs written as a DeepRank2 HDF5
    file, ``GraphDataset`` on it, ``Trainer(GINet, ...)`` and ``train()``.
    Reports (1) the load rate: HDF5 -> GraphDataset (index, features) ->
    packed HBM ``GraphStore`` in graphs/s and per host core used, beside the
    reference's ~400 graphs/s/core per-item HDF5 read; (2) the
    training epochs' graphs/s and us per step through ``Trainer._epoch``
    (device loss, one D2H per epoch), beside the captured-step number of the
    headline line.  Prints one JSON line (diagnostic)."""
    import tempfile  # noqa: PLC0415

    import numpy as np  # noqa: PLC0415
    import torch  # noqa: PLC0415

    from deeprank2_amd.dataset import GraphDataset  # noqa: PLC0415
    from deeprank2_amd.exporters import MemoryOutputExporter  # noqa: PLC0415
    from deeprank2_amd.neuralnets.gnn.ginet import GINet  # noqa: PLC0415
    from deeprank2_amd.trainer import Trainer  # noqa: PLC0415
    from deeprank2_amd.utils import synthetic as S  # noqa: PLC0415

    B = args.batch or B_PER_GPU
    n = B * args.batches
    graphs = make_graphs("residue", n, seed=1000)
    dev = torch.device("cuda:0")
    # DR_BENCH_PG=1: Trainer(ngpu=2) on a one-rank RCCL group, the data-parallel
    # code path (shards, the all-reduce captured in the epoch graph, the epoch's
    # loss all-reduce and prediction gather) rehearsed on one GPU
    ddp = os.environ.get("DR_BENCH_PG") == "1"
    if ddp:
        torch.cuda.set_device(dev)
        torch.distributed.init_process_group("nccl", device_id=dev, init_method=f"tcp://127.0.0.1:{_free_port()}", world_size=1, rank=0)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "train.hdf5")
        t0 = time.perf_counter()
        S.write_hdf5(path, graphs)
        t_write = time.perf_counter() - t0
        t0 = time.perf_counter()
        ds = GraphDataset(path, node_features=S.SYNTH_NODE_FEATURES, edge_features=S.SYNTH_EDGE_FEATURES, target="irmsd", clustering_method="mcl")
        t_index = time.perf_counter() - t0
        t0 = time.perf_counter()
        store = ds.graph_store(dev)
        torch.cuda.synchronize()
        t_pack = time.perf_counter() - t0
        cores, affinity = host_cores()
        load = {"graphs": n, "hdf5_write_s": round(t_write, 3), "dataset_init_s": round(t_index, 3), "graph_store_s": round(t_pack, 3), "graphs_per_s": round(n / (t_index + t_pack), 1), "cores": cores, "graphs_per_s_per_core": round(n / (t_index + t_pack) / cores, 1), "reference_graphs_per_s_per_core": 400, "note": "GraphDataset(HDF5) construction (file read, index, feature checks) + graph_store (per-entry arrays, threaded C++ pack, H2D) for the whole file; the reference reads one entry per item (dataset.py:883-1052, ~2.5 ms/graph/core, SURVEY §6)"}
        # the same host-side load on ONE core (a child pinned to one CPU,
        # OMP_NUM_THREADS=1: one HDF5 worker, one packer thread, no upload)
        try:
            cpu = sorted(os.sched_getaffinity(0))[0]
            env = dict(os.environ, OMP_NUM_THREADS="1")
            r = subprocess.run([sys.executable, "-c", f"import os, runpy, sys; os.sched_setaffinity(0, {{{cpu}}}); sys.argv = ['load_one_core.py', {path!r}]; runpy.run_path({os.path.join(ROOT, 'tools', 'load_one_core.py')!r}, run_name='__main__')"], capture_output=True, text=True, env=env, timeout=600, check=False)
            one = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
            load["one_core"] = {**one, "note": "GraphDataset + per-entry arrays + C++ pack on one pinned CPU (tools/load_one_core.py): graphs/s on one core, the reference's per-core unit"}
        except Exception as e:  # noqa: BLE001  (diagnostic only)
            load["one_core"] = {"error": str(e)[:200]}
        del store
        torch.manual_seed(1234)
        mem = MemoryOutputExporter()
        tr = Trainer(GINet, ds, cuda=True, output_exporters=[mem], precluster=False, ngpu=2 if ddp else 0)
        epoch_s, eval_s = [], []

        def timer(orig, sink):
            def timed(*a, **k):
                torch.cuda.synchronize()
                t = time.perf_counter()
                r = orig(*a, **k)
                torch.cuda.synchronize()
                sink.append(time.perf_counter() - t)
                return r

            return timed

        tr._epoch = timer(tr._epoch, epoch_s)  # noqa: SLF001
        tr._eval = timer(tr._eval, eval_s)  # noqa: SLF001
        val = bool(args.validate)
        tr.train(nepoch=1, batch_size=B, shuffle=True, best_model=False, filename=None, validate=val)  # warm-up epoch (store, plans, the epoch's HIP graphs)
        epoch_s.clear()
        eval_s.clear()
        t0 = time.perf_counter()
        tr.train(nepoch=args.epochs, batch_size=B, shuffle=True, best_model=False, filename=None, validate=val)
        t_train = time.perf_counter() - t0
        per_epoch = float(np.median(epoch_s))
        # evaluations: the epoch-0 pass over the training set, then one validation per epoch
        val_evals = eval_s[2:] if val else []
        per_eval = float(np.median(val_evals)) if val_evals else None
        captured = any(not (isinstance(k, tuple) and k and k[0] == "eval") for k in tr._runners)  # noqa: SLF001
        eval_captured = any(isinstance(k, tuple) and k and k[0] == "eval" for k in tr._runners)  # noqa: SLF001
        # the same epochs through the per-batch loop (descriptors + two launches per batch from Python)
        Trainer.capture_epochs = False
        try:
            tr.train(nepoch=1, batch_size=B, shuffle=True, best_model=False, filename=None, validate=val)
            epoch_s.clear()
            eval_s.clear()
            tr.train(nepoch=args.epochs, batch_size=B, shuffle=True, best_model=False, filename=None, validate=val)
        finally:
            Trainer.capture_epochs = True
        per_epoch_loop = float(np.median(epoch_s))
        per_eval_loop = float(np.median(eval_s[2:])) if val and len(eval_s) > 2 else None
    steps = int(np.ceil(len(tr.dataset_train) / B))
    val_batches = int(np.ceil(len(tr.dataset_val) / B)) if tr.dataset_val is not None else 0
    res = {
        "metric": "graphs/sec per Trainer training epoch (drop-in path: Trainer(GINet, GraphDataset(HDF5)).train), configs[1] graphs",
        "value": round(len(tr.dataset_train) / per_epoch, 1),
        "unit": "graphs/s",
        "us_per_step": round(per_epoch / steps * 1e6, 2),
        "steps_per_epoch": steps,
        "train_graphs": len(tr.dataset_train),
        "batch_size": B,
        "epochs_timed": args.epochs,
        "fused_step": bool(tr._fused),  # noqa: SLF001
        "captured_epochs": captured,
        "per_batch_loop": {"graphs_per_s": round(len(tr.dataset_train) / per_epoch_loop, 1), "us_per_step": round(per_epoch_loop / steps * 1e6, 2), "note": "Trainer.capture_epochs = False: per batch, the host builds descriptors and launches the graph pass and reduce/Adam"},
        "data_parallel": {"process_group": "nccl, world 1 (DR_BENCH_PG=1: Trainer(ngpu=2) code path on one GPU)", "world": 1} if ddp else None,
        "validation": None if per_eval is None else {
            "graphs": len(tr.dataset_val), "batches": val_batches, "captured": eval_captured,
            "us_per_eval": round(per_eval * 1e6, 1), "us_per_batch": round(per_eval / max(val_batches, 1) * 1e6, 2),
            "per_batch_loop_us_per_batch": None if per_eval_loop is None else round(per_eval_loop / max(val_batches, 1) * 1e6, 2),
            "note": "Trainer._eval on the validation loader (forward passes, per-batch loss on the device, exporters, one D2H): captured = the evaluation's passes as one HIP graph (epoch.EvalRunner)"},
        "train_call_s": round(t_train, 3),
        "train_call_note": "the whole train() call: epoch-0 evaluation, the timed epochs, model selection and the final state load",
        "load": load,
        "data": "synthetic (seeded residue graphs per SURVEY §8(d), written as a DeepRank2 HDF5 file); random-init GINet(30,1,3)",
    }
    print(json.dumps(res), flush=True)
    if ddp:
        torch.distributed.destroy_process_group()
    return res


def dry_run(args):
    """CPU-only rehearsal of the N-rank launch: the line carries the world size
    and backend the ranks actually formed (tests/test_bench_launch.py)."""
    import torch  # noqa: PLC0415

    world = int(os.environ.get("WORLD_SIZE", "1"))
    backend = None
    if world > 1:
        torch.distributed.init_process_group("gloo")
        world = torch.distributed.get_world_size()
        backend = torch.distributed.get_backend()
        t = torch.ones(1)
        torch.distributed.all_reduce(t)
        assert int(t.item()) == world
    rank = int(os.environ.get("RANK", "0"))
    _graphs, _packed, local, plans, B = global_batches(args, world, rank)
    mine = [int(_packed.edge_off[g + 1] - _packed.edge_off[g]) for g in local[0]]
    if world > 1:  # every rank's own count of its first shard, checked against rank 0's plan
        t = torch.zeros(world, dtype=torch.int64)
        t[rank] = sum(mine)
        torch.distributed.all_reduce(t)
        assert t.tolist() == list(plans[0].loads), (t.tolist(), plans[0].loads)
    if rank == 0:
        shards = {"policy": args.shard_policy, "balanced": [p.balanced for p in plans], "rank_graphs": [p.sizes() for p in plans], "rank_edge_loads": [list(p.loads) for p in plans]}
        print(json.dumps({"metric": HEADLINE_METRIC, "value": None, "unit": "graphs/s", "n_gpus": world, "world_size": world, "backend": backend, "dry_run": True, "config": {"graphs": args.graphs, "graphs_per_gpu": B, "global_batch": B * world, "parallelism": f"dp{world}"}, "shards": shards}), flush=True)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


def main(args):  # noqa: PLR0915, PLR0912, C901
    import numpy as np  # noqa: PLC0415
    import torch  # noqa: PLC0415

    from deeprank2_amd.engine import FusedTrainStep  # noqa: PLC0415
    from deeprank2_amd.fused import BatchHandle  # noqa: PLC0415
    from deeprank2_amd.neuralnets.gnn.foutnet import FoutNet  # noqa: PLC0415
    from deeprank2_amd.neuralnets.gnn.ginet import GINet  # noqa: PLC0415
    from deeprank2_amd.neuralnets.gnn.ginet_nocluster import GINet as GINetNoCluster  # noqa: PLC0415
    from deeprank2_amd.neuralnets.gnn.sgat import SGAT  # noqa: PLC0415
    from deeprank2_amd.neuralnets.gnn.vanilla_gnn import VanillaNetwork  # noqa: PLC0415
    from deeprank2_amd.store import GraphStore  # noqa: PLC0415

    models = {"ginet": GINet, "foutnet": FoutNet, "vanilla": VanillaNetwork, "sgat": SGAT, "ginet_nocluster": GINetNoCluster}
    if args.dtype == "bf16" and args.model != "ginet":
        msg = "--dtype bf16 is implemented for GINet (BASELINE.json configs[3])"
        raise SystemExit(msg)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pg = None
    # DR_BENCH_SHARED_GPU=1 rehearses the N>1 code path on a one-GPU box (all
    # ranks on cuda:0 over gloo); real multi-GPU runs use RCCL, one GPU per rank.
    shared = os.environ.get("DR_BENCH_SHARED_GPU") == "1"
    # DR_BENCH_PG=1 runs the data-parallel step (RCCL all-reduce between the
    # graph pass and Adam) even at WORLD_SIZE=1: a one-GPU rehearsal of the
    # N>1 launch path, captured all-reduce included.
    force_pg = os.environ.get("DR_BENCH_PG") == "1"
    if shared:
        local = 0
    backend = None
    if world > 1 or force_pg:
        torch.cuda.set_device(local)
        if shared:
            torch.distributed.init_process_group("gloo")
        else:
            torch.distributed.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        pg = torch.distributed.group.WORLD
        world = torch.distributed.get_world_size()
        backend = torch.distributed.get_backend()
    dev = torch.device(f"cuda:{local}")

    graphs, packed, local, plans, B = global_batches(args, world, rank)
    store = GraphStore(packed, dev, dtype=args.dtype)
    if any(len(g) == 0 for g in local):
        msg = f"rank {rank}: an empty shard (global batch {B * world} over {world} ranks)"
        raise SystemExit(msg)
    handles = [BatchHandle(store, g) for g in local]
    for h in handles:
        h.force_large = bool(args.force_large) or args.ginet_path != "auto"
        h.large_tile = args.force_large or None
        h.vanilla_pipeline = bool(args.vanilla_pipeline)
        if os.environ.get("DR_VANILLA_TILE") is not None:  # diagnostic: rows per pipeline edge tile (0: untiled)
            h.vanilla_tile_rows = int(os.environ["DR_VANILLA_TILE"])

    torch.manual_seed(1234)
    model = models[args.model](30, 1, 3).to(dev).train()
    if pg is not None:
        for p in model.parameters():
            torch.distributed.broadcast(p.data, 0)
    step = FusedTrainStep(model, lr=1e-3, weight_decay=1e-5, loss="mse", process_group=pg, compute_dtype=args.dtype)
    model._drop_seed = 77 + rank  # training-mode dropout drawn in-kernel (counter hash)
    step.acc = {"auto": None, "on": True, "off": False}[args.acc]
    step.acc_prefetch = not args.no_acc_prefetch

    def run_eager(i):
        return step.step(handles[i % len(handles)], global_batch=B * world)

    for i in range(args.warmup):
        run_eager(i)
    # steps i0.. run in mini-batch order i % len(handles): the sweep graph is
    # captured starting at the first timed mini-batch, so every timed step
    # replays a captured graph whatever --steps / --warmup are
    rot = args.warmup % len(handles)
    sweep_handles = handles[rot:] + handles[:rot]
    captured = sweep = None
    capture_note = ""
    # batches beyond the model's graph pass (FoutNet/SGAT/ginet_nocluster on
    # atom-level graphs) take the layer-level path: autograd over the layer
    # kernels, with host-side shape checks, so those steps run eagerly
    from deeprank2_amd import layered  # noqa: PLC0415

    layer_path = any(layered.needs_layers(step.spec, h, step.out_dim) for h in handles)
    if layer_path:
        capture_note = " (layer-level path for graphs beyond one workgroup's LDS: autograd, not capturable)"
    if not args.eager and not layer_path and (pg is None or (not shared and not args.eager_ddp)):
        # one captured graph per resident mini-batch, plus one graph holding a
        # whole sweep over them (one launch per len(handles) steps); N>1: the
        # RCCL all-reduce is captured with the kernels
        try:
            captured = [step.capture(h, global_batch=B * world) for h in handles]
            sweep = step.capture_sweep(sweep_handles, global_batch=B * world)
        except RuntimeError as e:
            if pg is None:
                raise
            captured = sweep = None  # fall back to eager steps
            capture_note = f" (capture failed: {str(e)[:120]})"
            print(f"[bench] rank {rank}: HIP graph capture of the DDP step failed, running eager steps: {e}", file=sys.stderr)
        if pg is not None:  # every rank runs the same launch mode
            ok = torch.tensor([0.0 if captured is None else 1.0], device=dev)
            torch.distributed.all_reduce(ok, op=torch.distributed.ReduceOp.MIN)
            if float(ok.item()) < 1.0:
                captured = sweep = None
                capture_note = capture_note or " (capture failed on another rank)"

    n_sweeps = args.steps // len(handles) if sweep is not None else 0
    # the steps after the whole sweeps: one more captured graph (one launch),
    # not one replay per step; up to 64 timed steps: all of them in one graph
    n_rest = args.steps - n_sweeps * len(handles) if sweep is not None else 0
    if sweep is not None and args.steps <= 64:
        n_sweeps, n_rest = 0, args.steps
    rest = None
    if n_rest and os.environ.get("DR_BENCH_REST", "1") == "1":
        rest = step.capture_sweep([sweep_handles[i % len(handles)] for i in range(n_rest)], global_batch=B * world)

    if sweep is not None:
        # prime: replay each graph the timed region launches once (their first
        # launch uploads them), then restore the training state, so the timed
        # region starts from the state W warmup steps left
        snap = [t.detach().clone() for t in step._state_tensors()]  # noqa: SLF001
        for gr in [sweep if n_sweeps else None, rest, *(captured if n_rest and rest is None else [])]:
            if gr is not None:
                gr.replay()
        torch.cuda.synchronize()
        for t, v in zip(step._state_tensors(), snap):  # noqa: SLF001
            t.data.copy_(v)
        del snap

    def run_steps(i0, k):
        """Steps i0 .. i0+k-1 (mini-batch i % len(handles)): whole sweeps first, then the rest graph (or per-step graphs)."""
        i = i0
        for _ in range(n_sweeps):
            sweep.replay()
            i += len(handles)
        if rest is not None:
            rest.replay()
            i += n_rest
        while i < i0 + k:
            if captured is not None:
                captured[i % len(captured)].replay()
            else:
                run_eager(i)
            i += 1
        return step.loss_out

    torch.cuda.synchronize()
    if pg is not None:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if os.environ.get("DR_BENCH_EVT"):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    loss = run_steps(args.warmup, args.steps)
    if os.environ.get("DR_BENCH_EVT"):
        t_issue = time.perf_counter() - t0
        e1.record()
    torch.cuda.synchronize()
    if os.environ.get("DR_BENCH_EVT"):
        print(f"[bench] timed region: wall {1e6 * (time.perf_counter() - t0):.1f} us, events {1e3 * e0.elapsed_time(e1):.1f} us, host issue {1e6 * t_issue:.1f} us", file=sys.stderr)
    if pg is not None:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0

    # Dominant-kernel duration: the graph pass alone, args.steps launches over
    # the resident mini-batches captured back to back in one HIP graph and
    # timed with HIP events on the launch stream (no host launch overhead;
    # agrees with the rocprofv3 kernel average, profiles/).
    # (at least 200 launches: a graph of K launches also carries the graph's
    # own launch latency, ~9 us, which at the driver's K = 20 would add ~0.45
    # us to every launch's average; the rocprofv3 average is the cross-check)
    n_kernel = max(args.steps, 200)
    kernel_ms = None if layer_path else step.time_graph_pass(handles, n_kernel, global_batch=B * world)
    if kernel_ms is None:  # layer path: no single graph-pass kernel; price the whole step
        kernel_ms = elapsed / args.steps * 1e3
    # the step split (pass / reduce + Adam / the rest: launch gaps inside the
    # replayed graphs), world of one only
    reduce_ms = None if (layer_path or pg is not None) else step.time_reduce(handles, n_kernel, global_batch=B * world)
    if pg is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
        km = torch.tensor([kernel_ms], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(km, op=torch.distributed.ReduceOp.MAX)
        kernel_ms = float(km.item())

    graphs_total = B * world * args.steps
    edges_local = sum(store.edges_in(handles[(args.warmup + i) % len(handles)].gids_host) for i in range(args.steps))
    et = torch.tensor([float(edges_local)], dtype=torch.float64, device=dev)
    if pg is not None:
        torch.distributed.all_reduce(et)
    edges_total = float(et.item())
    s = 2 if args.dtype == "bf16" else 4
    alg = float(np.mean([algorithmic_bytes(packed, h.gids_host, args.model, s) for h in handles]))
    design = float(np.mean([design_bytes(packed, h.gids_host, args.model) for h in handles]))
    n_params = sum(p.numel() for p in model.parameters())
    adam_bytes = 28 * n_params  # Adam fp32: read param, grad, m, v; write param, m, v (§8(d))
    kernel_alg = alg
    achieved = kernel_alg / (kernel_ms * 1e-3) / 1e9
    ms_step = elapsed / args.steps * 1e3
    wall_gbs = (alg + adam_bytes) / (ms_step * 1e-3) / 1e9
    default_cfg = args.model == "ginet" and args.graphs == "residue" and B == B_PER_GPU and args.dtype == "f32"
    pmc_cfg = default_cfg or (args.model in ("foutnet", "sgat", "vanilla", "ginet_nocluster") and args.graphs == "residue" and B == B_PER_GPU and args.dtype == "f32")
    traffic, traffic_src = pmc_traffic_bytes(args.model) if pmc_cfg else (None, None)
    large = args.model == "ginet" and (bool(args.force_large) or args.ginet_path != "auto" or args.dtype == "bf16" or any(h.lds((step.spec.entry, 1), lambda *sz: 0) > 160 * 1024 for h in handles))
    # multi-kernel graph passes (Vanilla pipeline, GINet tile + tail kernels):
    # the per-kernel PMC table of the same workload (tools/pmc_run.py <model>_<graphs>[_bf16])
    if traffic is None and B == B_PER_GPU_FOR.get(args.graphs) and not args.force_large and args.ginet_path == "auto" and (
        (args.model == "vanilla" and args.graphs in ("atom", "mixed")) or (args.model == "ginet" and args.graphs in ("atom", "mixed"))
    ):
        traffic, traffic_src = pmc_traffic_step(args.model, args.graphs, args.dtype)
    copy_gbs = None if args.no_stream_copy else stream_copy_gbs(dev)
    # §8(d) FLOP side: algorithmic FLOPs per launch against the dense MFMA peak
    # of the compute dtype, and MFMA utilisation from the committed PMC pass
    flops = float(np.mean([algorithmic_flops(packed, h.gids_host, args.model) for h in handles]))
    tflops = flops / (kernel_ms * 1e-3) / 1e12
    n_wg = B
    if args.model == "vanilla" and not layer_path:
        from deeprank2_amd.neuralnets.gnn.vanilla_gnn import split_k  # noqa: PLC0415

        n_wg = B * split_k(handles[0], 30, 3)
    mfma = pmc_mfma(args.model, kernel_ms, n_wg) if pmc_cfg else None

    result = None
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(graphs[:B], model_name=args.model)
        workload = WORKLOADS.get((args.model, args.graphs), f"{args.model} on {args.graphs} graphs (diagnostic)")
        kname = "layer-level path (FoutLayer/SGAT/GINetConvLayer + pooling kernels, torch autograd): whole-step wall clock" if layer_path else {"ginet": "ginet_large_conv1_kernel + ginet_large_tail_kernel (dr_ginet_large_pass)" if large else ((f"ginet_acc_kernel (dr_ginet_acc_pass: {step._acc_rows(handles[0])} workgroups, each runs every R-th graph's fwd+loss+bwd and sums its gradients on chip; one partial row per workgroup)" if step._acc_rows(handles[0]) else "ginet_graph_kernel (dr_ginet_graph_pass, fwd+loss+bwd, 1 workgroup/graph)")), "foutnet": "fout_graph_kernel<false> (dr_fout_graph_pass)", "vanilla": "vanilla_graph_kernel (dr_vanilla_fused_pass) / vanilla pipeline (dr_vanilla_graph_pass)", "sgat": "fout_graph_kernel<true> (dr_sgat_graph_pass)", "ginet_nocluster": "ginet_nocluster_kernel (dr_ginet_nocluster_graph_pass)"}[args.model]
        result = {
            "metric": HEADLINE_METRIC if default_cfg else f"graphs/sec per training step, {workload} (fwd+MSE+bwd+Adam)",
            "value": round(graphs_total / elapsed, 1),
            "unit": "graphs/s",
            "edges_per_sec": round(edges_total / elapsed, 1),
            "n_gpus": world,
            "world_size": world,
            "backend": backend,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": f"synthetic (seeded {args.graphs} graphs per SURVEY §8(d); random-init {models[args.model].__name__}(30,1,3))",
            "config": {
                "workload": workload,
                "ginet_path": args.ginet_path if args.model == "ginet" else None,
                "graphs_per_gpu": B,
                "global_batch": B * world,
                "mean_nodes_per_graph": round(float(np.diff(packed.node_off).mean()), 1),
                "mean_edges_per_graph": round(float(np.diff(packed.edge_off).mean()), 1),
                "node_features": 30,
                "edge_features": 1 if args.model == "sgat" else 3,
                "resident_graphs": packed.n_graphs,
                "parallelism": f"dp{world}",
                "shard_policy": args.shard_policy if world > 1 else None,
                "shards_edge_balanced": sum(p.balanced for p in plans) if world > 1 else None,
                "rank_edge_loads_first_batch": list(plans[0].loads) if world > 1 else None,
            },
            "roofline": {
                "kernel": kname,
                "bound": "hbm",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": int(kernel_alg),
                "algorithmic_definition": "SURVEY §8(d) B_alg: s*N*F + 4E + 4(N+1) + 4N + 4K0 + 4 per graph (s=2 bf16, 4 fp32; +s*E*Fe Vanilla, no clusters for Vanilla/ginet_nocluster)",
                "design_bytes_per_launch": int(design),
                "design_definition": "per-graph gradient slab + head vectors (written, then read by the reduce) and the precomputed pooling structures: intermediates of this design, not compulsory",
                "kernel_ms_avg": round(kernel_ms, 5),
                "kernel_timing": "wall clock per eager step (layer-level path)" if layer_path else f"HIP events around one HIP graph of {n_kernel} back-to-back {step.spec.entry if not large else 'dr_ginet_large_pass'} launches on the launch stream, divided by {n_kernel}",
                "stream_copy_GBs": None if copy_gbs is None else round(copy_gbs, 1),
                "frac_of_stream_copy": None if copy_gbs is None else round(achieved / copy_gbs, 5),
                "flops_per_launch": int(flops),
                "flops_definition": "algorithmic FLOPs of one graph pass (fwd+bwd), bench.algorithmic_flops: GINet 3*(2*N*F*32) + 2*E*32 per graph (SURVEY §8(d) formula)",
                "achieved_tflops": round(tflops, 4),
                "mfma_peak_tflops": MFMA_PEAK_TFLOPS[args.dtype],
                "flop_frac": round(tflops / MFMA_PEAK_TFLOPS[args.dtype], 6),
                "mfma": mfma,
                "wallclock": {"bytes_per_step": int(alg + adam_bytes), "achieved": round(wall_gbs, 2), "frac": round(wall_gbs / HBM_PEAK_GBS, 5), "note": "B_alg(step) = sum_g B_alg(g) + 28*P (Adam fp32) over ms_per_step"},
            },
            "step_split_us": None if reduce_ms is None else {"graph_pass": round(kernel_ms * 1e3, 2), "reduce_adam": round(reduce_ms * 1e3, 2), "other": round(ms_step * 1e3 - (kernel_ms + reduce_ms) * 1e3, 2), "note": "graph pass and dr_reduce_update each timed alone (HIP events around a HIP graph of max(--steps, 200) launches); other = ms_per_step minus both: the gaps between launches in the replayed step graphs"},
            "launch": ("eager" + capture_note) if captured is None else f"hipgraph-replay ({n_sweeps} x {len(handles)}-step sweep graph + " + (f"one {n_rest}-step graph" if rest is not None else f"{n_rest} per-step graphs") + f"{', RCCL all-reduce captured' if pg is not None else ''})",
            "cpu_baseline": cpu,
            "final_loss": float(loss.item()),
        }
        print(json.dumps(result), flush=True)
    if pg is not None:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    return result


if __name__ == "__main__":
    _argv = sys.argv[1:]
    _args = parse_args(_argv)
    if _args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch(_args.gpus, _argv))
    if _args.dry_run:
        dry_run(_args)
    elif _args.trainer:
        trainer_bench(_args)
    else:
        main(_args)
