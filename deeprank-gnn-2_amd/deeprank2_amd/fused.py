"""Machinery shared by the per-graph fused models (GINet, FoutNet, ...).

* ``BatchHandle``: a mini-batch as the kernels see it — graph ids into an
  HBM-resident ``GraphStore`` plus their 64-byte ``dr_graph_desc`` records
  (this is the whole "collate" of ``trainer.py:541``).
* ``Dropout``: explicit keep mask, or the in-kernel counter hash.
* ``FusedSpec``: what a model contributes — its C graph-pass entry, weight
  struct, per-graph partial layout and the recipe that turns the partials
  into each parameter's gradient (``dr_reduce_update``).
* ``param_table`` / ``reduce_update``: the shared gradient reduction + Adam.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Callable

import numpy as np
import torch

from deeprank2_amd import _lib
from deeprank2_amd.store import GraphStore, pack_graphs, records_from_batch


class BatchHandle:
    """A mini-batch: graph ids into a store, with their device descriptors."""

    def __init__(self, store: GraphStore, gids_host: np.ndarray):
        self.store = store
        self.gids_host = np.ascontiguousarray(gids_host, dtype=np.int32)
        self.gids = torch.from_numpy(self.gids_host).to(store.device)
        self.descs = store.descriptors(self.gids_host)
        self.B = int(self.gids_host.size)
        self.max_sizes = store.max_sizes(self.gids_host)
        nf = store.packed.nonfinite
        self.nonfinite = bool(nf is not None and nf[self.gids_host.astype(np.int64)].any())
        self._lds = {}
        self.force_large = False  # run the split (tile + tail) path on small graphs too
        self.large_tile = None  # nodes per tile of the split path (default 128)
        self.large_halos = True  # stage each tile's neighbour rows in LDS (False: per-edge HBM gather)
        self.large_atomic_max = True  # depth-0 max over tiles by 64-bit atomic max (False: per-tile partials)
        self.force_layers = False  # run the layer-level path (layered.py) even when the graph pass fits (diagnostic)
        self.vanilla_words = True  # Vanilla pipeline: forward ReLU words feed the backward (False: recomputed)
        self.vanilla_split = None  # Vanilla per-graph kernel: workgroups per graph (None: by batch size)
        self.vanilla_tile_rows = VANILLA_CHUNK  # Vanilla pipeline: rows per halo-staged tile (64: the chunk-fused kernels; 16 / 32: edge kernels only; 0: untiled gathers)
        self.fault = None  # device uint32 [2] (dr_pass.fault) of the autograd path's passes, made on first use

    def lds(self, key, fn):
        """Dynamic LDS bytes for the largest graph of the batch (cached per model kind)."""
        v = self._lds.get(key)
        if v is None:
            v = int(fn(*self.max_sizes))
            self._lds[key] = v
        return v

    def vanilla_scratch(self, n_feat, n_edge_feat):
        """Node-level HBM scratch of dr_vanilla_graph_pass for this batch (row0 + buffer)."""
        key = ("vanilla", n_feat, n_edge_feat)
        sc = self._lds.get(key)
        if sc is None:
            n = self.store._sizes[0][self.gids_host.astype(np.int64)]  # noqa: SLF001
            row0 = np.concatenate([[0], np.cumsum(n)]).astype(np.int32)
            rows = int(row0[-1])
            slot = np.repeat(np.arange(self.B, dtype=np.int32), n)
            chunks = (n + VANILLA_CHUNK - 1) // VANILLA_CHUNK
            chunk_first = np.concatenate([[0], np.cumsum(chunks)]).astype(np.int32)
            chunk_slot = np.repeat(np.arange(self.B, dtype=np.int32), chunks)
            lib = _lib.load()
            floats = int(lib.dr_vanilla_scratch_floats(rows, n_feat, n_edge_feat))
            # the chunk-fused kernels (tiles of DR_VANILLA_CHUNK rows, Fe <= 4) keep both
            # layers' partial rows at once (dr_vanilla_scratch.part_layers)
            chunk_fused = self.vanilla_words and self.vanilla_tile_rows == VANILLA_CHUNK and 0 <= n_edge_feat <= 4 and n_feat <= 32  # noqa: PLR2004
            part_layers = 2 if chunk_fused else 1
            part = int(lib.dr_vanilla_part_floats(n_feat, n_edge_feat)) * int(chunk_first[-1]) * part_layers
            dev = self.store.device
            ints = torch.from_numpy(np.concatenate([row0, slot, chunk_first, chunk_slot])).to(dev)
            c = _lib.VanillaScratchC()
            buf = torch.empty(floats, dtype=torch.float32, device=dev)
            pbuf = torch.empty(part, dtype=torch.float32, device=dev)
            base = ints.data_ptr()
            c.base, c.row0, c.row_slot, c.n_rows = buf.data_ptr(), base, base + 4 * (self.B + 1), rows
            c.chunk_first = base + 4 * (self.B + 1 + rows)
            c.chunk_slot = base + 4 * (2 * (self.B + 1) + rows)
            c.n_chunks = int(chunk_first[-1])
            c.part = pbuf.data_ptr()
            c.part_layers = part_layers
            # per-edge ReLU words of both layers (forward -> backward);
            # vanilla_words = False: the backward recomputes them (diagnostic)
            ne = self.store._sizes[1][self.gids_host.astype(np.int64)]  # noqa: SLF001
            e0 = torch.from_numpy(np.concatenate([[0], np.cumsum(ne)]).astype(np.int32)).to(dev)
            words = torch.empty(max(1, 2 * int(ne.sum())), dtype=torch.int32, device=dev)
            keep = [ints, buf, pbuf, e0, words]
            if self.vanilla_words:
                c.edge0, c.relu_words = e0.data_ptr(), words.data_ptr()
                if self.vanilla_tile_rows:
                    tr = int(self.vanilla_tile_rows)
                    meta = [] if chunk_fused else None
                    plan = vanilla_tile_plan(self, n, row0, tr, n_edge_feat, meta_out=meta)
                    if plan is not None:
                        tensors, (n_tiles, hmax, emax, tmax) = plan
                        keep += tensors
                        (c.tile_row0, c.halo_off, c.halo_ids, c.lcol_off, c.lcol, c.ltcol_off, c.ltcol) = (t.data_ptr() for t in tensors)
                        c.n_tiles, c.halo_max, c.tile_edges_max, c.tile_tedges_max = n_tiles, hmax, emax, tmax
                        c.tile_rows = tr
                        if meta:
                            m = np.zeros(len(meta), dtype=VTILE_DTYPE)
                            for k, name in enumerate(VTILE_DTYPE.names[:-1]):
                                m[name] = [row[k] for row in meta]
                            mt = torch.from_numpy(m.view(np.uint8)).to(dev)
                            pm = torch.empty(len(meta) * 32, dtype=torch.float32, device=dev)  # per-tile column sums of X2
                            keep += [mt, pm]
                            c.tile_meta, c.part_mean = mt.data_ptr(), pm.data_ptr()
                        if VANILLA_CHUNK % tr == 0 and 0 < n_edge_feat <= 4 and not chunk_fused:  # the 16/32-row tiled kernels; tiles never straddle a weight-gradient chunk
                            tfirst = torch.from_numpy(np.concatenate([[0], np.cumsum((n + tr - 1) // tr)]).astype(np.int32)).to(dev)
                            twc = torch.empty(n_tiles * 32 * max(1, n_edge_feat), dtype=torch.float32, device=dev)
                            keep += [tfirst, twc]
                            c.tile_wc, c.tile_first, c.tile_rows = twc.data_ptr(), tfirst.data_ptr(), tr
            sc = (c, tuple(keep))
            self._lds[key] = sc
        return sc

    def vanilla_fused_scratch(self):
        """Per-graph global scratch of dr_vanilla_fused_pass (S1, the edge ReLU
        words of both layers in CSR order, the split's exchange rows), each
        slot's float offset into it, and the split's arrival counters."""
        sc = self._lds.get("vanilla_fused_scratch")
        if sc is None:
            idx = self.gids_host.astype(np.int64)
            n, e = self.store._sizes[0][idx], self.store._sizes[1][idx]  # noqa: SLF001
            per = vanilla_fused_scratch_floats(n, e, self.store.n_edge_feat)
            off = np.concatenate([[0], np.cumsum(per)]).astype(np.int64)
            dev = self.store.device
            buf = torch.empty(max(1, int(off[-1])), dtype=torch.float32, device=dev)
            offs = torch.from_numpy(off[:-1].copy()).to(dev)
            sync = torch.zeros(2 * self.B + 1, dtype=torch.int32, device=dev)  # arrival counters, left zero by every launch
            wpack = torch.empty(int(_lib.load().dr_vanilla_wpack_floats()), dtype=torch.float32, device=dev)  # weights in fragment order
            sc = (buf, offs, sync, wpack)
            self._lds["vanilla_fused_scratch"] = sc
        return sc

    def vanilla_sync_ok(self):
        """False if a VanillaNetwork split launch on this batch gave up waiting
        for a sibling workgroup (its timeout flag; one device read)."""
        sc = self._lds.get("vanilla_fused_scratch")
        return sc is None or int(sc[2][-1].item()) == 0

    def large_plan(self, out_dim, bf16=False, kind="ginet"):
        """Tiling + workspaces of the large-graph path (dr_large_plan), built once per batch
        (kind: "ginet", or "fout" / "sgat" for dr_fout_large_pass / dr_sgat_large_pass)."""
        plan = self._lds.get(("large", out_dim, bf16, kind))
        if plan is None:
            if kind == "ginet":
                plan = LargePlan(self, out_dim, use_halos=self.large_halos, use_atomic_max=self.large_atomic_max, bf16=bf16)
            else:
                plan = LargePlan(self, out_dim, use_halos=self.large_halos, use_atomic_max=True, kind=kind)
            self._lds[("large", out_dim, bf16, kind)] = plan
        return plan


LDS_MAX = 160 * 1024
VANILLA_CHUNK = 64  # DR_VANILLA_CHUNK: rows per weight-gradient partial of the Vanilla pipeline


# dr_vanilla_tile (include/deeprank2_amd.h): one chunk-fused tile's offsets, 128 bytes
VTILE_DTYPE = np.dtype([(k, "<i8") for k in ("rt0", "g0", "rp0", "col0", "xrow", "word0")]
                       + [(k, "<i4") for k in ("nr", "slot", "i0", "e0", "ne", "q0", "nq", "h0", "n_halo", "lcol_off", "ltcol_off", "n_graph", "e_graph")]
                       + [("pad", "<i4", (7,))])  # fmt: skip


def vanilla_tile_plan(h: BatchHandle, n, row0, tile_rows, n_edge_feat, lds_check=True, meta_out=None):
    """Edge-tile plan of the VanillaNetwork pipeline (dr_vanilla_scratch tile_*
    fields; also ginet_nocluster's large-graph pipeline, dr_nc_plan): each graph's rows cut into tiles of ``tile_rows``; per tile the
    ascending union of its rows' out- and in-neighbours (the halo staged in LDS)
    and every CSR / transposed edge's column as an index into it.  None when a
    tile's LDS would exceed one workgroup's 160 KiB (the untiled kernels run).
    ``meta_out`` (a list): receives each tile's dr_vanilla_tile fields."""
    p = h.store.packed
    tile_row0, hoff, hids, loff, lcs, toff, tcs = [0], [0], [], [0], [], [0], []
    hmax = emax = tmax = 0
    word0 = 0
    for slot, gid in enumerate(h.gids_host.astype(np.int64)):
        ng = int(n[slot])
        n0, e0, e1 = int(p.node_off[gid]), int(p.edge_off[gid]), int(p.edge_off[gid + 1])
        rp = p.rowptr[n0 + gid : n0 + gid + ng + 1].astype(np.int64)
        trp = p.t_rowptr[n0 + gid : n0 + gid + ng + 1].astype(np.int64)
        col, tcol = p.col[e0:e1], p.t_col[e0:e1]
        for r0 in range(0, ng, tile_rows):
            r1 = min(ng, r0 + tile_rows)
            cs, ts = col[rp[r0] : rp[r1]], tcol[trp[r0] : trp[r1]]
            halo = np.union1d(cs, ts).astype(np.int32)
            if meta_out is not None:
                meta_out.append((int(row0[slot]) + r0, int(row0[slot]), n0 + int(gid), int(h.store.col_off_host[gid]), n0 + r0, word0,
                                 r1 - r0, slot, r0, int(rp[r0]), cs.size, int(trp[r0]), ts.size, hoff[-1], halo.size, loff[-1], toff[-1], ng, e1 - e0))
            hids.append(halo)
            hoff.append(hoff[-1] + halo.size)
            lcs.append(np.searchsorted(halo, cs).astype(np.uint16))
            loff.append(loff[-1] + cs.size)
            tcs.append(np.searchsorted(halo, ts).astype(np.uint16))
            toff.append(toff[-1] + ts.size)
            tile_row0.append(int(row0[slot]) + r1)
            hmax, emax, tmax = max(hmax, halo.size), max(emax, cs.size), max(tmax, ts.size)
        word0 += e1 - e0
    n_tiles = len(tile_row0) - 1
    if n_tiles == 0 or hmax == 0 or hmax > 65535:  # noqa: PLR2004
        return None
    rs = 4 if n_edge_feat <= 3 else 8  # floats per CSR edge record
    lds = 4 * (hmax * 32 + emax * rs + 2 * tmax)  # tile_carve (backward, the larger)
    if lds_check and lds > LDS_MAX:
        return None
    dev = h.store.device
    cat16 = lambda parts: np.concatenate([*parts, np.zeros(8, np.uint16)])  # noqa: E731
    arrays = [np.asarray(tile_row0, np.int32), np.asarray(hoff, np.int32), np.concatenate(hids), np.asarray(loff, np.int32), cat16(lcs).view(np.int16), np.asarray(toff, np.int32), cat16(tcs).view(np.int16)]
    return [torch.from_numpy(a).to(dev) for a in arrays], (n_tiles, hmax, emax, tmax)


class LargePlan:
    """Host side of ``dr_large_plan``: tiles of DR_LARGE_TILE nodes per graph,
    the Z workspace and the per-tile partial pooling buffers."""

    TILE = 64  # measured best for atom-level graphs with tile halos (tools/large_tiles.py)

    def __init__(self, h: BatchHandle, out_dim, tile_rows=None, use_halos=True, use_atomic_max=True, bf16=False, kind="ginet"):
        st = h.store
        self.kind = kind
        self.TILE = int(tile_rows or h.large_tile or self.TILE)
        n, _e, k0, p1, k1 = (a[h.gids_host.astype(np.int64)] for a in st._sizes)  # noqa: SLF001
        self.k0_max = int(k0.max())
        if self.k0_max > 64:  # noqa: PLR2004
            msg = f"a graph of the batch has {self.k0_max} depth-0 clusters (> 64): not supported by the large-graph path"
            raise RuntimeError(msg)
        tiles = (n + self.TILE - 1) // self.TILE
        tile_first = np.concatenate([[0], np.cumsum(tiles)]).astype(np.int32)
        z_row0 = np.concatenate([[0], np.cumsum(n)]).astype(np.int32)
        tile_slot = np.repeat(np.arange(h.B, dtype=np.int32), tiles)
        self.n_tiles = int(tile_first[-1])
        dev = st.device
        self.ints = torch.from_numpy(np.concatenate([tile_first, z_row0, tile_slot])).to(dev)
        # z rows: GINet's Z = A X; FoutNet's Zm (stride r4(F)); SGAT's Zw + c1 (r4(F) + 4)
        self.zs = st.x_stride + (4 if kind == "sgat" else 0)
        self.z = torch.empty(max(1, int(z_row0[-1])) * self.zs, dtype=torch.float32, device=dev)
        self.part_val = torch.empty(self.n_tiles * self.k0_max * 32, dtype=torch.float32, device=dev)
        self.part_arg = torch.empty(self.n_tiles * self.k0_max * 32, dtype=torch.int32, device=dev)
        self.part_key = torch.zeros(h.B * self.k0_max * 32, dtype=torch.int64, device=dev)  # kept zero between passes
        lib = _lib.load()
        halo = self._halos(h, n) if use_halos else None
        hmax, emax = (halo[0], halo[1]) if halo is not None else (0, 0)
        if kind == "ginet":
            conv_lds = lib.dr_ginet_large_conv_lds_bytes_bf16 if bf16 else lib.dr_ginet_large_conv_lds_bytes
        else:
            sg = int(kind == "sgat")
            conv_lds = lambda *a: lib.dr_fout_large_conv_lds_bytes(*a, sg)  # noqa: E731
        self.conv_lds = int(conv_lds(int(n.max()), st.n_feat, self.k0_max, hmax, emax))
        if halo is not None and self.conv_lds > LDS_MAX:  # halos too wide for LDS: per-edge HBM gather
            halo, hmax = None, 0
            self.conv_lds = int(conv_lds(int(n.max()), st.n_feat, self.k0_max, 0, 0))
        tail_args = (self.k0_max, int(p1.max()), int(k1.max()), int(st.packed.transpose_aliased), out_dim)
        self.tail_lds = int(lib.dr_ginet_tail_lds_bytes(*tail_args) if kind == "ginet" else lib.dr_fout_tail_lds_bytes(*tail_args, int(kind == "sgat")))
        if max(self.conv_lds, self.tail_lds) > LDS_MAX:
            msg = f"large-graph path needs {max(self.conv_lds, self.tail_lds)} B of LDS (> 160 KiB)"
            raise RuntimeError(msg)
        c = _lib.LargePlanC()
        base = self.ints.data_ptr()
        c.tile_first = base
        c.z_row0 = base + 4 * (h.B + 1)
        c.tile_slot = base + 8 * (h.B + 1)
        c.n_tiles = self.n_tiles
        c.k0_max = self.k0_max
        c.tile_rows = self.TILE
        c.z = self.z.data_ptr()
        c.part_val = self.part_val.data_ptr()
        c.part_arg = self.part_arg.data_ptr()
        c.halo_max = hmax
        c.part_key = self.part_key.data_ptr() if use_atomic_max else None
        c.arrive = None
        self.halo_tensors = None
        if halo is not None:
            _, _, hoff, hids, loff, lcol, tmem, tmptr = halo
            self.halo_tensors = [torch.from_numpy(a).to(dev) for a in (hoff, hids, loff, lcol.view(np.int16), tmem, tmptr)]
            c.halo_off, c.halo_ids, c.lcol_off, c.lcol, c.tile_members, c.tile_mptr = (t.data_ptr() for t in self.halo_tensors)
        self.c = c

    def _halos(self, h, n):
        """Per tile: its neighbours (distinct local node ids, ascending) and its
        edges re-indexed into that list (uint16), 8-aligned per tile."""
        p = h.store.packed
        hoff, hids, loff, lcols = [0], [], [0], []
        tmem = np.zeros((self.n_tiles, self.TILE), np.int32)
        tmptr = np.zeros((self.n_tiles, self.k0_max + 1), np.int32)
        tile = 0
        hmax = emax = 0
        for slot, gid in enumerate(h.gids_host.astype(np.int64)):
            n0, e0 = int(p.node_off[gid]), int(p.edge_off[gid])
            rp = p.rowptr[n0 + gid : n0 + gid + int(n[slot]) + 1].astype(np.int64)
            col = p.col[e0 : int(p.edge_off[gid + 1])]
            cl0 = p.cl0[n0 : n0 + int(n[slot])]
            k0 = int(p.k0_off[gid + 1] - p.k0_off[gid])
            for r0 in range(0, int(n[slot]), self.TILE):
                r1 = min(int(n[slot]), r0 + self.TILE)
                order = np.argsort(cl0[r0:r1], kind="stable")  # by cluster, nodes ascending
                tmem[tile, : r1 - r0] = r0 + order
                np.cumsum(np.bincount(cl0[r0:r1], minlength=k0), out=tmptr[tile, 1 : k0 + 1])
                tile += 1
                cs = col[rp[r0] : rp[r1]]
                uniq, inv = np.unique(cs, return_inverse=True)
                hids.append(uniq.astype(np.int32))
                hoff.append(hoff[-1] + uniq.size)
                pad = (-cs.size) % 8
                lcols.append(np.concatenate([inv.astype(np.uint16), np.zeros(pad, np.uint16)]))
                loff.append(loff[-1] + cs.size + pad)
                hmax, emax = max(hmax, uniq.size), max(emax, cs.size)
        if hmax == 0 or hmax > 65535:
            return None
        lcol = np.concatenate([*lcols, np.zeros(8, np.uint16)])
        return hmax, emax, np.asarray(hoff, np.int32), np.concatenate(hids), np.asarray(loff, np.int32), lcol, tmem.reshape(-1), tmptr.reshape(-1)


def resolve_batch(data, device, require_clusters=True) -> BatchHandle:
    """Our DataLoader's batches name their graphs in the dataset's resident
    store; any other PyG-style batch is packed here (one upload per call).
    Models that pool (GINet, FoutNet) need the stored clusters, as the
    reference's get_preloaded_cluster does."""
    h = getattr(data, "_dr_handle", None)
    if h is None:
        fn = getattr(data, "dr_handle", None)
        h = fn(device) if callable(fn) else None
    if h is None:
        store = GraphStore(pack_graphs(records_from_batch(data), require_clusters=require_clusters), device)
        h = BatchHandle(store, np.arange(store.n_graphs, dtype=np.int32))
    if require_clusters and not h.store.packed.has_clusters:
        msg = "this model pools over the stored clusters: build the dataset with clustering_method set (cluster0/cluster1 are missing)"
        raise ValueError(msg)
    return h


class Dropout:
    """``mask`` (uint8 [B,128] keep mask) or the in-kernel counter hash ``(seed, offset)``."""

    def __init__(self, p, mask=None, seed=None, offset=0):
        self.p = float(p)
        self.mask = mask
        self.seed = seed
        self.offset = int(offset)

    @property
    def scale(self):
        return 1.0 / (1.0 - self.p)


@dataclass
class FusedSpec:
    param_names: list
    recipe: Callable  # (F, out) -> [(kind, off1, off2, cols)] per parameter
    slab_stride: Callable  # F -> floats per graph
    head_stride: Callable  # out -> floats per graph
    entry: str  # C graph-pass entry point
    weights: Callable  # params -> ctypes weights struct
    lds: Callable  # (n, e, k0, p1, k1, F, alias, out) -> bytes
    dropout: float = 0.0
    slab_rows: int = 1  # most slab rows a graph's pass writes (slab_stride(F) covers them all)
    slab_k: Callable | None = None  # handle -> slab rows per graph of that batch's pass (default 1)
    large: Callable | None = None  # (handle, weights struct, pass struct) for graphs beyond one workgroup's LDS
    run: Callable | None = None  # (handle, weights struct, pass struct): replaces the default entry call
    layers: Callable | None = None  # (model, batch tensors, training) -> out: layer-level path (layered.py) for batches beyond LDS
    bf16: bool = False  # dr_pass.compute_dtype = DR_DTYPE_BF16 supported (runs on the large-graph path)
    attention: bool = False  # GINetConvLayer model: batches with non-finite inputs need the layer path
    handoffs: bool = False  # the graph pass hands rows between workgroups in-launch (dr_pass.fault can be set)
    wpack: Callable | None = None  # params -> (packed weights, dr_adam.mirror_idx, refresh()): run(..., wpack=) takes the buffer as current


def vanilla_fused_scratch_floats(n, e, fe):
    """Mirror of dr_vanilla_fused_scratch_floats (vanilla_graph.hip), vectorised
    over graphs: S1 (32N), two ReLU word arrays (E + 1 each, CSR order), the
    split's exchange rows XA, XB (32N each) and column sums (4 x 32), every part
    rounded up to 16 bytes (fe: no per-edge-feature part since r03)."""
    r4 = lambda v: (np.asarray(v, dtype=np.int64) + 3) & ~3  # noqa: E731
    del fe
    return 3 * r4(32 * np.asarray(n, dtype=np.int64)) + 2 * r4(np.asarray(e, dtype=np.int64) + 1) + 32 * 4


def make_pass(out_dim, flags, *, dropout: Dropout | None = None, dout=None, loss_kind=_lib.DR_LOSS_NONE, loss_scale=1.0, class_w=None, out=None, loss_per_graph=None, slab=None, head=None, stamps=None, step_counter=None, fault=None, spin_limit=0):
    p = _lib.PassC()
    p.flags = flags
    p.out_dim = out_dim
    p.loss_kind = loss_kind
    if dropout is None:
        p.use_dropout = _lib.DR_DROPOUT_OFF
    elif dropout.mask is not None:
        p.use_dropout = _lib.DR_DROPOUT_MASK
        p.drop_scale = dropout.scale
        p.mask = dropout.mask.data_ptr()
    else:
        p.use_dropout = _lib.DR_DROPOUT_HASH
        p.drop_scale = dropout.scale
        p.drop_p = dropout.p
        p.drop_seed = dropout.seed
        p.drop_offset = dropout.offset
    p.loss_scale = loss_scale
    p.class_w = _lib.ptr(class_w)
    p.out = _lib.ptr(out)
    p.dout = _lib.ptr(dout)
    p.loss_per_graph = _lib.ptr(loss_per_graph)
    p.slab = _lib.ptr(slab)
    p.head = _lib.ptr(head)
    p.stamps = _lib.ptr(stamps)
    p.step_counter = _lib.ptr(step_counter)
    p.fault = _lib.ptr(fault)
    p.spin_limit = int(spin_limit)
    return p


def lds_for(spec: FusedSpec, h: BatchHandle, out_dim):
    alias = int(h.store.packed.transpose_aliased)
    f = h.store.n_feat
    return h.lds((spec.entry, out_dim), lambda n, e, k0, p1, k1: spec.lds(n, e, k0, p1, k1, f, alias, out_dim))


def launch(spec: FusedSpec, h: BatchHandle, w, p, wpack=None):
    """One graph pass on the current stream: the single-workgroup kernel when
    the batch's largest graph fits in LDS, else the model's large-graph path.
    wpack: the model's packed weights, already current (``FusedSpec.wpack``)."""
    if spec.run is not None:
        if wpack is not None:
            spec.run(h, w, p, wpack=wpack)
        else:
            spec.run(h, w, p)
        return
    if p.compute_dtype == _lib.DR_DTYPE_BF16:
        if not spec.bf16 or spec.large is None:
            msg = f"{spec.entry}: no bf16 compute path"
            raise RuntimeError(msg)
        if h.store.x_bf16 is None:
            msg = "bf16 compute needs the store's bf16 copy of x: GraphStore(packed, device, dtype='bf16')"
            raise RuntimeError(msg)
        spec.large(h, w, p)  # the tile kernel holds the bf16 node GEMM, for every graph size
        return
    lds = lds_for(spec, h, p.out_dim)
    if lds <= LDS_MAX and not (h.force_large and spec.large is not None):
        fn = getattr(_lib.load(), spec.entry)
        _lib.check(fn(h.store.cstruct(), h.descs.data_ptr(), h.B, w, p, lds, _lib.stream_ptr(h.store.device)), spec.entry)
    elif spec.large is not None:
        spec.large(h, w, p)
    else:
        msg = f"largest graph of the batch needs {lds} B of LDS (> 160 KiB) and {spec.entry} has no large-graph path"
        raise RuntimeError(msg)


def _device_cus(device):
    try:
        return int(torch.cuda.get_device_properties(torch.device(device)).multi_processor_count)
    except (RuntimeError, AssertionError, ValueError):
        return 256


def run_pass(spec: FusedSpec, h: BatchHandle, params, p, w=None):
    """Launch the model's graph pass on the current stream."""
    launch(spec, h, spec.weights(params) if w is None else w, p)


def param_table(spec: FusedSpec, params, grads, states, n_feat, out_dim):
    t = _lib.ParamTableC()
    recipe = spec.recipe(n_feat, out_dim)
    if len(params) != len(recipe) or len(params) > _lib.DR_MAX_PARAMS:
        msg = "parameter list and gradient recipe disagree"
        raise ValueError(msg)
    for i, prm in enumerate(params):
        t.param[i] = prm.data_ptr()
        t.grad[i] = None if grads is None or grads[i] is None else grads[i].data_ptr()
        t.numel[i] = prm.numel()
        if states is not None:
            t.exp_avg[i] = states[i][0].data_ptr()
            t.exp_avg_sq[i] = states[i][1].data_ptr()
        kind, off1, off2, cols = recipe[i]
        t.recipe[i].kind, t.recipe[i].off1, t.recipe[i].off2, t.recipe[i].cols = kind, off1, off2, cols
    t.n_params = len(params)
    t.slab_stride = spec.slab_stride(n_feat) // spec.slab_rows  # floats per slab row
    t.head_stride = spec.head_stride(out_dim)
    t.slab_rows = 1  # set per batch (slab_rows_for) before each reduce
    return t


def slab_rows_for(spec: FusedSpec, h: BatchHandle) -> int:
    """Slab rows per graph the model's pass writes for this batch."""
    return 1 if spec.slab_k is None else int(spec.slab_k(h))


def reduce_update(table, B, slab, head, device, adam=None, loss_per_graph=None, loss_scale=1.0, loss_out=None, fault=None):
    a = adam if adam is not None else _lib.AdamC()
    if fault is not None:
        a.fault = fault.data_ptr()
    rc = _lib.load().dr_reduce_update(table, _lib.ptr(slab), _lib.ptr(head), B, a, _lib.ptr(loss_per_graph), loss_scale, _lib.ptr(loss_out), _lib.stream_ptr(device))
    _lib.check(rc, "dr_reduce_update")


class FusedFn(torch.autograd.Function):
    """Autograd bridge: forward = graph pass (FORWARD); backward = graph pass
    (BACKWARD, upstream dout) + gradient reduction into every parameter."""

    @staticmethod
    def forward(ctx, spec, h, dropout, out_dim, *params):
        out = torch.empty(h.B, out_dim, dtype=torch.float32, device=h.store.device)
        run_pass(spec, h, params, make_pass(out_dim, _lib.DR_PASS_FORWARD, dropout=dropout, out=out))
        ctx.spec, ctx.h, ctx.dropout, ctx.out_dim = spec, h, dropout, out_dim
        ctx.save_for_backward(*params)
        return out

    @staticmethod
    def backward(ctx, dout):
        params = ctx.saved_tensors
        spec, h, out_dim = ctx.spec, ctx.h, ctx.out_dim
        dev = h.store.device
        f = h.store.n_feat
        slab = torch.empty(h.B * spec.slab_stride(f), dtype=torch.float32, device=dev)
        head = torch.zeros(h.B * spec.head_stride(out_dim), dtype=torch.float32, device=dev)
        fault = None
        if spec.handoffs:  # a hand-off that gave up: NaN gradients rather than wrong ones
            if h.fault is None:
                h.fault = torch.zeros(2, dtype=torch.int32, device=dev)
            fault = h.fault
        run_pass(spec, h, params, make_pass(out_dim, _lib.DR_PASS_BACKWARD, dropout=ctx.dropout, dout=dout.contiguous(), slab=slab, head=head, fault=fault))
        grads = [torch.empty_like(p) for p in params]
        t = param_table(spec, params, grads, None, f, out_dim)
        t.slab_rows = slab_rows_for(spec, h)
        reduce_update(t, h.B, slab, head, dev, fault=fault)
        return (None, None, None, None, *grads)
