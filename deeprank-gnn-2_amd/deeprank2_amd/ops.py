"""Thin torch-facing wrappers over the C ABI (device tensors in, device tensors out).

Each wrapper checks shapes/dtypes/devices, preallocates outputs with torch's
caching allocator, launches on the current stream and converts a non-zero
status into ``RuntimeError``.  No wrapper has a CPU path.
"""

from __future__ import annotations

import weakref

import torch

from deeprank2_amd import _lib

# Per edge_index tensor (held weakly; dropped when the tensor dies or is
# modified in place): its CSR, transposed CSR and range check.  A batch's
# edge_index is static across the layers and steps that reuse it (the layer
# path of layered.py), so those CSR builds and the host-syncing range check
# run once per tensor instead of once per call.
_GRAPHS: dict = {}


def _graph_entry(edge_index, n_rows):
    key = id(edge_index)
    ent = _GRAPHS.get(key)
    if ent is not None and (ent["ref"]() is not edge_index or ent["version"] != edge_index._version or ent["n"] != n_rows):
        ent = None
    if ent is None:
        ent = {"ref": weakref.ref(edge_index, lambda _r, k=key: _GRAPHS.pop(k, None)), "version": edge_index._version, "n": n_rows}
        _GRAPHS[key] = ent
    return ent


def check_edge_range(edge_index, n_rows):
    """IndexError if edge_index refers to a node outside [0, n_rows) (one host sync per tensor)."""
    ent = _graph_entry(edge_index, n_rows)
    if not ent.get("checked"):
        if edge_index.numel() and (int(edge_index.min()) < 0 or int(edge_index.max()) >= n_rows):
            msg = f"edge_index refers to a node outside [0, {n_rows})"
            raise IndexError(msg)
        ent["checked"] = True


def graph_csr(edge_index, n_rows, transpose=False):
    """(rowptr, perm, col) of edge_index by edge_index[0] (transpose: by
    edge_index[1]), stable; cached per tensor."""
    ent = _graph_entry(edge_index, n_rows)
    k = "tcsr" if transpose else "csr"
    if k not in ent:
        r, c = (edge_index[1], edge_index[0]) if transpose else (edge_index[0], edge_index[1])
        ent[k] = csr_from_coo(r, c, n_rows)
    return ent[k]


def _f32(t, name):
    if t.dtype != torch.float32:
        msg = f"{name} must be float32 (got {t.dtype})"
        raise TypeError(msg)
    return t.contiguous()


def csr_from_coo(row: torch.Tensor, col: torch.Tensor, n_rows: int):
    """Stable CSR of (row, col) sorted by row -> (rowptr int32 [n+1], perm int32 [E], col int32 [E])."""
    _lib.require_device(row, col)
    lib = _lib.load()
    row = row.to(torch.int64).contiguous()
    col = col.to(torch.int64).contiguous()
    e = row.numel()
    dev = row.device
    rowptr = torch.empty(n_rows + 1, dtype=torch.int32, device=dev)
    perm = torch.empty(max(e, 1), dtype=torch.int32, device=dev)
    col_s = torch.empty(max(e, 1), dtype=torch.int32, device=dev)
    scratch = torch.empty(n_rows + 1, dtype=torch.int32, device=dev)
    _lib.check(lib.dr_csr_from_coo(row.data_ptr(), col.data_ptr(), e, n_rows, rowptr.data_ptr(), perm.data_ptr(), col_s.data_ptr(), scratch.data_ptr(), _lib.stream_ptr(dev)), "dr_csr_from_coo")
    return rowptr, perm[:e], col_s[:e]


def spmm_csr(rowptr, col, y, n_rows, relu=False, mean=False):
    """Row sum (or row mean, NaN on empty rows) of y over a CSR adjacency."""
    _lib.require_device(rowptr, col, y)
    y = _f32(y, "y")
    out = torch.empty(n_rows, y.shape[1], dtype=torch.float32, device=y.device)
    _lib.check(_lib.load().dr_spmm_csr(rowptr.data_ptr(), col.data_ptr(), y.data_ptr(), n_rows, y.shape[1], int(relu) * _lib.DR_SPMM_RELU + int(mean) * _lib.DR_SPMM_MEAN, out.data_ptr(), _lib.stream_ptr(y.device)), "dr_spmm_csr")
    return out


def linear_xwT(x, w):
    _lib.require_device(x, w)
    x, w = _f32(x, "x"), _f32(w, "weight")
    m, k = x.shape
    n = w.shape[0]
    y = torch.empty(m, n, dtype=torch.float32, device=x.device)
    _lib.check(_lib.load().dr_linear_xwT(x.data_ptr(), w.data_ptr(), m, k, n, y.data_ptr(), _lib.stream_ptr(x.device)), "dr_linear_xwT")
    return y


def linear_xw(dy, w):
    _lib.require_device(dy, w)
    dy, w = _f32(dy, "dy"), _f32(w, "weight")
    m, n = dy.shape
    k = w.shape[1]
    dx = torch.empty(m, k, dtype=torch.float32, device=dy.device)
    _lib.check(_lib.load().dr_linear_xw(dy.data_ptr(), w.data_ptr(), m, n, k, dx.data_ptr(), _lib.stream_ptr(dy.device)), "dr_linear_xw")
    return dx


def linear_dw(dy, x):
    _lib.require_device(dy, x)
    dy, x = _f32(dy, "dy"), _f32(x, "x")
    m, n = dy.shape
    k = x.shape[1]
    n_split = max(1, min(64, m // 256))
    dw = torch.empty(n, k, dtype=torch.float32, device=dy.device)
    scratch = torch.empty(n_split * n * k, dtype=torch.float32, device=dy.device)
    _lib.check(_lib.load().dr_linear_dw(dy.data_ptr(), x.data_ptr(), m, n, k, dw.data_ptr(), scratch.data_ptr(), n_split, _lib.stream_ptr(dy.device)), "dr_linear_dw")
    return dw


class EdgeGraph:
    """CSR (by edge_index[0]) + transposed CSR + slot map + edge features in CSR order, on the device."""

    def __init__(self, edge_index, n, ea):
        row, col = edge_index[0], edge_index[1]
        self.rowptr, perm, self.col = csr_from_coo(row, col, n)
        self.trowptr, tperm, self.tcol = csr_from_coo(col, row, n)
        e = perm.numel()
        inv = torch.empty(max(e, 1), dtype=torch.int32, device=row.device)
        inv[perm.long()] = torch.arange(e, dtype=torch.int32, device=row.device)
        self.teid = inv[tperm.long()].contiguous() if e else inv
        self.ea = ea[perm.long()].contiguous() if e else ea.new_zeros((1, max(ea.shape[1], 1)))
        self.n = n


def edge_graph(edge_index, n, ea):
    _lib.require_device(edge_index, ea)
    return EdgeGraph(edge_index, n, ea)


def edge_mlp_scatter(g: EdgeGraph, a, b, we, be, f, fe):
    """S = sum over CSR rows of relu(A_i + B_j + We[:, 2F:] ea_e + be) (32 channels)."""
    s = torch.empty(g.n, 32, dtype=torch.float32, device=a.device)
    wc = we[:, 2 * f:]
    _lib.check(_lib.load().dr_edge_mlp_scatter(g.rowptr.data_ptr(), g.col.data_ptr(), g.n, a.data_ptr(), b.data_ptr(), g.ea.data_ptr(), fe, wc.data_ptr(), we.stride(0), be.data_ptr(), s.data_ptr(), _lib.stream_ptr(a.device)), "dr_edge_mlp_scatter")
    return s


def edge_mlp_scatter_bwd(g: EdgeGraph, a, b, we, be, f, fe, ds):
    dev = a.device
    d = torch.empty(g.n, 32, dtype=torch.float32, device=dev)
    dp = torch.empty_like(d)
    eap = torch.empty(g.n * 32 * max(fe, 1), dtype=torch.float32, device=dev)
    wc = we[:, 2 * f:]
    _lib.check(_lib.load().dr_edge_mlp_scatter_bwd(g.rowptr.data_ptr(), g.col.data_ptr(), g.trowptr.data_ptr(), g.tcol.data_ptr(), g.teid.data_ptr(), g.n, a.data_ptr(), b.data_ptr(), g.ea.data_ptr(), fe, wc.data_ptr(), we.stride(0), be.data_ptr(), ds.data_ptr(), d.data_ptr(), dp.data_ptr(), eap.data_ptr(), _lib.stream_ptr(dev)), "dr_edge_mlp_scatter_bwd")
    return d, dp, eap
