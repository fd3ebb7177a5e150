"""The C-ABI library loads on a CPU-only host and exports every symbol
``include/deeprank2_amd.h`` declares (no compute calls without a GPU)."""

from __future__ import annotations

import ctypes
import os
import re

from conftest import ROOT

from deeprank2_amd import _lib


def _declared():
    src = open(os.path.join(ROOT, "include", "deeprank2_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dr_[A-Za-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_entry():
    lib = _lib.load()
    declared = _declared()
    assert "dr_ginet_graph_pass" in declared
    for name in declared:
        assert hasattr(lib, name), name
    assert sorted(n for n, *_ in _lib.SIGNATURES) == declared


def test_version_and_lds_query_are_host_only():
    lib = _lib.load()
    assert b"gfx950" in lib.dr_version()
    small = lib.dr_ginet_lds_bytes(200, 3000, 30, 5, 20, 1, 1, 1)
    big = lib.dr_ginet_lds_bytes(200, 3000, 30, 5, 20, 1, 0, 1)
    assert 0 < small < big <= 200 * 1024
    assert small % 16 == 0


def test_struct_layouts_match_header():
    # 4 int32 + 20 pointers; 8 pointers; 4 int32 + 2 float + 2 uint64 + float/int32 + 7 pointers
    assert ctypes.sizeof(_lib.GraphStoreC) == 16 + 22 * 8 + 8 + 2 * 8 + 8 + 8 + 8  # ... x_bf16, x_bf16_stride + pad, cl0
    assert ctypes.sizeof(_lib.GinetWeightsC) == 8 * 8
    assert ctypes.sizeof(_lib.FoutWeightsC) == 10 * 8
    assert ctypes.sizeof(_lib.LargePlanC) == 3 * 8 + 16 + 3 * 8 + 7 * 8 + 8  # ... part_key, arrive
    assert ctypes.sizeof(_lib.PassC) == 16 + 8 + 16 + 8 + 9 * 8 + 8 + 8 + 8  # + fault, spin_limit, slot
    assert ctypes.sizeof(_lib.AdamC) == 32 + 8 + 8 + 8 + 4 * 8  # + grad_div, fault, mirror, mirror_idx, fault_clear, ticket
    assert ctypes.sizeof(_lib.MclGraphsC) == 10 * 8
    assert ctypes.sizeof(_lib.VanillaScratchC) == 6 * 8 + 8 + 3 * 8 + 7 * 8 + 16 + 2 * 8 + 8 + 8 + 8  # ... tile plan, tile_wc, tile_first, tile_meta, part_mean
    from deeprank2_amd.fused import VTILE_DTYPE  # noqa: PLC0415

    assert VTILE_DTYPE.itemsize == 128  # dr_vanilla_tile: 6 int64 + 13 int32 + 7 pad
    assert ctypes.sizeof(_lib.ParamTableC) == 4 * 24 * 8 + 24 * 4 + 24 * 16 + 16


def test_library_is_built_for_gfx950():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_dropout_hash_host_replica_statistics():
    keep = _lib.dropout_keep_host(1234, 7, 128 * 512, 0.4)
    assert abs(keep.mean() - 0.6) < 0.01
    again = _lib.dropout_keep_host(1234, 7, 128 * 512, 0.4)
    other = _lib.dropout_keep_host(1234, 8, 128 * 512, 0.4)
    assert (keep == again).all()
    assert (keep != other).mean() > 0.3


def test_vanilla_fused_sizes_host_mirror():
    """The host's per-graph scratch sizing (fused.vanilla_fused_scratch_floats)
    equals the library's, and residue graphs of SURVEY §8(d) up to N=220,
    E=3606 fit one workgroup's 160 KiB of LDS for Fe <= 3."""
    import numpy as np  # noqa: PLC0415

    from deeprank2_amd.fused import vanilla_fused_scratch_floats  # noqa: PLC0415

    lib = _lib.load()
    for n, e, fe in [(1, 0, 0), (1, 1, 1), (33, 190, 2), (200, 3000, 3), (220, 3606, 4), (57, 342, 2)]:
        assert int(vanilla_fused_scratch_floats(np.array([n]), np.array([e]), fe)[0]) == lib.dr_vanilla_fused_scratch_floats(n, e, fe)
        assert lib.dr_vanilla_fused_lds_bytes(n, e, fe) % 16 == 0
    for fe in (1, 2, 3):
        assert lib.dr_vanilla_fused_lds_bytes(220, 3606, fe) <= 160 * 1024


def test_vanilla_fused_pass_argument_checks_are_host_only():
    """dr_vanilla_fused_pass refuses a split outside 1..DR_VANILLA_MAX_SPLIT and
    missing sync / wpack buffers before touching the GPU; the fragment-order
    weight buffer has a fixed size; dr_param_table.slab_rows is the field the
    split's partial rows are summed by."""
    lib = _lib.load()
    wpack = int(lib.dr_vanilla_wpack_floats())
    assert wpack > 0 and wpack % 64 == 0
    st, w, p = _lib.GraphStoreC(), _lib.VanillaWeightsC(), _lib.PassC()
    p.out_dim = 1
    st.n_feat, st.x_stride, st.n_edge_feat = 30, 32, 3
    dummy = ctypes.c_void_p(16)  # never dereferenced: the checks return first
    for split, sync, wp in [(0, dummy, dummy), (5, dummy, dummy), (4, None, dummy), (4, dummy, None)]:
        rc = lib.dr_vanilla_fused_pass(ctypes.byref(st), dummy, 8, ctypes.byref(w), ctypes.byref(p), dummy, dummy, split, sync, wp, 1024, None)
        assert rc == -1, (split, sync, wp, rc)  # DR_E_ARG
    assert [f for f, _ in _lib.ParamTableC._fields_][-1] == "slab_rows"
