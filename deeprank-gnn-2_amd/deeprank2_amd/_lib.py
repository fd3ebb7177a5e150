"""ctypes binding of the C ABI declared in ``include/deeprank2_amd.h``.

The shared library ``libdeeprank2_amd.so`` is built in-tree (``make -C
deeprank-gnn-2_amd/csrc`` or ``__graft_entry__.build()``).  There is no CPU
fallback: if the library is missing, or a compute entry is called with
non-device tensors, an error is raised.
"""

from __future__ import annotations

import ctypes
import os

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), os.environ.get("DR_LIB_NAME", "libdeeprank2_amd.so"))

DR_PASS_FORWARD = 1
DR_PASS_BACKWARD = 2
DR_PASS_WPACK_CURRENT = 4
DR_LOSS_NONE = 0
DR_LOSS_MSE = 1
DR_LOSS_CE = 2
DR_MAX_OUT = 16
DR_DROPOUT_OFF = 0
DR_DROPOUT_MASK = 1
DR_DROPOUT_HASH = 2
DR_MAX_PARAMS = 24
DR_GRAD_ZERO = 0
DR_GRAD_SLAB = 1
DR_GRAD_OUTER = 2
DR_GRAD_HEAD = 3
DR_SPMM_RELU = 1
DR_SPMM_MEAN = 2
DR_SPMM_MEAN_CLAMP = 4

ERRORS = {-1: "bad argument", -2: "graph does not fit the per-graph LDS kernel", -3: "unsupported configuration"}

_c_f = ctypes.POINTER(ctypes.c_float)
_c_i32 = ctypes.POINTER(ctypes.c_int32)
_c_i64 = ctypes.POINTER(ctypes.c_int64)
_c_u8 = ctypes.POINTER(ctypes.c_uint8)
VP = ctypes.c_void_p


class GraphStoreC(ctypes.Structure):
    _fields_ = [
        ("n_graphs", ctypes.c_int32),
        ("n_feat", ctypes.c_int32),
        ("x_stride", ctypes.c_int32),
        ("transpose_aliased", ctypes.c_int32),
        ("x", VP),
        ("node_off", VP),
        ("edge_off", VP),
        ("col_off", VP),
        ("rowptr", VP),
        ("col", VP),
        ("t_rowptr", VP),
        ("t_col", VP),
        ("k0_off", VP),
        ("m0_ptr", VP),
        ("m0_idx", VP),
        ("p1_off", VP),
        ("p1_rowptr", VP),
        ("p1_col", VP),
        ("p1t_rowptr", VP),
        ("p1t_col", VP),
        ("k1_off", VP),
        ("m1_ptr", VP),
        ("m1_idx", VP),
        ("y", VP),
        ("ea", VP),
        ("t_eid", VP),
        ("n_edge_feat", ctypes.c_int32),
        ("pad0", ctypes.c_int32),
        ("p1_ea", VP),
        ("p1t_pid", VP),
        ("x_bf16", VP),
        ("x_bf16_stride", ctypes.c_int32),
        ("pad1", ctypes.c_int32),
        ("cl0", VP),
    ]


class GinetWeightsC(ctypes.Structure):
    _fields_ = [(n, VP) for n in ("w1", "w1e", "w2", "w2e", "fc1w", "fc1b", "fc2w", "fc2b")]


class LargePlanC(ctypes.Structure):
    _fields_ = [
        ("tile_first", VP),
        ("z_row0", VP),
        ("tile_slot", VP),
        ("n_tiles", ctypes.c_int32),
        ("k0_max", ctypes.c_int32),
        ("tile_rows", ctypes.c_int32),
        ("halo_max", ctypes.c_int32),
        ("z", VP),
        ("part_val", VP),
        ("part_arg", VP),
        ("halo_off", VP),
        ("halo_ids", VP),
        ("lcol_off", VP),
        ("lcol", VP),
        ("tile_members", VP),
        ("tile_mptr", VP),
        ("part_key", VP),
        ("arrive", VP),
    ]


class FoutWeightsC(ctypes.Structure):
    _fields_ = [(n, VP) for n in ("wc1", "wn1", "b1", "wc2", "wn2", "b2", "fc1w", "fc1b", "fc2w", "fc2b")]


class VanillaWeightsC(ctypes.Structure):
    _fields_ = [(n, VP) for n in ("we1", "be1", "wn1", "bn1", "we2", "be2", "wn2", "bn2", "g1w", "g1b", "g2w", "g2b")]


class VanillaScratchC(ctypes.Structure):
    _fields_ = [("base", VP), ("row0", VP), ("row_slot", VP), ("n_rows", ctypes.c_int64), ("chunk_first", VP), ("chunk_slot", VP), ("n_chunks", ctypes.c_int32), ("pad0", ctypes.c_int32), ("part", VP), ("edge0", VP), ("relu_words", VP),
                ("tile_row0", VP), ("halo_off", VP), ("halo_ids", VP), ("lcol_off", VP), ("lcol", VP), ("ltcol_off", VP), ("ltcol", VP),
                ("n_tiles", ctypes.c_int32), ("halo_max", ctypes.c_int32), ("tile_edges_max", ctypes.c_int32), ("tile_tedges_max", ctypes.c_int32),
                ("tile_wc", VP), ("tile_first", VP), ("tile_rows", ctypes.c_int32), ("part_layers", ctypes.c_int32), ("tile_meta", VP), ("part_mean", VP)]


class NcPlanC(ctypes.Structure):
    _fields_ = [("base", VP), ("row0", VP), ("row_slot", VP), ("n_rows", ctypes.c_int64), ("tile_row0", VP), ("tile_first", VP),
                ("halo_off", VP), ("halo_ids", VP), ("lcol_off", VP), ("lcol", VP), ("ltcol_off", VP), ("ltcol", VP),
                ("n_tiles", ctypes.c_int32), ("halo_max", ctypes.c_int32), ("tile_edges_max", ctypes.c_int32), ("tile_tedges_max", ctypes.c_int32)]


class PackInputC(ctypes.Structure):
    _fields_ = [
        ("n_graphs", ctypes.c_int32), ("n_feat", ctypes.c_int32), ("n_edge_feat", ctypes.c_int32), ("require_clusters", ctypes.c_int32),
        ("node_off", VP), ("edge_off", VP), ("c1_off", VP), ("edge_index", VP), ("edge_attr", VP), ("cluster0", VP), ("cluster1", VP),
    ]  # fmt: skip


class PackOutputC(ctypes.Structure):
    _fields_ = [(n, VP) for n in (
        "k0_off", "p1_off", "k1_off", "rowptr", "col", "eperm", "t_rowptr", "t_col", "t_eid", "m0_ptr", "m0_idx", "cl0",
        "p1_rowptr", "p1_col", "p1t_rowptr", "p1t_col", "m1_ptr", "m1_idx", "cl1", "edge_attr", "p1_ea", "p1t_pid",
    )]  # fmt: skip


class MclGraphsC(ctypes.Structure):
    _fields_ = [(n, VP) for n in ("node_off", "rowptr", "edge_off", "col", "weight", "ws_off", "ws", "pat_off", "pattern", "iters")]


DR_DTYPE_F32 = 0
DR_DTYPE_BF16 = 1


class PassC(ctypes.Structure):
    _fields_ = [
        ("flags", ctypes.c_int32),
        ("out_dim", ctypes.c_int32),
        ("loss_kind", ctypes.c_int32),
        ("use_dropout", ctypes.c_int32),
        ("drop_scale", ctypes.c_float),
        ("drop_p", ctypes.c_float),
        ("drop_seed", ctypes.c_uint64),
        ("drop_offset", ctypes.c_uint64),
        ("loss_scale", ctypes.c_float),
        ("compute_dtype", ctypes.c_int32),
        ("mask", VP),
        ("class_w", VP),
        ("out", VP),
        ("dout", VP),
        ("loss_per_graph", VP),
        ("slab", VP),
        ("head", VP),
        ("stamps", VP),
        ("step_counter", VP),
        ("fault", VP),
        ("spin_limit", ctypes.c_int32),
        ("pad0", ctypes.c_int32),
        ("slot", VP),
    ]


class AdamC(ctypes.Structure):
    _fields_ = [
        ("lr", ctypes.c_float),
        ("beta1", ctypes.c_float),
        ("beta2", ctypes.c_float),
        ("eps", ctypes.c_float),
        ("weight_decay", ctypes.c_float),
        ("bias_c1", ctypes.c_float),
        ("bias_c2_sqrt", ctypes.c_float),
        ("enabled", ctypes.c_int32),
        ("step_counter", VP),
        ("grad_div", VP),
        ("fault", VP),
        ("mirror", VP),
        ("mirror_idx", VP),
        ("fault_clear", VP),
        ("ticket", VP),
    ]


class GradRecipeC(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("off1", ctypes.c_int32), ("off2", ctypes.c_int32), ("cols", ctypes.c_int32)]


class ParamTableC(ctypes.Structure):
    _fields_ = [
        ("param", VP * DR_MAX_PARAMS),
        ("grad", VP * DR_MAX_PARAMS),
        ("exp_avg", VP * DR_MAX_PARAMS),
        ("exp_avg_sq", VP * DR_MAX_PARAMS),
        ("numel", ctypes.c_int32 * DR_MAX_PARAMS),
        ("recipe", GradRecipeC * DR_MAX_PARAMS),
        ("n_params", ctypes.c_int32),
        ("slab_stride", ctypes.c_int32),
        ("head_stride", ctypes.c_int32),
        ("slab_rows", ctypes.c_int32),
    ]


# (name, restype, argtypes) for every entry of include/deeprank2_amd.h
SIGNATURES = [
    ("dr_ginet_graph_pass", ctypes.c_int, [ctypes.POINTER(GraphStoreC), VP, ctypes.c_int32, ctypes.POINTER(GinetWeightsC), ctypes.POINTER(PassC), ctypes.c_int32, VP]),
    ("dr_ginet_lds_bytes", ctypes.c_int64, [ctypes.c_int32] * 8),
    ("dr_ginet_acc_pass", ctypes.c_int, [ctypes.POINTER(GraphStoreC), VP, ctypes.c_int32, ctypes.POINTER(GinetWeightsC), ctypes.POINTER(PassC), ctypes.c_int32, ctypes.c_int32, VP, _c_i32, VP]),
    ("dr_ginet_acc_row_floats", ctypes.c_int32, [ctypes.c_int32] * 2),
    ("dr_ginet_acc_lds_bytes", ctypes.c_int64, [_c_i32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    ("dr_ginet_large_pass", ctypes.c_int, [ctypes.POINTER(GraphStoreC), VP, ctypes.c_int32, ctypes.POINTER(LargePlanC), ctypes.POINTER(GinetWeightsC), ctypes.POINTER(PassC), ctypes.c_int32, ctypes.c_int32, VP]),
    ("dr_ginet_large_conv_lds_bytes", ctypes.c_int64, [ctypes.c_int32] * 5),
    ("dr_ginet_nocluster_large_pass", ctypes.c_int, [ctypes.POINTER(GraphStoreC), VP, ctypes.c_int32, ctypes.POINTER(NcPlanC), ctypes.POINTER(GinetWeightsC), ctypes.POINTER(PassC), VP]),
    ("dr_nc_large_scratch_floats", ctypes.c_int64, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    ("dr_nc_large_lds_bytes", ctypes.c_int64, [ctypes.c_int32] * 5),
    ("dr_fout_large_pass", ctypes.c_int, [ctypes.POINTER(GraphStoreC), VP, ctypes.c_int32, ctypes.POINTER(LargePlanC), ctypes.POINTER(FoutWeightsC), ctypes.POINTER(PassC), ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, VP]),
    ("dr_sgat_large_pass", ctypes.c_int, [ctypes.POINTER(GraphStoreC), VP, ctypes.c_int32, ctypes.POINTER(LargePlanC), ctypes.POINTER(FoutWeightsC), ctypes.POINTER(PassC), ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, VP]),
    ("dr_fout_large_conv_lds_bytes", ctypes.c_int64, [ctypes.c_int32] * 6),
    ("dr_fout_tail_lds_bytes", ctypes.c_int64, [ctypes.c_int32] * 6),
    ("dr_ginet_large_conv_lds_bytes_bf16", ctypes.c_int64, [ctypes.c_int32] * 5),
    ("dr_ginet_tail_lds_bytes", ctypes.c_int64, [ctypes.c_int32] * 5),
    ("dr_vanilla_graph_pass", ctypes.c_int, [ctypes.POINTER(GraphStoreC), VP, ctypes.c_int32, ctypes.POINTER(VanillaWeightsC), ctypes.POINTER(PassC), ctypes.POINTER(VanillaScratchC), ctypes.c_int32, VP]),
    ("dr_vanilla_scratch_floats", ctypes.c_int64, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]),
    ("dr_vanilla_lds_bytes", ctypes.c_int64, [ctypes.c_int32] * 3),
    ("dr_vanilla_part_floats", ctypes.c_int64, [ctypes.c_int32] * 2),
    ("dr_vanilla_fused_pass", ctypes.c_int, [ctypes.POINTER(GraphStoreC), VP, ctypes.c_int32, ctypes.POINTER(VanillaWeightsC), ctypes.POINTER(PassC), VP, VP, ctypes.c_int32, VP, VP, ctypes.c_int32, VP]),
    ("dr_vanilla_wpack_floats", ctypes.c_int64, []),
    ("dr_vanilla_wpack", ctypes.c_int, [ctypes.POINTER(VanillaWeightsC), ctypes.c_int32, ctypes.c_int32, VP, VP]),
    ("dr_vanilla_fused_lds_bytes", ctypes.c_int64, [ctypes.c_int32] * 3),
    ("dr_vanilla_fused_scratch_floats", ctypes.c_int64, [ctypes.c_int32] * 3),
    ("dr_fout_graph_pass", ctypes.c_int, [ctypes.POINTER(GraphStoreC), VP, ctypes.c_int32, ctypes.POINTER(FoutWeightsC), ctypes.POINTER(PassC), ctypes.c_int32, VP]),
    ("dr_fout_lds_bytes", ctypes.c_int64, [ctypes.c_int32] * 8),
    ("dr_ginet_nocluster_graph_pass", ctypes.c_int, [ctypes.POINTER(GraphStoreC), VP, ctypes.c_int32, ctypes.POINTER(GinetWeightsC), ctypes.POINTER(PassC), ctypes.c_int32, VP]),
    ("dr_ginet_nocluster_lds_bytes", ctypes.c_int64, [ctypes.c_int32] * 4),
    ("dr_sgat_graph_pass", ctypes.c_int, [ctypes.POINTER(GraphStoreC), VP, ctypes.c_int32, ctypes.POINTER(FoutWeightsC), ctypes.POINTER(PassC), ctypes.c_int32, VP]),
    ("dr_sgat_lds_bytes", ctypes.c_int64, [ctypes.c_int32] * 8),
    ("dr_reduce_update", ctypes.c_int, [ctypes.POINTER(ParamTableC), VP, VP, ctypes.c_int32, ctypes.POINTER(AdamC), VP, ctypes.c_float, VP, VP]),
    ("dr_csr_from_coo", ctypes.c_int, [VP, VP, ctypes.c_int64, ctypes.c_int32, VP, VP, VP, VP, VP]),
    ("dr_spmm_csr", ctypes.c_int, [VP, VP, VP, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, VP, VP]),
    ("dr_spmm_csr_w", ctypes.c_int, [VP, VP, VP, VP, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, VP, VP]),
    ("dr_linear_xwT", ctypes.c_int, [VP, VP, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, VP, VP]),
    ("dr_linear_xw", ctypes.c_int, [VP, VP, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, VP, VP]),
    ("dr_linear_dw", ctypes.c_int, [VP, VP, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, VP, VP, ctypes.c_int32, VP]),
    ("dr_edge_mlp_scatter", ctypes.c_int, [VP, VP, ctypes.c_int32, VP, VP, VP, ctypes.c_int32, VP, ctypes.c_int32, VP, VP, VP]),
    ("dr_edge_mlp_scatter_bwd", ctypes.c_int, [VP, VP, VP, VP, VP, ctypes.c_int32, VP, VP, VP, ctypes.c_int32, VP, ctypes.c_int32, VP, VP, VP, VP, VP, VP]),
    ("dr_segment_max", ctypes.c_int, [VP, VP, VP, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, VP, VP, VP]),
    ("dr_segment_max_bwd", ctypes.c_int, [VP, VP, VP, VP, VP, VP, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, VP, VP]),
    ("dr_segment_mean", ctypes.c_int, [VP, VP, VP, ctypes.c_int32, ctypes.c_int32, VP, VP]),
    ("dr_pack_sizes", ctypes.c_int, [ctypes.POINTER(PackInputC), VP, VP, VP, ctypes.c_int32, ctypes.c_char_p, ctypes.c_int32]),
    ("dr_pack_fill", ctypes.c_int, [ctypes.POINTER(PackInputC), ctypes.POINTER(PackOutputC), VP, ctypes.c_int32]),
    ("dr_mcl_workspace_doubles", ctypes.c_int64, [ctypes.c_int32]),
    ("dr_mcl", ctypes.c_int, [ctypes.POINTER(MclGraphsC), ctypes.c_int32, ctypes.c_int32, ctypes.c_double, VP]),
    ("dr_mcl_assign", ctypes.c_int, [VP, VP, VP, ctypes.c_int32, VP, VP]),
    ("dr_dropout_mask", ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int32, ctypes.c_float, VP]),
    *[(f"dr_debug_carve_{k}", ctypes.c_int, [VP, ctypes.c_char_p, ctypes.c_int32]) for k in ("ginet", "ginet_conv", "ginet_conv_bf16", "ginet_tail", "fout", "fout_conv", "fout_tail", "nocluster", "vanilla_graph", "vanilla_tile", "vanilla_chunk_fwd", "vanilla_chunk_bwd")],
    ("dr_debug_xcd_tile", ctypes.c_int, [ctypes.c_int32, VP]),
    ("dr_version", ctypes.c_char_p, []),
    ("dr_device_arch", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int32]),
]

_LIB = None


def load():
    """Load the in-tree library (raises if it has not been built)."""
    global _LIB  # noqa: PLW0603
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        msg = f"{LIB_PATH} is missing: build it with `make -C deeprank-gnn-2_amd/csrc` (or __graft_entry__.build()). There is no CPU fallback."
        raise RuntimeError(msg)
    lib = ctypes.CDLL(LIB_PATH)
    variant = "DR_LIB_NAME" in os.environ  # an A/B build of an older HEAD may lack newer entries
    for name, res, args in SIGNATURES:
        try:
            fn = getattr(lib, name)
        except AttributeError:
            if variant:
                continue
            raise
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = f"{what} failed: {ERRORS.get(rc, f'hip error {rc}')}"
        raise RuntimeError(msg)


def ptr(t) -> int | None:
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_ptr(device) -> int:
    import torch  # noqa: PLC0415

    return torch.cuda.current_stream(device).cuda_stream


def require_device(*tensors) -> None:
    for t in tensors:
        if t is not None and not t.is_cuda:
            msg = "deeprank2_amd kernels run on the MI355X only: got a CPU tensor (no CPU fallback by design)"
            raise RuntimeError(msg)


def dropout_keep_host(seed: int, offset: int, n: int, p: float):
    """Host replica of the in-kernel dropout hash (DR_DROPOUT_HASH) -> numpy uint8 [n]."""
    import numpy as np  # noqa: PLC0415

    out = np.empty(n, dtype=np.uint8)
    check(load().dr_dropout_mask(seed, offset, n, p, out.ctypes.data), "dr_dropout_mask")
    return out
