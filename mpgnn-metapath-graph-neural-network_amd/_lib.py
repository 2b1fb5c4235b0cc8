"""ctypes binding of libmpgnn_rgcn.so (the C ABI declared in include/mpgnn_rgcn.h).

The library is built in-tree by ``csrc/Makefile`` (``__graft_entry__.build()``). Importing
this module without the library raises ImportError: there is no CPU fallback anywhere on the
product path.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmpgnn_rgcn.so")

MPGNN_OK = 0
MPGNN_ERR_ARG = -1
MPGNN_ERR_INDEX = -2
MPGNN_ERR_HIP = -3
MPGNN_ERR_NOT_ON_DEVICE = -4
MPGNN_ERR_ALLOC = -5
MPGNN_ERR_UNSUPPORTED = -6

MODE_SINGLE = 0
MODE_ALL = 1

SHARD_SIDES = {"gathered": 0, "rows": 1}  # mpgnn_shard_side

TABLES = {
    "rel_values": (0, "int64"), "rel_seg_ptr": (1, "int32"), "rel_edge_ptr": (2, "int32"),
    "e_col": (3, "int32"), "e_id": (4, "int32"), "s_ptr": (5, "int32"), "s_row": (6, "int32"),
    "s_rel": (7, "int32"), "s_cnt": (8, "int32"), "s_pos": (9, "int32"), "rw_ptr": (10, "int32"),
    "rw_seg": (11, "int32"), "t_ptr": (12, "int32"), "t_seg": (13, "int32"),
    "ta_col": (14, "int32"), "ta_seg": (15, "int32"), "rel_invalid": (16, "uint8"),
}
# flat chunked lists (fast-path row sums): <list>_f_<table>, ids 17..34
for _i, _l in enumerate(("seg", "t", "rw")):
    for _j, _n in enumerate(("chunk_ptr", "chunk_info", "row_of", "split_row", "split_ptr", "split_slot")):
        TABLES[f"{_l}_f_{_n}"] = (17 + 6 * _i + _j, "int32")
# multi-edge segments (the compact means the layers materialise), ids 35..45
TABLES.update({"s_src": (35, "int32"), "m_ptr": (36, "int32"), "em_col": (37, "int32"), "m_cnt": (38, "int32"),
               "rel_m_ptr": (39, "int32")})
for _j, _n in enumerate(("chunk_ptr", "chunk_info", "row_of", "split_row", "split_ptr", "split_slot")):
    TABLES[f"segm_f_{_n}"] = (40 + _j, "int32")
for _i, _l in enumerate(("seg", "t", "rw", "segm")):  # workgroup groups of the flat lists, ids 46..53
    TABLES[f"{_l}_f_group_ptr"] = (46 + 2 * _i, "int32")
    TABLES[f"{_l}_f_group_long"] = (47 + 2 * _i, "int32")


class PlanInfo(ctypes.Structure):
    _fields_ = [
        ("num_nodes", ctypes.c_int64), ("num_edges_in", ctypes.c_int64),
        ("num_edges", ctypes.c_int64), ("num_segments", ctypes.c_int64),
        ("num_relations", ctypes.c_int64), ("num_tiles", ctypes.c_int64),
        ("num_chunks", ctypes.c_int64), ("shard_lo", ctypes.c_int64),
        ("shard_hi", ctypes.c_int64), ("device", ctypes.c_int32), ("reserved", ctypes.c_int32),
    ]


class AdamTensor(ctypes.Structure):
    """mpgnn_adam_tensor of include/mpgnn_rgcn.h."""
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("step", ctypes.c_void_p), ("numel", ctypes.c_int64)]


# (name, restype, argtypes) — exactly the symbols of include/mpgnn_rgcn.h
_P = ctypes.c_void_p
_I32, _I64 = ctypes.c_int32, ctypes.c_int64
_PI64 = ctypes.POINTER(ctypes.c_int64)
SIGNATURES = [
    ("mpgnn_plan_create", _I32, [_P, _P, _I64, _I64, _I64, _I64, ctypes.POINTER(_P)]),
    ("mpgnn_plan_create_sharded", _I32, [_P, _P, _I64, _I64, _I64, _I64, _I32, ctypes.POINTER(_P)]),
    ("mpgnn_plan_create_device", _I32, [_P, _P, _I64, _I64, _I64, _I64, _I32, _I32, _P, ctypes.POINTER(_P)]),
    ("mpgnn_plan_destroy", _I32, [_P]),
    ("mpgnn_plan_digest", _I32, [_P, ctypes.POINTER(ctypes.c_uint64)]),
    ("mpgnn_plan_get_info", _I32, [_P, ctypes.POINTER(PlanInfo)]),
    ("mpgnn_plan_table_size", _I32, [_P, _I32, _PI64, ctypes.POINTER(_I32)]),
    ("mpgnn_plan_export", _I32, [_P, _I32, _P, _I64]),
    ("mpgnn_plan_upload", _I32, [_P, _I32]),
    ("mpgnn_plan_select", _I32, [_P, _I32, _I64, _I32, _PI64, _PI64]),
    ("mpgnn_last_error", ctypes.c_char_p, []),
    ("mpgnn_status_string", ctypes.c_char_p, [_I32]),
    ("mpgnn_abi_version", _I32, []),
    ("mpgnn_rel_mean_fwd", _I32, [_P, _I32, _I64, _I32, _P, _I32, _P, _P]),
    ("mpgnn_rel_mean_bwd_workspace_bytes", _I32, [_P, _I32, _I64, _I32, _I32, _PI64]),
    ("mpgnn_rel_mean_bwd", _I32, [_P, _I32, _I64, _I32, _P, _I32, _P, _P, _P]),
    ("mpgnn_rgcn_workspace_bytes", _I32, [_P, _I32, _I64, _I32, _I32, _I32, _I64, _I64, _PI64]),
    ("mpgnn_rgcn_hsave_rows", _I32, [_P, _I32, _I64, _I32, _PI64]),
    ("mpgnn_rgcn_fwd_workspace_bytes", _I32, [_P, _I32, _I64, _I32, _I32, _I32, _I64, _I64, _PI64]),
    ("mpgnn_rgcn_fwd", _I32, [_P, _I32, _I64, _I32, _P, _I32, _P, _P, _P, _I32, _I64, _I64,
                              _P, _P, _P, _P]),
    ("mpgnn_rgcn_fwd_act", _I32, [_P, _I32, _I64, _I32, _P, _I32, _P, _P, _P, _I32, _P, _P, _P, _I32, _P]),
    ("mpgnn_rgcn_bwd", _I32, [_P, _I32, _I64, _I32, _P, _I32, _P, _P, _I32, _P, _P, _I64, _I64,
                              _P, _P, _P, _P, _P, _P]),
    ("mpgnn_rgcn_bwd_accumulate", _I32, [_P, _I32, _I64, _I32, _P, _I32, _P, _P, _I32, _P, _P, _I64, _I64,
                                         _P, _P, _P, _P, _P, _P]),
    ("mpgnn_rgcn_bwd_relu_in", _I32, [_P, _I32, _I64, _I32, _P, _I32, _P, _P, _I32, _P, _P, _I64, _I64,
                                      _P, _P, _P, _P, _P, _P, _I32]),
    ("mpgnn_relu_bwd", _I32, [_P, _P, _I64, _P, _P]),
    ("mpgnn_dropout_relu_bwd", _I32, [_P, _P, _P, ctypes.c_float, _I64, _P, _P]),
    ("mpgnn_linear_wgrad_workspace_bytes", _I32, [_I64, _I32, _I32, _PI64]),
    ("mpgnn_linear_wgrad", _I32, [_P, _P, _I64, _I32, _I32, _P, _P, _P, _P]),
    ("mpgnn_linear_fwd", _I32, [_P, _I64, _I32, _P, _I32, _P, _I32, _P, _P]),
    ("mpgnn_linear_dgrad", _I32, [_P, _I64, _I32, _P, _I32, _P, _P]),
    ("mpgnn_linear_dgrad_relu_in", _I32, [_P, _I64, _I32, _P, _I32, _P, _P, _P]),
    ("mpgnn_linear_logsoftmax_bwd_workspace_bytes", _I32, [_I64, _I32, _I32, _PI64]),
    ("mpgnn_linear_logsoftmax_bwd", _I32, [_P, _P, _P, _I64, _I32, _I32, _P, _P, _P, _P, _P, _P, _P]),
    ("mpgnn_adam_step", _I32, [ctypes.POINTER(AdamTensor), _I32, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                ctypes.c_double, ctypes.c_double, _P, _P]),
    ("mpgnn_score_argmax", _I32, [_P, _I64, _P, _P, _P, _I64, _P, _P, _P, _P]),
    ("mpgnn_score_argmax_bwd", _I32, [_P, _I64, _P, _P, _P, _P, _P, _P, _P]),
    ("mpgnn_score_argmax_multi", _I32, [_P, _I64, _P, _P, _P, _P, _I64, _P, _P, _P, _P, _P, _P, _P, _P]),
    ("mpgnn_score_loss_multi", _I32, [_P, _P, _I64, _P, _P]),
    ("mpgnn_score_argmax_multi_bwd", _I32, [_P, _P, _P, _P, _P, _P, _I64, _I64, _P, _P]),
    ("mpgnn_confusion_counts", _I32, [_P, _I64, _I32, _I32, _P, _P, _P, _P, _P]),
    ("mpgnn_nll_rows_fwd", _I32, [_P, _I64, _I32, _P, _P, _I64, _I64, _P, _P, _P]),
    ("mpgnn_nll_rows_bwd", _I32, [_P, _P, _I64, _I32, _P, _P, _I64, _I64, _P, _P]),
    ("mpgnn_nll_rows_bwd_dense", _I32, [_P, _P, _I64, _I32, _P, _P, _P, _I64, _P, _P, _P]),
    ("mpgnn_nll_rows_fwd_weighted", _I32, [_P, _I64, _I32, _P, _P, _I64, _I64, _P, _P, _P, _P]),
    ("mpgnn_nll_rows_bwd_weighted", _I32, [_P, _P, _I64, _I32, _P, _P, _I64, _I64, _P, _P, _P]),
    ("mpgnn_score_bag_argmax", _I32, [_P, _P, _I32, _P, _P, _P, _P, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    ("mpgnn_score_bag_argmax_bwd", _I32, [_P, _I64, _P, _P, _P, _P, _P, _P, _I32, _I64, _P, _P, _P, _P, _P, _P,
                                          _P]),
    ("mpgnn_set_option", _I32, [_I32, _I64]),
    ("mpgnn_plan_set_option", _I32, [_P, _I32, _I64]),
    ("mpgnn_plan_get_option", _I32, [_P, _I32, _PI64]),
    ("mpgnn_get_option", _I32, [_I32, _PI64]),
    ("mpgnn_timing_enable", _I32, [_I32]),
    ("mpgnn_debug_occupancy", _I32, [_I32, ctypes.POINTER(_I32), ctypes.POINTER(_I32), ctypes.POINTER(_I32)]),
    ("mpgnn_timing_reset", _I32, []),
    ("mpgnn_timing_query", _I32, [_I32, ctypes.POINTER(ctypes.c_double), _PI64]),
    ("mpgnn_links_count", _I32, [ctypes.c_char_p, _PI64]),
    ("mpgnn_links_parse", _I32, [ctypes.c_char_p, _P, _P, _I64]),
    ("mpgnn_tsv_shape", _I32, [ctypes.c_char_p, _PI64, _PI64]),
    ("mpgnn_tsv_parse_f64", _I32, [ctypes.c_char_p, _P, _I64, _I64]),
]

KERNEL_KINDS = {"seg_fwd": 0, "row_fwd": 1, "seg_dgrad": 2, "row_dx": 3, "outer": 4, "reduce": 5, "mean": 6,
                "piece": 7, "final": 8}
OPT_EXACT_ORDER = 0
OPT_ADAM_CONTRACT = 40
ACT_NONE, ACT_RELU, ACT_LOG_SOFTMAX = 0, 1, 2


def _missing(name):
    def fn(*_a, **_k):
        raise RuntimeError(f"{name} is not in {LIB_PATH} (host-only sanitizer library)")
    return fn


def _load():
    global LIB_PATH
    override = os.environ.get("MPGNN_LIB_PATH")
    if override:
        # tests/test_host_sanitizers.py: the ASan/UBSan host-only build of plan.cpp + io.cpp
        # (csrc/Makefile `asan`); symbols it does not export raise when called
        LIB_PATH = os.path.abspath(override)
        lib = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            try:
                fn = getattr(lib, name)
            except AttributeError:
                setattr(lib, name, _missing(name))
                continue
            fn.restype = res
            fn.argtypes = args
        return lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make -C csrc` or __graft_entry__.build(). "
            "mpgnn_amd has no CPU fallback.")
    # a library shipped next to newer sources is stale: refuse it rather than run old kernels
    # (MPGNN_ALLOW_STALE_LIB=1 skips the check; the sources are always present in-tree)
    from . import _srchash
    if os.environ.get("MPGNN_ALLOW_STALE_LIB") != "1" and _srchash.sources_present():
        stamp = open(_srchash.STAMP).read().strip() if os.path.exists(_srchash.STAMP) else None
        if stamp != _srchash.source_hash():
            raise ImportError(
                f"{LIB_PATH} was not built from the current sources (stamp {_srchash.STAMP} "
                f"{'missing' if stamp is None else 'differs'}): rebuild with __graft_entry__.build().")
    lib = ctypes.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def _env_options() -> None:
    """MPGNN_OPTS="id=value,..." (A/B scripts): options set once when the library is loaded."""
    spec = os.environ.get("MPGNN_OPTS", "").strip()
    for item in filter(None, (t.strip() for t in spec.split(","))):
        k, _, v = item.partition("=")
        st = lib.mpgnn_set_option(int(k), int(v))
        if st != MPGNN_OK:
            raise ValueError(f"MPGNN_OPTS {item!r}: {lib.mpgnn_last_error().decode(errors='replace')}")


_env_options()


def kernel_timing(kind: str) -> tuple[float, int]:
    """(total ms, launches) of one kernel kind since mpgnn_timing_reset (syncs its events)."""
    ms, n = ctypes.c_double(), ctypes.c_int64()
    check(lib.mpgnn_timing_query(KERNEL_KINDS[kind], ctypes.byref(ms), ctypes.byref(n)), "mpgnn_timing_query")
    return float(ms.value), int(n.value)


def get_option(option: int) -> int:
    """Current value of an ``enum mpgnn_option`` switch."""
    v = ctypes.c_int64()
    check(lib.mpgnn_get_option(int(option), ctypes.byref(v)), "mpgnn_get_option")
    return int(v.value)


def set_option(option: int, value: int) -> None:
    """The process default of an option: kernel switches apply to plans created afterwards
    (``GraphPlan.set_option`` changes one plan); see include/mpgnn_rgcn.h."""
    check(lib.mpgnn_set_option(int(option), int(value)), "mpgnn_set_option")


def set_exact_order(on: bool) -> None:
    """Process default of the reference-sequential summation order: applies to plans created
    afterwards (``GraphPlan.set_exact_order`` switches one existing plan; see include/mpgnn_rgcn.h)."""
    check(lib.mpgnn_set_option(OPT_EXACT_ORDER, 1 if on else 0), "mpgnn_set_option")


def check(status: int, what: str = "") -> None:
    """Map a C status to the exception the reference raises for the same condition."""
    if status == MPGNN_OK:
        return
    msg = lib.mpgnn_last_error().decode(errors="replace")
    text = f"{what}: {msg}" if what else msg
    if status == MPGNN_ERR_INDEX:
        raise IndexError(text)  # reference: x.index_select / scatter_add_ with a bad index
    if status == MPGNN_ERR_ARG:
        raise ValueError(text)
    if status == MPGNN_ERR_UNSUPPORTED:
        raise NotImplementedError(text)
    raise RuntimeError(text)
