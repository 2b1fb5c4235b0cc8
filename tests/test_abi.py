"""CPU: the C-ABI library loads and exports every symbol include/mpgnn_rgcn.h declares;
host-only entry points behave; device entry points refuse a plan that is not on a device
(no compute without a GPU)."""
import ctypes
import os
import re

import pytest
import torch

from tests.conftest import ROOT

HEADER = os.path.join(ROOT, "include", "mpgnn_rgcn.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mpgnn_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    syms = declared_symbols()
    for s in ("mpgnn_plan_create", "mpgnn_plan_destroy", "mpgnn_plan_upload", "mpgnn_rgcn_fwd",
              "mpgnn_rgcn_bwd", "mpgnn_rel_mean_fwd", "mpgnn_rgcn_workspace_bytes"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from mpgnn_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    bound = {name for name, _, _ in _lib.SIGNATURES}
    assert bound == set(declared_symbols())


def test_version_and_status_strings():
    from mpgnn_amd._lib import lib
    assert lib.mpgnn_abi_version() == 1
    assert lib.mpgnn_status_string(0) == b"ok"
    assert lib.mpgnn_status_string(-2) == b"index out of range"


def test_kernels_refuse_plan_not_on_device():
    from mpgnn_amd import _lib
    from mpgnn_amd._lib import lib
    import mpgnn_amd
    g = mpgnn_amd.data.config_graph("C1")
    p = mpgnn_amd.GraphPlan(g.edge_index, g.edge_type, g.num_nodes)
    st = lib.mpgnn_rgcn_fwd(p.handle, 1, -1, 3, None, 128, None, None, None, 64, 0, g.num_nodes,
                            None, None, None, None)
    assert st == _lib.MPGNN_ERR_NOT_ON_DEVICE
    assert b"upload" in lib.mpgnn_last_error()
    st = lib.mpgnn_rel_mean_fwd(p.handle, 1, -1, 3, None, 128, None, None)
    assert st == _lib.MPGNN_ERR_NOT_ON_DEVICE


def test_bad_arguments():
    from mpgnn_amd import _lib
    from mpgnn_amd._lib import lib
    h = ctypes.c_void_p()
    assert lib.mpgnn_plan_create(None, None, 5, 10, 0, 10, ctypes.byref(h)) == _lib.MPGNN_ERR_ARG
    assert lib.mpgnn_plan_create(None, None, -1, 10, 0, 10, ctypes.byref(h)) == _lib.MPGNN_ERR_ARG
    assert lib.mpgnn_plan_destroy(None) == 0
    import mpgnn_amd
    g = mpgnn_amd.data.config_graph("C1")
    p = mpgnn_amd.GraphPlan(g.edge_index, g.edge_type, g.num_nodes)
    with pytest.raises(ValueError):
        p.select(7, 0, 0)          # unknown mode


def test_withdrawn_option_is_refused():
    """The round-1 profiling switches and measured-slower variants (ids 1, 2, 4, 6-10, 12-18,
    21-23) were withdrawn: refused with a message; the retained options still work."""
    from mpgnn_amd import _lib
    lib = _lib.lib
    for opt in (1, 2, 4, 6, 7, 8, 9, 10, 12, 13, 14, 15, 16, 17, 18, 21, 22, 23):
        assert lib.mpgnn_set_option(opt, 0) == _lib.MPGNN_ERR_ARG
        assert b"withdrawn" in lib.mpgnn_last_error()
    shipped = _lib.get_option(20)
    assert shipped == 256  # the header's documented default chunk length
    assert lib.mpgnn_set_option(20, 192) == 0 and _lib.get_option(20) == 192
    assert lib.mpgnn_set_option(20, shipped) == 0
    assert lib.mpgnn_set_option(11, 0) == 0
    with pytest.raises(ValueError):
        _lib.get_option(1)


def test_round4_switches_default_on_and_round_trip():
    """The round-4 / round-5 A/B switches (header enum mpgnn_option): the shipped values are the measured
    winners — hub rows finished in the gather launch (27), the 16-B-gather weight gradient (28),
    one workgroup per gather-list group (26 = 0), GEMM item ranges balanced with a weight switch
    priced at 1.5 items (29 = 150: re-swept in round 6 with the prologue records; 250 before), the
    interleaved GEMM item skeleton (30) and per-CU item ranges (31)
    — and each round-trips through set / get."""
    from mpgnn_amd import _lib
    lib = _lib.lib
    shipped = {26: 0, 27: 1, 28: 1, 29: 150, 30: 1, 31: 1, 32: 0, 33: 1, 34: 1}
    for opt, v in shipped.items():
        assert _lib.get_option(opt) == v, (opt, _lib.get_option(opt))
    try:
        for opt, v in ((26, 2), (27, 0), (28, 0), (29, 0), (30, 0), (31, 0), (32, 1), (33, 0), (34, 0)):
            assert lib.mpgnn_set_option(opt, v) == 0 and _lib.get_option(opt) == v
        assert lib.mpgnn_set_option(26, 65) == _lib.MPGNN_ERR_ARG  # 0..64 workgroups per CU
    finally:
        for opt, v in shipped.items():
            lib.mpgnn_set_option(opt, v)


def test_kernel_switches_are_per_plan():
    """VERDICT r4 item 5 / SURVEY §8b ("no global mutable state"): the kernel switches live in
    each plan. A plan copies the process defaults when it is created; mpgnn_plan_set_option
    changes that plan only; a later default change reaches plans created after it, not existing
    ones; the build-time and profiling options are refused on a plan."""
    import mpgnn_amd
    from mpgnn_amd import _lib
    lib = _lib.lib
    ei = torch.tensor([[0, 1, 2, 2], [1, 2, 0, 1]])
    et = torch.tensor([0, 1, 0, 1])
    a = mpgnn_amd.GraphPlan(ei, et, 3, build="host")
    b = mpgnn_amd.GraphPlan(ei, et, 3, build="host")
    assert a.get_option(29) == b.get_option(29) == _lib.get_option(29)
    a.set_option(29, 17)
    a.set_exact_order(True)
    assert a.get_option(29) == 17 and a.get_option(0) == 1
    assert b.get_option(29) == _lib.get_option(29) and b.get_option(0) == 0
    shipped = _lib.get_option(30)
    try:
        _lib.set_option(30, 0)
        c = mpgnn_amd.GraphPlan(ei, et, 3, build="host")
        assert c.get_option(30) == 0 and a.get_option(30) == shipped and b.get_option(30) == shipped
    finally:
        _lib.set_option(30, shipped)
    for opt in (3, 11, 20):  # timing mask, plan threads, chunk rows: process-wide
        assert lib.mpgnn_plan_set_option(a.handle, opt, 1) == _lib.MPGNN_ERR_ARG
        with pytest.raises(ValueError):
            a.get_option(opt)
    with pytest.raises(ValueError):
        a.set_option(29, -1)


def test_workspace_bytes_is_host_computable():
    import mpgnn_amd
    g = mpgnn_amd.data.config_graph("C1")
    p = mpgnn_amd.GraphPlan(g.edge_index, g.edge_type, g.num_nodes)
    b_all = p.workspace_bytes(mpgnn_amd.MODE_ALL, -1, 3, 128, 64, 0, g.num_nodes)
    assert b_all >= p.num_segments * 64 * 4
    b_one = p.workspace_bytes(mpgnn_amd.MODE_SINGLE, 1, 0, 128, 64, 0, g.num_nodes)
    assert 0 < b_one <= b_all


def test_product_path_fails_loudly_on_cpu_tensors():
    import mpgnn_amd
    g = mpgnn_amd.data.config_graph("C1")
    conv = mpgnn_amd.RGCNConv(128, 64, 3, flow="target_to_source")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        conv(g.x, g.edge_index, g.edge_type)
    c2 = mpgnn_amd.CustomRGCNConv(128, 64, 1, flow="target_to_source")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        c2(0, 1, g.x, g.edge_index, g.edge_type)


def test_round6_entry_points_check_arguments_before_launching():
    """The round-6 entry points refuse bad arguments and unsupported shapes before any launch
    (host-side checks only: callable without a GPU)."""
    from mpgnn_amd import _lib
    from mpgnn_amd._lib import lib
    # mpgnn_adam_step: at most 24 tensors, 16-byte aligned pointers, n >= 0, NULL arrays refused
    arr = (_lib.AdamTensor * 25)()
    assert lib.mpgnn_adam_step(arr, 25, 0.01, 0.9, 0.999, 5e-4, 1e-8, ctypes.c_void_p(64), None) == \
        _lib.MPGNN_ERR_UNSUPPORTED
    assert lib.mpgnn_adam_step(arr, -1, 0.01, 0.9, 0.999, 5e-4, 1e-8, ctypes.c_void_p(64), None) == _lib.MPGNN_ERR_ARG
    assert lib.mpgnn_adam_step(None, 1, 0.01, 0.9, 0.999, 5e-4, 1e-8, ctypes.c_void_p(64), None) == _lib.MPGNN_ERR_ARG
    assert lib.mpgnn_adam_step(arr, 0, 0.01, 0.9, 0.999, 5e-4, 1e-8, None, None) == _lib.MPGNN_OK
    one = (_lib.AdamTensor * 1)()
    one[0].param, one[0].grad, one[0].exp_avg, one[0].exp_avg_sq, one[0].step = 4096 + 4, 4096, 4096, 4096, 4096
    one[0].numel = 8
    assert lib.mpgnn_adam_step(one, 1, 0.01, 0.9, 0.999, 5e-4, 1e-8, ctypes.c_void_p(64), None) == \
        _lib.MPGNN_ERR_UNSUPPORTED  # a misaligned parameter: nothing launched
    # the fused log-softmax head: O <= 8, F <= 256, F % 4 == 0
    nb = ctypes.c_int64()
    assert lib.mpgnn_linear_logsoftmax_bwd_workspace_bytes(100, 128, 9, ctypes.byref(nb)) == _lib.MPGNN_ERR_UNSUPPORTED
    assert lib.mpgnn_linear_logsoftmax_bwd_workspace_bytes(100, 260, 2, ctypes.byref(nb)) == _lib.MPGNN_ERR_UNSUPPORTED
    assert lib.mpgnn_linear_logsoftmax_bwd_workspace_bytes(100, 126, 2, ctypes.byref(nb)) == _lib.MPGNN_ERR_UNSUPPORTED
    assert lib.mpgnn_linear_logsoftmax_bwd_workspace_bytes(100, 128, 2, ctypes.byref(nb)) == _lib.MPGNN_OK
    assert nb.value == 4 * 2 * 129 * 4  # 4 row slices of 32 rows, [O][F + 1] floats each
    # empty inputs are no-ops; negative sizes refused
    assert lib.mpgnn_dropout_relu_bwd(None, None, None, ctypes.c_float(2.5), 0, None, None) == _lib.MPGNN_OK
    assert lib.mpgnn_dropout_relu_bwd(None, None, None, ctypes.c_float(2.5), -1, None, None) == _lib.MPGNN_ERR_ARG
    assert lib.mpgnn_nll_rows_bwd_dense(None, None, 0, 2, None, None, None, -100, None, None, None) == _lib.MPGNN_OK
    assert lib.mpgnn_nll_rows_fwd_weighted(None, 10, 2, None, None, -1, -100, None, None, None, None) == \
        _lib.MPGNN_ERR_ARG
    # the process-wide contraction switch round-trips and refuses other values
    v = ctypes.c_int64()
    assert lib.mpgnn_get_option(_lib.OPT_ADAM_CONTRACT, ctypes.byref(v)) == _lib.MPGNN_OK and v.value == 1
    assert lib.mpgnn_set_option(_lib.OPT_ADAM_CONTRACT, 2) == _lib.MPGNN_ERR_ARG
