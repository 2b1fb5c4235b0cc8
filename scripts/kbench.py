#!/usr/bin/env python3
"""Kernel-level timing of one RGCN layer (mode ALL) on a named workload, with ablations.

  python scripts/kbench.py [--config fb15k237] [--feat 128] [--iters 30]

Reports per kernel [µs per launch, µs per call, launches per call] (HIP events on the launch stream, via the C ABI timing
hook) for: the default path, MPGNN_OPT_ABLATE=1 (no gather), =2 (no MFMA), exact order, and
the backward kernels. Ablated runs produce wrong numbers by design (profiling only).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402
from mpgnn_amd import _lib, data  # noqa: E402


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    _lib.lib.mpgnn_timing_reset()
    _lib.lib.mpgnn_timing_enable(1)
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    _lib.lib.mpgnn_timing_enable(0)
    out = {}
    for k in _lib.KERNEL_KINDS:
        ms, n = _lib.kernel_timing(k)
        if n:  # [µs per launch, µs per call, launches per call]
            out[k] = [round(ms / n * 1e3, 2), round(ms / iters * 1e3, 2), round(n / iters, 2)]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="fb15k237")
    ap.add_argument("--feat", type=int, default=128)
    ap.add_argument("--fout", type=int, default=None)
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    g = data.config_graph(args.config)
    F = args.feat
    fout = args.fout or F
    x = torch.rand(g.num_nodes, F, device="cuda")
    ei, et = g.edge_index.cuda(), g.edge_type.cuda()
    torch.manual_seed(0)
    conv = mpgnn_amd.RGCNConv(F, fout, g.num_relations, flow="target_to_source").cuda()
    res = {"config": args.config, "feat": F, "fout": fout}
    with torch.no_grad():
        res["fwd"] = timed(lambda: conv(x, ei, et), args.iters)
        _lib.lib.mpgnn_set_option(1, 1)
        res["fwd_no_gather"] = timed(lambda: conv(x, ei, et), args.iters)
        _lib.lib.mpgnn_set_option(1, 2)
        res["fwd_no_mfma"] = timed(lambda: conv(x, ei, et), args.iters)
        _lib.lib.mpgnn_set_option(1, 4)
        res["fwd_no_epilogue"] = timed(lambda: conv(x, ei, et), args.iters)
        _lib.lib.mpgnn_set_option(1, 8)
        res["fwd_no_mfma_loop"] = timed(lambda: conv(x, ei, et), args.iters)
        _lib.lib.mpgnn_set_option(1, 1 | 8)
        res["fwd_epilogue_only"] = timed(lambda: conv(x, ei, et), args.iters)
        _lib.lib.mpgnn_set_option(1, 1 | 4)
        res["fwd_mfma_only"] = timed(lambda: conv(x, ei, et), args.iters)
        _lib.lib.mpgnn_set_option(1, 0)
        _lib.set_exact_order(True)
        res["fwd_exact"] = timed(lambda: conv(x, ei, et), args.iters)
        _lib.set_exact_order(False)
    xg = x.clone().requires_grad_(True)

    def fb():
        o = conv(xg, ei, et)
        o.backward(torch.ones_like(o))

    res["fwd_bwd"] = timed(fb, args.iters)
    import ctypes
    occ, occ_t, grid_t = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    _lib.lib.mpgnn_debug_occupancy(F, ctypes.byref(occ), ctypes.byref(occ_t), ctypes.byref(grid_t))
    res["seg_tile_blocks_per_cu"] = occ.value
    res["tile_gemm_blocks_per_cu"] = occ_t.value
    res["tile_gemm_grid"] = grid_t.value
    plan = mpgnn_amd.get_plan(ei, et, g.num_nodes)
    res["plan"] = {"S": plan.num_segments, "E": plan.num_edges, "tiles": plan.num_tiles}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
