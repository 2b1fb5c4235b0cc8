#!/usr/bin/env python3
"""Debug-build probe (option 99 of a temporary build): C3 forward / dgrad GEMM time with parts
skipped: output stores (256), A-row gathers pinned to row 0 (512), MFMAs (1024), weight-slice
reloads (2048), the tile commit (4096). The switches were a local patch of rel_gemm_bf3_kernel
(`a.relu` bits read in issue_rows / store_prev / the chain, set by a temporary option 99) that is
not part of the product build: mpgnn_set_option refuses 99 there. Results: DESIGN.md §4."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402
from mpgnn_amd import _lib, data  # noqa: E402
from mpgnn_amd.functional import rgcn_conv  # noqa: E402

g = data.fb15k237_graph(feat_dim=128, seed=0, recipe="survey")
dev = "cuda"
N, R = g.num_nodes, g.num_relations
plan = mpgnn_amd.GraphPlan(g.edge_index.to(dev), g.edge_type.to(dev), N)
x = g.x.to(dev).requires_grad_(True)
W = ((torch.rand(R, 128, 128) - 0.5) * 0.2).to(dev).requires_grad_(True)
root = ((torch.rand(128, 128) - 0.5) * 0.2).to(dev).requires_grad_(True)
bias = (torch.rand(128) - 0.5).to(dev).requires_grad_(True)
gout = torch.randn(N, 128, device=dev)
for rep in range(2):
    for dbg in (0, 256, 512, 768, 2048, 4096, 768 | 2048, 768 | 2048 | 4096):
        _lib.set_option(99, dbg)
        for _ in range(3):
            out = rgcn_conv(x, W, root, bias, plan, 1, num_relations=R)
            out.backward(gout)
        torch.cuda.synchronize()
        _lib.lib.mpgnn_timing_reset()
        _lib.lib.mpgnn_timing_enable(1)
        for _ in range(20):
            out = rgcn_conv(x, W, root, bias, plan, 1, num_relations=R)
            out.backward(gout)
        torch.cuda.synchronize()
        _lib.lib.mpgnn_timing_enable(0)
        res = {}
        for k in ("seg_fwd", "seg_dgrad", "row_fwd", "mean", "outer"):
            ms, n = _lib.kernel_timing(k)
            if n:
                res[k] = round(ms * 1e3 / n, 2)
        print(f"dbg={dbg}: {res}", flush=True)
_lib.set_option(99, 0)
