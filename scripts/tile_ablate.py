#!/usr/bin/env python3
"""Time the persistent tile GEMM (forward, mode ALL, fb15k237 C3, F=128) under compile-time
ablations (MPGNN_OPT_ABLATE bits >> 4: 1 no MFMA, 2 no B loads, 4 no LDS A reads, 8 no stores).
Ablated runs compute wrong numbers by design (profiling only)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402
from mpgnn_amd import _lib, data  # noqa: E402

g = data.config_graph("fb15k237")
x = torch.rand(g.num_nodes, 128, device="cuda")
ei, et = g.edge_index.cuda(), g.edge_type.cuda()
conv = mpgnn_amd.RGCNConv(128, 128, g.num_relations, flow="target_to_source").cuda()
res = {}
with torch.no_grad():
    for rnd in range(3):
        for abl in [0, 1, 2, 3, 4, 6, 8, 9, 14]:
            _lib.lib.mpgnn_set_option(1, abl << 4)
            for _ in range(3):
                conv(x, ei, et)
            torch.cuda.synchronize()
            _lib.lib.mpgnn_timing_reset()
            _lib.lib.mpgnn_timing_enable(1)
            for _ in range(20):
                conv(x, ei, et)
            torch.cuda.synchronize()
            _lib.lib.mpgnn_timing_enable(0)
            ms, n = _lib.kernel_timing("seg_fwd")
            res.setdefault(abl, []).append(round(ms / n * 1e3, 2))
_lib.lib.mpgnn_set_option(1, 0)
print(json.dumps({"seg_fwd_us_by_ablation": res}))
