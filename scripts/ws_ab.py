#!/usr/bin/env python3
"""A/B of the tile GEMM variants (MPGNN_OPT_TILE_WS: 0 two-workgroup, 1 specialised + prio,
2 specialised without prio), interleaved rounds in one process; forward layer, FB15K, F=128."""
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
_lib.lib.mpgnn_set_option(3, 1)
with torch.no_grad():
    for rnd in range(4):
        for v in (0, 1, 2, 11, 12, 14, 17):  # 1x: ws kernel with ablation bits x (1 no stores, 2 no A loads, 4 const B)
            _lib.lib.mpgnn_set_option(4, v if v < 10 else 1)
            _lib.lib.mpgnn_set_option(1, (v - 10) << 8 if v >= 10 else 0)
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
            res.setdefault(v, []).append(round(ms / n * 1e3, 2))
_lib.lib.mpgnn_set_option(4, 0)
_lib.lib.mpgnn_set_option(1, 0)
_lib.lib.mpgnn_set_option(3, -1)
print(json.dumps(res))
