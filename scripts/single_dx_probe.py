#!/usr/bin/env python3
"""Mode-SINGLE backward at C3: per-relation grad_x cost (pieces launch + row launch) against
the relation's in-degree profile (rows of the transposed list longer than one 32-entry piece)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402
from mpgnn_amd import _lib, data  # noqa: E402
from mpgnn_amd.mp_rgcn_layer import CustomRGCNConv  # noqa: E402

dev = torch.device("cuda", 0)
g = data.fb15k237_graph(feat_dim=128, seed=0)
x, ei, et = g.x.to(dev), g.edge_index.to(dev), g.edge_type.to(dev)
rel_counts = torch.bincount(g.edge_type, minlength=g.num_relations)
rels = [int(v) for v in torch.argsort(rel_counts, descending=True, stable=True)[:3]]
out = {}
for r in rels:
    m = g.edge_type == r
    for side, col in (("node_1", 0), ("node_2", 1)):
        deg = torch.bincount(g.edge_index[col][m], minlength=g.num_nodes)
        long = deg[deg > 32]
        out.setdefault(r, {})[side] = {"edges": int(m.sum()), "rows": int((deg > 0).sum()), "max": int(deg.max()),
                                       "rows_gt32": int(long.numel()),
                                       "pieces": int(((long + 31) // 32).sum())}
    conv = CustomRGCNConv(128, 128, 1, flow="target_to_source").to(dev)
    xg = x.clone().requires_grad_(True)
    go = torch.randn(g.num_nodes, 128, device=dev)
    for _ in range(3):
        o = conv(0, r, xg, ei, et)
        o.backward(go)
    torch.cuda.synchronize()
    _lib.lib.mpgnn_timing_enable(1)
    _lib.lib.mpgnn_timing_reset()
    for _ in range(20):
        o = conv(0, r, xg, ei, et)
        o.backward(go)
    torch.cuda.synchronize()
    t = {k: _lib.kernel_timing(k) for k in _lib.KERNEL_KINDS}
    _lib.lib.mpgnn_timing_enable(0)
    out[r]["us_per_call"] = {k: round(ms * 1e3 / 20, 2) for k, (ms, n) in t.items() if n}
    out[r]["launches_per_call"] = {k: n / 20 for k, (ms, n) in t.items() if n}
print(json.dumps(out, indent=1))
