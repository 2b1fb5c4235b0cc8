#!/usr/bin/env python3
"""Per-workgroup timeline of fused_mean_gemm_kernel (debug stamps, MPGNN_OPT_STAMPS), one FB15K
layer forward: range search, prologue, per item the gather wave's index load / gather / fix-up
and the matrix wave's MFMA + barrier (shader clocks; realtime span in ns)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402
from mpgnn_amd import _lib, data  # noqa: E402

g = data.config_graph("fb15k237")
x = torch.rand(g.num_nodes, 128, device="cuda")
ei, et = g.edge_index.cuda(), g.edge_type.cuda()
conv = mpgnn_amd.RGCNConv(128, 128, g.num_relations, flow="target_to_source").cuda()
with torch.no_grad():
    for _ in range(5):
        conv(x, ei, et)
torch.cuda.synchronize()
buf = torch.zeros(256 * 64, dtype=torch.int64, device="cuda")
_lib.lib.mpgnn_set_option(2, buf.data_ptr())
with torch.no_grad():
    conv(x, ei, et)
torch.cuda.synchronize()
_lib.lib.mpgnn_set_option(2, 0)
st = buf.cpu().numpy().reshape(256, 64).astype(np.float64)
res = {}
span_ns = (st[:, 63] - st[:, 62]) * 10.0
rt0 = st[:, 62].min()
res["rt_start_ns_p90"] = float(np.percentile((st[:, 62] - rt0) * 10, 90))
res["rt_end_ns"] = {"p50": float(np.median((st[:, 63] - rt0) * 10)), "max": float(((st[:, 63] - rt0) * 10).max())}
res["span_ns"] = {"p50": float(np.median(span_ns)), "max": float(span_ns.max())}
clk = (st[:, 2] - st[:, 0])
res["find_clk_p50"] = float(np.median(st[:, 1] - st[:, 0]))
res["prologue_clk_p50"] = float(np.median(st[:, 2] - st[:, 1]))
idx, gat, fix, mf, bar, items = [], [], [], [], [], []
for row in st:
    k = 0
    prev = row[2]
    n = 0
    while 7 + 5 * k < 62 and row[7 + 5 * k] > 0:
        m, i0, i1, i2, b = row[3 + 5 * k], row[4 + 5 * k], row[5 + 5 * k], row[6 + 5 * k], row[7 + 5 * k]
        mf.append(m - prev)
        if i0 > 0:
            idx.append(i0 - prev)
            if i1 > 0:
                gat.append(i1 - i0)
                fix.append(i2 - i1)
        bar.append(b - prev)
        prev = b
        k += 1
        n += 1
    items.append(n)
for name, a in [("mfma", mf), ("gather_index", idx), ("gather_loop", gat), ("divide_fixup", fix), ("item", bar),
                ("items_per_wg", items)]:
    a = np.asarray(a)
    if len(a):
        res[name] = {"p10": float(np.percentile(a, 10)), "p50": float(np.median(a)), "p90": float(np.percentile(a, 90)),
                     "max": float(a.max()), "n": len(a)}
print(json.dumps(res))
