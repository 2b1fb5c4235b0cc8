#!/usr/bin/env python3
"""Per-workgroup timeline of rel_gemm_kernel (debug stamps, MPGNN_OPT_STAMPS): prologue, per-item
MFMA loop and epilogue+barrier lengths (shader clocks), one FB15K layer forward."""
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
buf = torch.zeros((1 << 20) + 65536 * 8, dtype=torch.int64, device="cuda")
_lib.lib.mpgnn_set_option(2, buf.data_ptr())
with torch.no_grad():
    conv(x, ei, et)
torch.cuda.synchronize()
_lib.lib.mpgnn_set_option(2, 0)
st = buf[: 512 * 32].cpu().numpy().reshape(512, 32).astype(np.float64)
live = st[:, 0] > 0
st = st[live]
res = {"wgs": int(live.sum())}
pro = st[:, 1] - st[:, 0]
mf, ep = [], []
for row in st:
    k = 0
    prev = row[1]
    while 3 + 2 * k < 32 and row[3 + 2 * k] > 0:
        mf.append(row[2 + 2 * k] - prev)
        ep.append(row[3 + 2 * k] - row[2 + 2 * k])
        prev = row[3 + 2 * k]
        k += 1
rt0 = st[:, 30].min()
rt_start = (st[:, 30] - rt0) * 10.0  # ns (100 MHz)
rt_end = (st[:, 31] - rt0) * 10.0
clk = (st[:, 2 * 0 + 0] * 0)  # placeholder
span_clk = np.array([max(r[k] for k in range(30) if r[k] > 0) - r[0] for r in st])
ghz = span_clk / np.maximum(rt_end - rt_start, 1.0)
res["clock_GHz_p50"] = float(np.median(ghz))
for name, a in [("rt_start_ns", rt_start), ("rt_end_ns", rt_end), ("rt_span_ns", rt_end - rt_start)]:
    res[name] = {"p10": float(np.percentile(a, 10)), "p50": float(np.median(a)), "p90": float(np.percentile(a, 90)),
                 "max": float(a.max())}
for name, a in [("prologue", pro), ("mfma_item", mf), ("epi_commit_barrier", ep)]:
    a = np.asarray(a)
    res[name] = {"p10": float(np.percentile(a, 10)), "p50": float(np.median(a)), "p90": float(np.percentile(a, 90)),
                 "max": float(a.max()), "n": len(a)}
print(json.dumps(res))
# per-workgroup: items processed vs end time (load balance)
items = np.array([sum(1 for k in range(30) if 3 + 2 * k < 30 and r[3 + 2 * k] > 0) for r in st])
ends = rt_end
bal = {}
for n in sorted(set(items.tolist())):
    m = items == n
    bal[int(n)] = {"wgs": int(m.sum()), "end_p50_ns": float(np.median(ends[m])), "end_max_ns": float(ends[m].max())}
print(json.dumps({"balance": bal}))
