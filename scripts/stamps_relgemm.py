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
t0 = st[:, 0].min()
res = {"wgs": int(live.sum())}
start = st[:, 0] - t0
pro = st[:, 1] - st[:, 0]
mf, ep, end = [], [], []
for row in st:
    k = 0
    prev = row[1]
    while 3 + 2 * k < 32 and row[3 + 2 * k] > 0:
        mf.append(row[2 + 2 * k] - prev)
        ep.append(row[3 + 2 * k] - row[2 + 2 * k])
        prev = row[3 + 2 * k]
        k += 1
    end.append(prev - t0)
for name, a in [("start", start), ("prologue", pro), ("mfma_item", mf), ("epi_commit_barrier", ep), ("end", end)]:
    a = np.asarray(a)
    res[name] = {"p10": float(np.percentile(a, 10)), "p50": float(np.median(a)), "p90": float(np.percentile(a, 90)),
                 "max": float(a.max()), "n": len(a)}
print(json.dumps(res))
