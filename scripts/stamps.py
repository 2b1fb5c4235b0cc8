#!/usr/bin/env python3
"""Per-workgroup timeline of the forward tile kernel (debug stamps, MPGNN_OPT_STAMPS).
Prints concurrency per CU, phase durations and the makespan for one FB15K layer forward."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402
from mpgnn_amd import _lib, data  # noqa: E402

abl = int(sys.argv[1]) if len(sys.argv) > 1 else 0
g = data.config_graph("fb15k237")
x = torch.rand(g.num_nodes, 128, device="cuda")
ei, et = g.edge_index.cuda(), g.edge_type.cuda()
conv = mpgnn_amd.RGCNConv(128, 128, g.num_relations, flow="target_to_source").cuda()
with torch.no_grad():
    for _ in range(5):
        conv(x, ei, et)
torch.cuda.synchronize()
buf = torch.zeros(4096 * 32, dtype=torch.int64, device="cuda")
_lib.lib.mpgnn_set_option(1, abl)
_lib.lib.mpgnn_set_option(2, buf.data_ptr())
with torch.no_grad():
    conv(x, ei, et)
torch.cuda.synchronize()
_lib.lib.mpgnn_set_option(2, 0)
_lib.lib.mpgnn_set_option(1, 0)
st = buf.cpu().numpy().reshape(-1, 4, 8)
st = st[st[:, 0, 0] != 0]
t0 = st[:, :, 0].min()
start, loaded, mf, end = (st[:, :, i] - t0 for i in range(4))
hw = st[:, 0, 4].astype(np.int64)
xcc = st[:, 0, 5]
cu = (hw >> 8) & 0xF
se = (hw >> 13) & 0x7
simd = (hw >> 4) & 0x3
key = xcc * 1000 + se * 100 + cu
res = {"blocks": int(len(st)), "makespan_ticks": int(end.max()),
       "load_phase_median": float(np.median(loaded[:, 0] - start[:, 0])),
       "mfma_phase_median": float(np.median(mf.max(1) - loaded[:, 0])),
       "epi_phase_median": float(np.median(end.max(1) - mf.max(1))),
       "block_life_median": float(np.median(end.max(1) - start[:, 0])),
       "block_life_max": float((end.max(1) - start[:, 0]).max()),
       "distinct_cus": int(len(np.unique(key)))}
# concurrency per CU: max overlapping blocks
conc = []
for k in np.unique(key):
    m = key == k
    ev = sorted([(s, 1) for s in start[m, 0]] + [(e, -1) for e in end[m].max(1)])
    c = mx = 0
    for _, d in ev:
        c += d
        mx = max(mx, c)
    conc.append(mx)
res["max_concurrent_per_cu_hist"] = np.bincount(conc).tolist()
res["blocks_per_cu_hist"] = np.bincount(np.unique(key, return_counts=True)[1]).tolist()
res["start_spread_ticks"] = float(np.percentile(start[:, 0], 99) - start[:, 0].min())
print(json.dumps(res))
