#!/usr/bin/env python3
"""Per-wave timeline of the segment-means row-sum launch (debug stamps, MPGNN_OPT_STAMPS):
wave lifetimes, prologue vs gather time, concurrency and entries per wave, one FB15K layer."""
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
st = buf[1 << 20:].cpu().numpy().reshape(-1, 8)
st = st[st[:, 7] == 1]
# s_memtime clocks are not comparable across CUs: normalise each CU to its own first wave
xcc_id = st[:, 5]
hw0 = st[:, 4].astype(np.int64)
cu_key = xcc_id * 10000 + ((hw0 >> 13) & 7) * 1000 + ((hw0 >> 12) & 1) * 100 + ((hw0 >> 8) & 0xF)
t0 = np.zeros(len(st), dtype=np.int64)
for kv in np.unique(cu_key):
    t0[cu_key == kv] = st[cu_key == kv, 0].min()
start, pro, end = st[:, 0] - t0, st[:, 1] - t0, st[:, 2] - t0
ent = st[:, 3]
life = end - start
hw = st[:, 4].astype(np.int64)
cu = (st[:, 5] * 1000 + ((hw >> 13) & 7) * 100 + ((hw >> 8) & 0xF))
res = {
    "waves": int(len(st)), "makespan": int(end.max()),
    "life_p50": float(np.percentile(life, 50)), "life_p90": float(np.percentile(life, 90)),
    "life_max": int(life.max()),
    "prologue_p50": float(np.percentile(pro - start, 50)),
    "gather_p50": float(np.percentile(end - pro, 50)),
    "entries_p50": float(np.percentile(ent, 50)), "entries_p99": float(np.percentile(ent, 99)),
    "entries_max": int(ent.max()),
    "start_p50": float(np.percentile(start, 50)), "start_p90": float(np.percentile(start, 90)),
    "start_max": int(start.max()),
    "end_p50": float(np.percentile(end, 50)), "end_p99": float(np.percentile(end, 99)),
    "distinct_cus": int(len(np.unique(cu))),
}
mk = np.array([end[cu_key == kv].max() for kv in np.unique(cu_key)])
res["cu_makespan_p50"] = float(np.median(mk))
res["cu_makespan_max"] = int(mk.max())
res["waves_per_cu_p50"] = float(np.median(np.unique(cu_key, return_counts=True)[1]))
# per-CU concurrency: max waves alive at once, and mean alive over the CU's makespan
mx, mean_alive = [], []
for kv in np.unique(cu_key):
    m = cu_key == kv
    ev = sorted([(a_, 1) for a_ in start[m]] + [(b_, -1) for b_ in end[m]])
    c = top = 0
    for _, d in ev:
        c += d
        top = max(top, c)
    mx.append(top)
    mean_alive.append(float(life[m].sum()) / float(end[m].max()))
res["cu_max_alive_p50"] = float(np.median(mx))
res["cu_mean_alive_p50"] = float(np.median(mean_alive))
# time-sampled concurrency (waves alive) over the makespan
ts = np.linspace(0, np.percentile(end, 99), 20)
res["alive_curve"] = [int(((start <= t) & (end > t)).sum()) for t in ts]
# life vs entries correlation
for lo, hi in [(0, 16), (16, 32), (32, 64), (64, 10**9)]:
    m = (ent >= lo) & (ent < hi)
    if m.any():
        res[f"life_p50_ent_{lo}_{hi}"] = float(np.median(life[m]))
        res[f"n_ent_{lo}_{hi}"] = int(m.sum())
print(json.dumps(res))
