#!/usr/bin/env python3
"""Per-rank compute of the dst-range-sharded forward at N = 1, 2, 4, 8 shards, measured on ONE
GPU (each shard's 3-layer partial forward timed in turn; the reduce-scatter / all-gather are
not included). Bounds what `bench.py --gpus N` can reach: step time ≥ max over ranks of this
compute + the collectives."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402
from mpgnn_amd import data  # noqa: E402
from mpgnn_amd.distributed import shard_ranges  # noqa: E402

g = data.config_graph("fb15k237")
torch.manual_seed(10)
net = mpgnn_amd.Net(128, 128, g.num_relations, 128, 2, 3).cuda()
x, ei, et = g.x.cuda(), g.edge_index.cuda(), g.edge_type.cuda()
convs = [net.conv1, net.conv2, net.conv2]
res = {}
side = sys.argv[1] if len(sys.argv) > 1 else "gathered"
# clock pre-warm (as bench.py): ~0.3 s of back-to-back unsharded steps before any timing, so the
# first world size is not timed on the chip's idle clocks
with torch.no_grad():
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        for _ in range(10):
            h = x
            for conv in convs:
                h = torch.relu(conv(h, ei, et))
        torch.cuda.synchronize()
for world in (1, 2, 4, 8):
    per_rank = []
    segs = []
    for lo, hi in shard_ranges(g.edge_index, g.num_nodes, world, side=side):
        shard = None if world == 1 else (lo, hi)

        def step():
            h = x
            for conv in convs:
                h = torch.relu(conv(h, ei, et, shard=shard, shard_side=side))
            return h

        with torch.no_grad():
            for _ in range(5):
                step()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(50):
                step()
            torch.cuda.synchronize()
        per_rank.append((time.perf_counter() - t) * 1e3 / 50)
        segs.append(mpgnn_amd.get_plan(ei, et, g.num_nodes, shard=shard, device=x.device,
                                       shard_side=side).num_segments)
    res[world] = {"max_rank_ms_per_step": round(max(per_rank), 4), "per_rank_ms": [round(v, 4) for v in per_rank],
                  "segments_per_rank": segs, "compute_speedup": None}
base = res[1]["max_rank_ms_per_step"]
for w in res:
    res[w]["compute_speedup"] = round(base / res[w]["max_rank_ms_per_step"], 3)
print(json.dumps({"workload": "C3 FB15K-237, 3-layer forward, per-rank compute only (no collectives)",
                  "shard_side": side,
                  "by_world": res}))
