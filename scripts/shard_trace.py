#!/usr/bin/env python3
"""One node_2 shard's 3-layer partial forward (C3, `world` shards, rank `rank`), 30 steps after a
0.3-s pre-warm — run under `rocprofv3 --kernel-trace` to see which launches make up the per-rank
step at the latency floor (scripts/shard_compute.py times it without a profiler); then
`python scripts/shard_trace.py --report <run_kernel_trace.csv>` prints per-kernel averages.
usage: python scripts/shard_trace.py [world] [rank]"""
import csv
import os
import sys
import time
from collections import defaultdict

if len(sys.argv) > 2 and sys.argv[1] == "--report":
    rows = list(csv.DictReader(open(sys.argv[2])))
    by = defaultdict(list)
    for r in rows:
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:80]
        by[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for n, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        if len(v) >= 30:
            print(f"{len(v):6d}x {sum(v) / len(v):8.2f} us  {n}")
    sys.exit(0)
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402
from mpgnn_amd import data  # noqa: E402
from mpgnn_amd.distributed import shard_ranges  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
rank = int(sys.argv[2]) if len(sys.argv) > 2 else 0
g = data.config_graph("fb15k237")
torch.manual_seed(10)
net = mpgnn_amd.Net(128, 128, g.num_relations, 128, 2, 3).cuda()
x, ei, et = g.x.cuda(), g.edge_index.cuda(), g.edge_type.cuda()
convs = [net.conv1, net.conv2, net.conv2]
lo, hi = shard_ranges(g.edge_index, g.num_nodes, world)[rank]


def step():
    h = x
    for conv in convs:
        h = torch.relu(conv(h, ei, et, shard=(lo, hi)))
    return h


with torch.no_grad():
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        for _ in range(10):
            step()
        torch.cuda.synchronize()
    for _ in range(30):
        step()
    torch.cuda.synchronize()
print("done", world, rank, lo, hi)
