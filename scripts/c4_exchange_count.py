"""C4 (the C3 graph sharded by node_2 range over W ranks): how many rows of each
rank's partial output are non-zero, i.e. what a sparse row exchange would move against the
padded reduce-scatter of distributed.sharded_stack_forward. A partial row i
is non-zero on rank k when some edge (i, r, j) has node_2 j in k's range, or i is in k's range
(x_i @ root + bias). Exact integer counts from the graph; CPU only.
usage: python scripts/c4_exchange_count.py [--workload fb15k237] > profiles/r05_c4_exchange_count.json"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpgnn_amd import data  # noqa: E402
from mpgnn_amd.distributed import shard_ranges  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="fb15k237")
ap.add_argument("--feat", type=int, default=128)
a = ap.parse_args()
g = data.config_graph(a.workload)
N = g.num_nodes
n1, n2 = g.edge_index[0].numpy(), g.edge_index[1].numpy()
res = {"workload": a.workload, "N": N, "E": int(n1.size), "F": a.feat, "worlds": {}}
for W in (2, 4, 8):
    ranges = shard_ranges(g.edge_index, N, W)
    per = []
    for lo, hi in ranges:
        m = (n2 >= lo) & (n2 < hi)
        rows = np.zeros(N, bool)
        rows[n1[m]] = True
        rows[lo:hi] = True  # root term of the own rows
        nz = int(rows.sum())
        per.append({"range": [int(lo), int(hi)], "edges": int(m.sum()), "nonzero_rows": nz,
                    "nonzero_frac": round(nz / N, 4)})
    pad = max(hi - lo for lo, hi in ranges)
    # bytes sent per rank per layer: padded reduce-scatter (ring) = (W-1)/W of the W·pad padded rows;
    # sparse exchange = its non-zero rows outside its own range (row id + F floats each)
    rs_bytes = (W - 1) * pad * a.feat * 4
    sparse = [p["nonzero_rows"] - (p["range"][1] - p["range"][0]) for p in per]
    res["worlds"][W] = {
        "ranks": per,
        "nonzero_frac_max": max(p["nonzero_frac"] for p in per),
        "nonzero_frac_mean": round(float(np.mean([p["nonzero_frac"] for p in per])), 4),
        "reduce_scatter_bytes_per_rank": rs_bytes,
        "sparse_bytes_per_rank_max": max(sparse) * (a.feat * 4 + 4),
        "sparse_over_reduce_scatter": round(max(sparse) * (a.feat * 4 + 4) / rs_bytes, 3),
    }
print(json.dumps(res, indent=1))
