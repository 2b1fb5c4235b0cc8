"""Per-epoch time of the drop-in loops on C3 (mode ALL: main_rgcn, mode SINGLE: main) with the
per-epoch HIP graph on and off, and whether the capture fell back to eager epochs (its reason).
usage: python scripts/loop_capture_check.py"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpgnn_amd import data, main, main_rgcn  # noqa: E402

dev = torch.device("cuda", 0)
g = data.config_graph("fb15k237")
F = 128
x, ei, et = g.x[:, :F].contiguous().to(dev), g.edge_index.to(dev), g.edge_type.to(dev)
n = g.num_nodes
gen = torch.Generator().manual_seed(0)
y = torch.randint(0, 2, (n,), generator=gen)
perm = torch.randperm(n, generator=gen)
a, b = int(0.6 * n), int(0.8 * n)
tr, va, te = (perm[:a].sort().values, perm[a:b].sort().values, perm[b:].sort().values)
d = main.Data(x=x, edge_index=ei, edge_type=et, train_idx=tr.to(dev), train_y=y[tr].to(dev),
              val_idx=va.to(dev), val_y=y[va].to(dev), test_idx=te.to(dev), test_y=y[te].to(dev))
rel_counts = torch.bincount(g.edge_type, minlength=g.num_relations)
metapath = [int(v) for v in torch.argsort(rel_counts, descending=True, stable=True)[:3]]
runs = {"all": lambda k: main_rgcn.mpgnn_parallel_multiple(d, F, F, g.num_relations, F, 2, 3, epochs=k, verbose=False),
        "single": lambda k: main.mpgnn_parallel_multiple(d, F, F, g.num_relations, F, 2, [metapath], epochs=k)}
res = {}
for mode, run in runs.items():
    for graph in ("1", "0"):
        os.environ["MPGNN_LOOP_GRAPH"] = graph
        main.LAST_CAPTURE_ERROR = None
        run(6)
        ts = {}
        for k in (6, 46):
            best = None
            for _ in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                run(k)
                torch.cuda.synchronize()
                t = time.perf_counter() - t0
                best = t if best is None else min(best, t)
            ts[k] = best
        res[f"{mode}_graph{graph}"] = {"ms_per_epoch": round((ts[46] - ts[6]) / 40 * 1e3, 4),
                                       "capture_error": main.LAST_CAPTURE_ERROR}
        print(json.dumps(res), flush=True)
