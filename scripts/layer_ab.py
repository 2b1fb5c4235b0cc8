"""A/B probe: per-kernel-kind µs of one RGCN layer (forward, and with --backward the training
step's backward) on a bench workload; compare builds / env switches by running it twice.
usage: python scripts/layer_ab.py [--workload fb15k237|C2|C5] [--iters 30] [--backward] [--label X]"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mpgnn_amd  # noqa: E402
from mpgnn_amd import _lib, data  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="fb15k237")
ap.add_argument("--iters", type=int, default=30)
ap.add_argument("--backward", action="store_true")
ap.add_argument("--label", default="")
ap.add_argument("--chunk-rows", type=int, default=0, help="MPGNN_OPT_CHUNK_ROWS (0: default)")
a = ap.parse_args()
if a.chunk_rows:
    _lib.check(_lib.lib.mpgnn_set_option(20, a.chunk_rows))
g = data.config_graph(a.workload)
dev = torch.device("cuda", 0)
F = g.x.shape[1]
torch.manual_seed(10)
conv = mpgnn_amd.RGCNConv(F, F, g.num_relations, flow="target_to_source").to(dev)
x, ei, et = g.x.to(dev), g.edge_index.to(dev), g.edge_type.to(dev)
xg = x.clone().requires_grad_(a.backward)


def run():
    if a.backward:
        out = conv(xg, ei, et, activation="relu")
        out.sum().backward()
    else:
        with torch.no_grad():
            conv(x, ei, et, activation="relu")


for _ in range(3):
    run()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.iters):
    run()
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / a.iters * 1e6
_lib.lib.mpgnn_timing_reset()
_lib.lib.mpgnn_timing_enable(1)
for _ in range(a.iters):
    run()
torch.cuda.synchronize()
_lib.lib.mpgnn_timing_enable(0)
res = {"label": a.label, "workload": a.workload, "env": {k: v for k, v in os.environ.items() if k.startswith("MPGNN_")},
       "chunk_rows": a.chunk_rows,
       "wall_us_per_iter": round(wall, 2)}
for kind in _lib.KERNEL_KINDS:
    ms, n = _lib.kernel_timing(kind)
    if n:
        res[kind] = round(ms * 1e3 / a.iters, 2)
print(json.dumps(res), flush=True)
