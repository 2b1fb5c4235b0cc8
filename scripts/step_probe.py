#!/usr/bin/env python3
"""Where the C3 forward step's time between kernels goes (bench.py's headline step, mode ALL,
3 layers, 128-d): eager step time as bench.py times it, the host's issue time per step (steps
enqueued behind a long GPU sleep, so the host never waits), and the step replayed from a HIP
graph (no host issue at all). Alternated --rounds times in one process.
usage: python scripts/step_probe.py [--steps 20] [--rounds 3] [--opt K=V ...]"""
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
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--opt", action="append", default=[], help="K=V process default before the plan is built")
ap.add_argument("--json", default=None)
ap.add_argument("--no-check", action="store_true", help="skip the graph == eager check (probe libraries)")
a = ap.parse_args()
for kv in a.opt:
    k, v = kv.split("=")
    _lib.set_option(int(k), int(v))
dev = torch.device("cuda", 0)
g = data.fb15k237_graph(feat_dim=128, seed=0, recipe="survey")
F = 128
model = mpgnn_amd.Net(F, F, g.num_relations, F, 2, 3).to(dev)
convs = [model.conv1] + [model.conv2] * 2
x = g.x.to(dev).contiguous()
ei, et = g.edge_index.to(dev), g.edge_type.to(dev)


def step():
    h = x
    for conv in convs:
        h = conv(h, ei, et, activation="relu")
    return h


with torch.no_grad():
    for _ in range(5):
        ref = step()
torch.cuda.synchronize()


def eager():
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.no_grad():
        for _ in range(a.steps):
            step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / a.steps * 1e6


def host_issue():
    torch.cuda.synchronize()
    torch.cuda._sleep(int(2e8))  # ~0.1 s of GPU spin: the steps queue behind it
    t0 = time.perf_counter()
    with torch.no_grad():
        for _ in range(a.steps):
            step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) / a.steps * 1e6


side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side), torch.no_grad():
    for _ in range(3):
        step()
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph), torch.no_grad():
    gout = step()
graph.replay()
torch.cuda.synchronize()
assert a.no_check or torch.equal(gout, ref), "graph replay differs from the eager step"


def replay():
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        graph.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / a.steps * 1e6


res = {"eager_us": [], "host_issue_us": [], "graph_us": []}
for _ in range(a.rounds):
    res["eager_us"].append(round(eager(), 2))
    res["host_issue_us"].append(round(host_issue(), 2))
    res["graph_us"].append(round(replay(), 2))
res["opts"] = a.opt
res["edges_per_step"] = 3 * g.num_edges
res["eager_G_edges_s"] = round(3 * g.num_edges / (min(res["eager_us"]) * 1e-6) / 1e9, 3)
res["graph_G_edges_s"] = round(3 * g.num_edges / (min(res["graph_us"]) * 1e-6) / 1e9, 3)
print(json.dumps(res), flush=True)
if a.json:
    json.dump(res, open(a.json, "w"), indent=1)
