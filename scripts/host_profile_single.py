#!/usr/bin/env python3
"""cProfile of the eager C3 mode-SINGLE training epoch (bench.py's epoch(): MPNetm train forward,
NLL, backward, LeanAdam step, validation forward) on the GPU: where the host time goes.
usage: python scripts/host_profile_single.py [epochs] > out.txt"""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402
from mpgnn_amd import data  # noqa: E402

n_ep = int(sys.argv[1]) if len(sys.argv) > 1 else 200
dev = torch.device("cuda", 0)
g = data.config_graph("fb15k237")
x, ei, et = g.x.to(dev), g.edge_index.to(dev), g.edge_type.to(dev)
F = x.shape[1]
rel_counts = torch.bincount(g.edge_type, minlength=g.num_relations)
metapath = [int(v) for v in torch.argsort(rel_counts, descending=True, stable=True)[:3]]
torch.manual_seed(10)
model = mpgnn_amd.MPNetm(F, F, g.num_relations, F, 2, 1, [metapath]).to(dev)
opt = mpgnn_amd.main._adam(model)
y = torch.randint(0, 2, (g.num_nodes,), generator=torch.Generator().manual_seed(0)).to(dev)
train_idx = torch.arange(0, g.num_nodes, 3, device=dev)
train_y = y[train_idx]


def epoch():
    model.train()
    opt.zero_grad()
    out = model(x, ei, et)
    loss = mpgnn_amd.metrics.nll_loss_rows(out, train_idx, train_y)
    loss.backward()
    opt.step()
    model.eval()
    with torch.no_grad():
        model(x, ei, et)


for _ in range(10):
    epoch()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(n_ep):
    epoch()
torch.cuda.synchronize()
print(f"eager epoch {(time.perf_counter() - t0) * 1e3 / n_ep:.3f} ms (no profiler)")
pr = cProfile.Profile()
pr.enable()
for _ in range(n_ep):
    epoch()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(40)
