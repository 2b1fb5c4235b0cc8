#!/usr/bin/env python3
"""cProfile of the eager MPNetm training epoch at C3 (mode SINGLE, 3-hop metapath of the three
most frequent relations, 128-d): where the host time of an epoch goes (bench.py --mode single)."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402
from mpgnn_amd import data  # noqa: E402

g = data.fb15k237_graph(feat_dim=128, seed=0)
dev = torch.device("cuda", 0)
x, ei, et = g.x.to(dev), g.edge_index.to(dev), g.edge_type.to(dev)
counts = torch.bincount(g.edge_type, minlength=g.num_relations)
meta = [int(v) for v in torch.argsort(counts, descending=True, stable=True)[:3]]
torch.manual_seed(10)
model = mpgnn_amd.MPNetm(128, 128, g.num_relations, 128, 2, 1, [meta]).to(dev)
opt = mpgnn_amd.main._adam(model)
y = torch.randint(0, 2, (g.num_nodes,)).to(dev)
idx = torch.arange(0, g.num_nodes, 3, device=dev)
ty = y[idx]


def epoch():
    model.train()
    opt.zero_grad()
    out = model(x, ei, et)
    loss = torch.nn.functional.nll_loss(out.index_select(0, idx), ty)
    loss.backward()
    opt.step()
    model.eval()
    with torch.no_grad():
        model(x, ei, et)


for _ in range(5):
    epoch()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(50):
    epoch()
torch.cuda.synchronize()
print("eager epoch ms", (time.perf_counter() - t) * 1e3 / 50)
t = time.perf_counter()
for _ in range(50):
    epoch()
print("host issue ms per epoch (no sync)", (time.perf_counter() - t) * 1e3 / 50)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(50):
    epoch()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(30)
