#!/usr/bin/env python3
"""Kernel-time vs wall-time of the bench epoch (run under rocprofv3 --kernel-trace): prints the
wall ms per epoch; the trace gives the GPU busy time of the same epochs."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402
from mpgnn_amd import data  # noqa: E402

g = data.config_graph("fb15k237")
dev = "cuda"
x, ei, et = g.x.to(dev), g.edge_index.to(dev), g.edge_type.to(dev)
y = torch.randint(0, 2, (g.num_nodes,), generator=torch.Generator().manual_seed(0)).to(dev)
train_idx = torch.arange(0, g.num_nodes, 3, device=dev)
torch.manual_seed(10)
net = mpgnn_amd.Net(128, 128, g.num_relations, 128, 2, 3).to(dev)
opt = mpgnn_amd.main._adam(net)


def epoch():
    net.train()
    opt.zero_grad()
    out = net(x, ei, et)
    loss = torch.nn.functional.nll_loss(out[train_idx], y[train_idx])
    loss.backward()
    opt.step()
    net.eval()
    with torch.no_grad():
        net(x, ei, et)


for _ in range(5):
    epoch()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(20):
    epoch()
torch.cuda.synchronize()
print("wall ms/epoch", round((time.perf_counter() - t) * 1e3 / 20, 4), flush=True)
