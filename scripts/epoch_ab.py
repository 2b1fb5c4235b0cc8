#!/usr/bin/env python3
"""A/B the epoch of bench.py (main_rgcn.py:458-461: train fwd + NLL + bwd + Adam, then a
validation forward) on the FB15K shape for optimizer implementations (foreach vs fused Adam)
and reports the spread of parameters after N epochs between them."""
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
res = {}
for kind in ["foreach", "fused", "foreach"]:
    torch.manual_seed(10)
    net = mpgnn_amd.Net(128, 128, g.num_relations, 128, 2, 3).to(dev)
    opt = torch.optim.Adam(net.parameters(), lr=0.01, weight_decay=0.0005, **{kind: True})

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

    for _ in range(3):
        epoch()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(30):
        epoch()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 1e3 / 30
    res.setdefault(kind, []).append(ms)
    print(kind, round(ms, 4), "ms/epoch", flush=True)
    if kind == "fused":
        p_fused = [p.detach().clone() for p in net.parameters()]
    else:
        p_fe = [p.detach().clone() for p in net.parameters()]
print("max |fused - foreach| after 33 epochs:", max(float((a - b).abs().max()) for a, b in zip(p_fused, p_fe)))
