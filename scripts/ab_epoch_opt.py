#!/usr/bin/env python3
"""A/B of one library option on the bench's C3 mode-ALL epoch (main_rgcn.py:458-461: train
forward + NLL + backward + Adam, then a validation forward), eager and graph-replayed, the
settings alternated three times on one box.  usage: ab_epoch_opt.py OPTION VALUE_A VALUE_B"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402
from mpgnn_amd import _lib, data  # noqa: E402

opt_id, va, vb = (int(v) for v in sys.argv[1:4])
g = data.fb15k237_graph(feat_dim=128, seed=0, recipe="survey")
dev = "cuda"
x, ei, et = g.x.to(dev), g.edge_index.to(dev), g.edge_type.to(dev)
y = torch.randint(0, 2, (g.num_nodes,), generator=torch.Generator().manual_seed(0)).to(dev)
train_idx = torch.arange(0, g.num_nodes, 3, device=dev)
res = {}
for rep in range(3):
    for val in (va, vb):
        _lib.set_option(opt_id, val)
        torch.manual_seed(10)
        net = mpgnn_amd.Net(128, 128, g.num_relations, 128, 2, 3).to(dev)
        opt = torch.optim.Adam(net.parameters(), lr=0.01, weight_decay=0.0005, fused=True, capturable=True)

        def epoch():
            net.train()
            opt.zero_grad(set_to_none=False)
            out = net(x, ei, et)
            loss = torch.nn.functional.nll_loss(out[train_idx], y[train_idx])
            loss.backward()
            opt.step()
            net.eval()
            with torch.no_grad():
                net(x, ei, et)

        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(3):
                epoch()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(30):
            epoch()
        torch.cuda.synchronize()
        eager = (time.perf_counter() - t) * 1e3 / 30
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            epoch()
        gr.replay()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(30):
            gr.replay()
        torch.cuda.synchronize()
        graphed = (time.perf_counter() - t) * 1e3 / 30
        res.setdefault(val, []).append((round(eager, 4), round(graphed, 4)))
        print(f"option {opt_id}={val}: eager {eager:.4f} ms, graphed {graphed:.4f} ms", flush=True)
        del gr
for val, v in res.items():
    print(val, "eager min", min(e for e, _ in v), "graphed min", min(gg for _, gg in v))
