"""Python-level host cost of the eager C3 epoch (bench.py's kernel epoch) by function: cProfile
over N epochs, sorted by own time (which Python lines of the wrappers cost host time).
usage: python scripts/epoch_cprofile.py [--mode single|all] [--epochs 50]"""
import argparse
import cProfile
import io
import os
import pstats
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mpgnn_amd  # noqa: E402
from mpgnn_amd import data  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--mode", default="single", choices=["single", "all"])
ap.add_argument("--epochs", type=int, default=50)
a = ap.parse_args()
dev = torch.device("cuda", 0)
g = data.config_graph("fb15k237")
F = 128
x, ei, et = g.x[:, :F].contiguous().to(dev), g.edge_index.to(dev), g.edge_type.to(dev)
torch.manual_seed(10)
if a.mode == "single":
    rel_counts = torch.bincount(g.edge_type, minlength=g.num_relations)
    metapath = [int(v) for v in torch.argsort(rel_counts, descending=True, stable=True)[:3]]
    model = mpgnn_amd.MPNetm(F, F, g.num_relations, F, 2, 1, [metapath]).to(dev)
else:
    model = mpgnn_amd.Net(F, F, g.num_relations, F, 2, 3).to(dev)
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
pr = cProfile.Profile()
pr.enable()
for _ in range(a.epochs):
    epoch()
torch.cuda.synchronize()
pr.disable()
s = io.StringIO()
st = pstats.Stats(pr, stream=s)
st.sort_stats("tottime").print_stats(45)
print(s.getvalue())
