"""Diagnostic: one mode-ALL layer's weight / root / bias / x gradients on the GPU against the
float64 oracle on a chosen graph; per-relation error table for the worst relations.
Usage: python scripts/diag_dw.py [--graph fb15k237] [--fout 64] [--opt NAME=VAL ...]"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mpgnn_amd  # noqa: E402
from mpgnn_amd import _lib, data  # noqa: E402
from mpgnn_amd.functional import MODE_ALL, rgcn_conv  # noqa: E402
from mpgnn_amd.plan import GraphPlan  # noqa: E402
from oracle import rgcn_oracle as orc  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--graph", default="fb15k237")
ap.add_argument("--fout", type=int, default=64)
ap.add_argument("--fin", type=int, default=0)
ap.add_argument("--opt", action="append", default=[])
a = ap.parse_args()
for o in a.opt:
    k, v = o.split("=")
    _lib.check(_lib.lib.mpgnn_set_option(int(k), int(v)), "opt")

g = data.config_graph(a.graph)
if a.fin:
    g.x = g.x[:, :a.fin].contiguous()
F, R, N = g.x.shape[1], g.num_relations, g.num_nodes
gen = torch.Generator().manual_seed(5)
W = torch.randn(R, F, a.fout, generator=gen) * 0.1
root = torch.randn(F, a.fout, generator=gen) * 0.1
bias = torch.randn(a.fout, generator=gen) * 0.1
dout = torch.randn(N, a.fout, generator=gen)

p = {k: v.double().requires_grad_(True) for k, v in dict(W=W, root=root, bias=bias).items()}
x64 = g.x.double().requires_grad_(True)
out64 = orc.rgcn_forward(x64, g.edge_index, g.edge_type, p["W"], p["root"], p["bias"])
out64.backward(dout.double())

dev = "cuda"
plan = GraphPlan(g.edge_index, g.edge_type, N)
print("plan: S", plan.num_segments, "tiles", plan.num_tiles, "chunks", plan.num_chunks)
xg = g.x.to(dev).requires_grad_(True)
Wg, rg, bg = (t.to(dev).requires_grad_(True) for t in (W, root, bias))
out = rgcn_conv(xg, Wg, rg, bg, plan, MODE_ALL, -1, R)
out.backward(dout.to(dev))
torch.cuda.synchronize()


def rep(name, got, ref):
    got = got.detach().double().cpu()
    ref = ref.detach().cpu()
    scale = float(ref.abs().max())
    err = (got - ref).abs()
    print(f"{name}: max|ref| {scale:.3e} max abs err {float(err.max()):.3e} norm {float(err.max()) / max(scale, 1e-30):.3e}")
    return err, scale


rep("out", out, out64)
rep("gx", xg.grad, x64.grad)
rep("groot", rg.grad, p["root"].grad)
rep("gbias", bg.grad, p["bias"].grad)
err, scale = rep("gW", Wg.grad, p["W"].grad)
per = err.flatten(1).max(1).values / p["W"].grad.abs().flatten(1).max(1).values.clamp_min(1e-30)
cnt = np.bincount(g.edge_type.numpy(), minlength=R)
s_rel = plan.table("s_rel")
scnt = np.bincount(s_rel, minlength=R)
order = torch.argsort(per, descending=True)[:12]
for r in order.tolist():
    print(f"  rel {r:4d} edges {cnt[r]:6d} segs {scnt[r]:6d} rel-normalised err {float(per[r]):.3e}")
print("relations with normalised err > 1e-3:", int((per > 1e-3).sum()))
