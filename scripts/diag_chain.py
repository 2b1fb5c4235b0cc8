"""Diagnostic: two stacked mode-ALL layers (fused ReLU or not, shared weights or not) on the GPU vs
the float64 oracle; prints each gradient's normalised max error. Usage: python scripts/diag_chain.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mpgnn_amd  # noqa: E402
from mpgnn_amd import _lib, data  # noqa: E402
from mpgnn_amd.functional import MODE_ALL, rgcn_conv  # noqa: E402
from mpgnn_amd.plan import GraphPlan  # noqa: E402
from oracle import rgcn_oracle as orc  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "fb15k237"
g = data.config_graph(name)
F, R, N = g.x.shape[1], g.num_relations, g.num_nodes
gen = torch.Generator().manual_seed(5)
H = 64
P = dict(W1=torch.randn(R, F, H, generator=gen) * 0.1, r1=torch.randn(F, H, generator=gen) * 0.1,
         b1=torch.randn(H, generator=gen) * 0.1, W2=torch.randn(R, H, H, generator=gen) * 0.1,
         r2=torch.randn(H, H, generator=gen) * 0.1, b2=torch.randn(H, generator=gen) * 0.1)
dout = torch.randn(N, H, generator=gen)
plan = GraphPlan(g.edge_index, g.edge_type, N)


def run(dev, fused, layers):
    p = {k: (v.double() if dev == "cpu" else v.to(dev)).requires_grad_(True) for k, v in P.items()}
    x = g.x.double() if dev == "cpu" else g.x.to(dev)
    h = x
    for li in range(layers):
        W, r, b = (p["W1"], p["r1"], p["b1"]) if li == 0 else (p["W2"], p["r2"], p["b2"])
        if dev == "cpu":
            h = torch.relu(orc.rgcn_forward(h, g.edge_index, g.edge_type, W, r, b))
        elif fused:
            h = rgcn_conv(h, W, r, b, plan, MODE_ALL, -1, R, activation="relu")
        else:
            h = torch.relu(rgcn_conv(h, W, r, b, plan, MODE_ALL, -1, R))
    h.backward(dout.double() if dev == "cpu" else dout.to(dev))
    return h.detach().double().cpu(), {k: v.grad.detach().double().cpu() for k, v in p.items() if v.grad is not None}


for layers in (1, 2, 3):
    ref_o, ref_g = run("cpu", False, layers)
    for fused in (True, False):
        o, gr = run("cuda", fused, layers)
        msg = [f"out {float((o - ref_o).abs().max() / ref_o.abs().max()):.1e}"]
        for k in ref_g:
            msg.append(f"{k} {float((gr[k] - ref_g[k]).abs().max() / ref_g[k].abs().max()):.1e}")
        print(f"layers {layers} fused {fused}: " + "  ".join(msg), flush=True)
