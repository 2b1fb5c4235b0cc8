"""Diagnostic: Net layer-by-layer activations and activation gradients (GPU vs float64)."""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mpgnn_amd  # noqa: E402
from mpgnn_amd import _lib, data  # noqa: E402
from mpgnn_amd.functional import MODE_ALL, rgcn_conv  # noqa: E402
from mpgnn_amd.plan import GraphPlan  # noqa: E402
from oracle import rgcn_oracle as orc  # noqa: E402

g = data.config_graph(sys.argv[1] if len(sys.argv) > 1 else "fb15k237")
Fdim = g.x.shape[1]
R, N = g.num_relations, g.num_nodes
torch.manual_seed(10)
net0 = mpgnn_amd.Net(Fdim, 64, R, 64, 5, 3)
sd = net0.state_dict()
gout = torch.randn(N, 5, generator=torch.Generator().manual_seed(3))
plan = GraphPlan(g.edge_index, g.edge_type, N)


def run(dev, exact=False, fused=True):
    if dev == "cuda":
        plan.set_exact_order(exact)  # the switch is per plan
    p = {k: (v.double() if dev == "cpu" else v.to(dev)).requires_grad_(True) for k, v in sd.items()}
    h = g.x.double() if dev == "cpu" else g.x.to(dev)
    acts = []
    for li in range(3):
        c = "conv1" if li == 0 else "conv2"
        W, r, b = p[c + ".weight"], p[c + ".root"], p[c + ".bias"]
        if dev == "cpu":
            h = torch.relu(orc.rgcn_forward(h, g.edge_index, g.edge_type, W, r, b))
        elif fused:
            h = rgcn_conv(h, W, r, b, plan, MODE_ALL, -1, R, activation="relu")
        else:
            h = torch.relu(rgcn_conv(h, W, r, b, plan, MODE_ALL, -1, R))
        h.retain_grad()
        acts.append(h)
    o = F.log_softmax(F.linear(h, p["LinearLayer.weight"], p["LinearLayer.bias"]), dim=1)
    o.backward(gout.double() if dev == "cpu" else gout.to(dev))
    return [a.detach().double().cpu() for a in acts], [a.grad.double().cpu() for a in acts], \
        {k: v.grad.double().cpu() for k, v in p.items()}


ra, rg, rp = run("cpu")
for exact, fused in ((False, True), (False, False), (True, True)):
    a, gr, pp = run("cuda", exact, fused)
    print(f"exact {exact} fused {fused}")
    for i in range(3):
        print(f"  h{i+1}: {float((a[i]-ra[i]).abs().max()/ra[i].abs().max()):.1e}  dh{i+1}: "
              f"{float((gr[i]-rg[i]).abs().max()/rg[i].abs().max()):.1e}  zeros-in-ref {int((ra[i]==0).sum())} "
              f"zeros-gpu {int((a[i]==0).sum())} negzero-gpu {int(((a[i]==0) & (torch.signbit(a[i]))).sum())}")
    print("  " + " ".join(f"{k} {float((pp[k]-rp[k]).abs().max()/rp[k].abs().max()):.1e}" for k in rp), flush=True)
