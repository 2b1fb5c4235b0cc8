#!/usr/bin/env python3
"""MPGNN_OPT_GEMM_SWITCH_COST (29) on the C3 layer: forward / backward outputs bit-identical
between the equal item split and the cost-balanced ranges (the per-item arithmetic is the same),
and the per-kernel GEMM times (HIP events, library timing) for each setting, alternated."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402
from mpgnn_amd import _lib, data  # noqa: E402
from mpgnn_amd.functional import rgcn_conv  # noqa: E402

g = data.fb15k237_graph(feat_dim=128, seed=0, recipe="survey")
dev = "cuda"
N, R = g.num_nodes, g.num_relations
plan = mpgnn_amd.GraphPlan(g.edge_index.to(dev), g.edge_type.to(dev), N)
gen = torch.Generator().manual_seed(3)
x0 = g.x.to(dev)
W = ((torch.rand((R, 128, 128), generator=gen) - 0.5) * 0.2).to(dev)
root = ((torch.rand((128, 128), generator=gen) - 0.5) * 0.2).to(dev)
bias = (torch.rand(128, generator=gen) - 0.5).to(dev)
gout = torch.randn(N, 128, generator=gen).to(dev)
OPT = int(os.environ.get("AB_OPT", "29"))  # option A/B'd (29: the switch cost)
costs = [int(v) for v in sys.argv[1:]] or [0, 0, 50, 100]
ref = None
for rep in range(3):
    for c in costs:
        _lib.set_option(OPT, c)
        x = x0.clone().requires_grad_(True)
        Wg, rg, bg = (t.clone().requires_grad_(True) for t in (W, root, bias))
        out = rgcn_conv(x, Wg, rg, bg, plan, 1, num_relations=R)
        out.backward(gout)
        torch.cuda.synchronize()
        got = [t.detach().clone() for t in (out, x.grad, Wg.grad, rg.grad, bg.grad)]
        if ref is None:
            ref = got
        else:
            names = ["out", "dx", "dW", "droot", "dbias"]
            diff = [(n, float((a - b).abs().max())) for n, a, b in zip(names, got, ref) if not torch.equal(a, b)]
            if diff:
                print(f"cost {c}: differs from the first run: {diff}", flush=True)
        _lib.lib.mpgnn_timing_reset()
        _lib.lib.mpgnn_timing_enable(1)
        for _ in range(20):
            out = rgcn_conv(x, Wg, rg, bg, plan, 1, num_relations=R)
            out.backward(gout)  # (accumulates into the leaves; the checked copies were taken above)
        torch.cuda.synchronize()
        _lib.lib.mpgnn_timing_enable(0)
        res = {}
        for k in ("seg_fwd", "seg_dgrad"):
            ms, n = _lib.kernel_timing(k)
            res[k] = round(ms * 1e3 / max(n, 1), 2)
        print(f"option {OPT}={c}: {res}", flush=True)
_lib.set_option(29, 250)
print("done")
