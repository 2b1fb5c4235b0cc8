#!/usr/bin/env python3
"""Which CPU ops issue the epoch's non-layer GPU work (memcpy, fill, add, library GEMMs)?

torch.profiler over 5 eager epochs of the bench's Net (mode ALL) and MPNetm (mode SINGLE) on
the C3 graph; prints, per CPU op, the GPU kernels it launched (count per epoch, µs per epoch).
Then times the MPNetm.fc1 weight gradient (K = N GEMM, 128 x 128 out) as: one mm, the
split-K bmm at several slice lengths, with its error against float64."""
import json
import os
import sys
import time
from collections import defaultdict

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402
from mpgnn_amd import data  # noqa: E402

dev = torch.device("cuda", 0)
g = data.fb15k237_graph(feat_dim=128, seed=0)
x, ei, et = g.x.to(dev), g.edge_index.to(dev), g.edge_type.to(dev)
y = torch.randint(0, 2, (g.num_nodes,), generator=torch.Generator().manual_seed(0)).to(dev)
train_idx = torch.arange(0, g.num_nodes, 3, device=dev)
train_y = y[train_idx]
rel_counts = torch.bincount(g.edge_type, minlength=g.num_relations)
metapath = [int(v) for v in torch.argsort(rel_counts, descending=True, stable=True)[:3]]
EP = 5


def run(model, name):
    opt = mpgnn_amd.main._adam(model)

    def epoch():
        model.train()
        opt.zero_grad()
        out = model(x, ei, et)
        loss = torch.nn.functional.nll_loss(out.index_select(0, train_idx), train_y)
        loss.backward()
        opt.step()
        model.eval()
        with torch.no_grad():
            model(x, ei, et)

    for _ in range(3):
        epoch()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        for _ in range(EP):
            epoch()
        torch.cuda.synchronize()
    # map each GPU kernel to its launching CPU op through correlation / parent chain
    evs = prof.events()
    per = defaultdict(lambda: [0, 0.0])
    for e in evs:
        if e.device_type != torch.autograd.DeviceType.CUDA:
            continue
        p = e.cpu_parent
        chain = []
        while p is not None and len(chain) < 4:
            chain.append(p.name)
            p = p.cpu_parent
        key = (e.name[:70], " <- ".join(chain[:3]))
        per[key][0] += 1
        per[key][1] += e.device_time_total if hasattr(e, "device_time_total") else e.cuda_time_total
    rows = sorted(per.items(), key=lambda kv: -kv[1][1])
    print(f"== {name}: GPU kernels per epoch (count, us) by launching CPU op")
    for (k, chain), (n, t) in rows[:40]:
        print(f"{n / EP:5.1f} {t / EP:8.1f}  {k}  <=  {chain}")
    sys.stdout.flush()


run(mpgnn_amd.Net(128, 128, g.num_relations, 128, 2, 3).to(dev), "Net mode ALL")
run(mpgnn_amd.MPNetm(128, 128, g.num_relations, 128, 2, 1, [metapath]).to(dev), "MPNetm mode SINGLE")

# ---- fc1 weight gradient variants ---------------------------------------------------------
n = g.num_nodes
torch.manual_seed(0)
xa = torch.randn(n, 128, device=dev)
ga = torch.randn(n, 128, device=dev) * 1e-3
truth = ga.double().t().mm(xa.double())


def t_of(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


def splitk(rows):
    slices = (n + rows - 1) // rows
    pad = rows * slices - n
    gp = torch.nn.functional.pad(ga, (0, 0, 0, pad)) if pad else ga
    xp = torch.nn.functional.pad(xa, (0, 0, 0, pad)) if pad else xa
    return torch.bmm(gp.view(slices, rows, -1).transpose(1, 2), xp.view(slices, rows, -1)).sum(0)


res = {}
for name, fn in [("mm", lambda: ga.t().mm(xa))] + [(f"bmm_rows{r}", (lambda r=r: splitk(r))) for r in (1024, 512, 256, 128, 64)]:
    out = fn()
    err = float((out.double() - truth).abs().max() / truth.abs().max())
    res[name] = {"us": round(t_of(fn), 2), "err_rel_max": err}
print(json.dumps({"fc1_wgrad": res}))
