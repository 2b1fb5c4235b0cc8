"""Host-side cost of one eager epoch (bench.py's kernel epoch: train fwd + NLL + bwd + Adam + a
no-grad validation forward) of MPNetm mode SINGLE (C3) or Net mode ALL: wall time per epoch,
torch ops and kernel launches per epoch, and the ops with the most CPU time (torch.profiler).
usage: python scripts/epoch_host_profile.py [--workload fb15k237] [--mode single|all] [--epochs 20]"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mpgnn_amd  # noqa: E402
from mpgnn_amd import data  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="fb15k237")
ap.add_argument("--mode", default="single", choices=["single", "all"])
ap.add_argument("--epochs", type=int, default=20)
ap.add_argument("--top", type=int, default=40)
ap.add_argument("--ab-adam", action="store_true", help="alternate torch's fused Adam and main.LeanAdam, 3 rounds")
ap.add_argument("--ab-heads", action="store_true", help="alternate the Linear heads on the C ABI and on torch, 3 rounds")
ap.add_argument("--ab-small-fwd", action="store_true",
                help="alternate the narrow heads' (O <= 8) forward on the C ABI and on torch, 3 rounds")
ap.add_argument("--ab-loss", action="store_true", help="alternate metrics.nll_loss_rows and torch's ops, 3 rounds")
a = ap.parse_args()

dev = torch.device("cuda", 0)
g = data.config_graph(a.workload)
F = 128
x, ei, et = g.x[:, :F].contiguous().to(dev), g.edge_index.to(dev), g.edge_type.to(dev)
torch.manual_seed(10)
if a.mode == "single":
    rel_counts = torch.bincount(g.edge_type, minlength=g.num_relations)
    metapath = [int(v) for v in torch.argsort(rel_counts, descending=True, stable=True)[:3]]
    model = mpgnn_amd.MPNetm(F, F, g.num_relations, F, 2, 1, [metapath]).to(dev)

    def fwd():
        return model(x, ei, et)
else:
    model = mpgnn_amd.Net(F, F, g.num_relations, F, 2, 3).to(dev)

    def fwd():
        return model(x, ei, et)
opt = mpgnn_amd.main._adam(model)
y = torch.randint(0, 2, (g.num_nodes,), generator=torch.Generator().manual_seed(0)).to(dev)
train_idx = torch.arange(0, g.num_nodes, 3, device=dev)
train_y = y[train_idx]


def torch_loss(out, idx, y):
    return torch.nn.functional.nll_loss(out.index_select(0, idx), y)


LOSS = [mpgnn_amd.metrics.nll_loss_rows]


def epoch():
    model.train()
    opt.zero_grad()
    out = fwd()
    loss = LOSS[0](out, train_idx, train_y)
    loss.backward()
    opt.step()
    model.eval()
    with torch.no_grad():
        fwd()


if a.ab_loss:
    modes = {"fused": mpgnn_amd.metrics.nll_loss_rows, "torch": torch_loss}
    rec = {k: [] for k in modes}
    for _ in range(3):
        for k, f in modes.items():
            LOSS[0] = f
            for _ in range(5):
                epoch()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.epochs):
                epoch()
            torch.cuda.synchronize()
            rec[k].append(round((time.perf_counter() - t0) * 1e3 / a.epochs, 4))
    print(json.dumps({"workload": a.workload, "mode": a.mode, "epoch_wall_ms": rec}), flush=True)
    sys.exit(0)
if a.ab_heads or a.ab_small_fwd:
    import mpgnn_amd.model as M
    fwd0, dgrad0 = M._head_fwd, M._head_dgrad
    modes = {"abi": (fwd0, dgrad0), "torch": (lambda *_: None, lambda *_: None)}
    if a.ab_small_fwd:
        modes["torch"] = (lambda x, w, b, r: None if w.shape[0] <= 8 else fwd0(x, w, b, r), dgrad0)
    opt = mpgnn_amd.main.LeanAdam(list(model.parameters()), lr=0.01, weight_decay=0.0005, fused=True)
    rec = {k: [] for k in modes}
    for _ in range(3):
        for k, (f1, f2) in modes.items():
            M._head_fwd, M._head_dgrad = f1, f2
            for _ in range(5):
                epoch()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.epochs):
                epoch()
            torch.cuda.synchronize()
            rec[k].append(round((time.perf_counter() - t0) * 1e3 / a.epochs, 4))
    M._head_fwd, M._head_dgrad = fwd0, dgrad0
    print(json.dumps({"workload": a.workload, "mode": a.mode, "epoch_wall_ms": rec}), flush=True)
    sys.exit(0)
if a.ab_adam:
    params = list(model.parameters())
    opts = {"torch": torch.optim.Adam(params, lr=0.01, weight_decay=0.0005, fused=True),
            "lean": mpgnn_amd.main.LeanAdam(params, lr=0.01, weight_decay=0.0005, fused=True)}
    rec = {k: [] for k in opts}
    for _ in range(3):
        for k, o in opts.items():
            opt = o
            for _ in range(5):
                epoch()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.epochs):
                epoch()
            torch.cuda.synchronize()
            rec[k].append(round((time.perf_counter() - t0) * 1e3 / a.epochs, 4))
    print(json.dumps({"workload": a.workload, "mode": a.mode, "epoch_wall_ms": rec}), flush=True)
    sys.exit(0)
for _ in range(5):
    epoch()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.epochs):
    epoch()
torch.cuda.synchronize()
wall_ms = (time.perf_counter() - t0) * 1e3 / a.epochs
# host issue time alone: the same epochs with the GPU never waited on (enqueue rate)
t0 = time.perf_counter()
for _ in range(a.epochs):
    epoch()
host_ms = (time.perf_counter() - t0) * 1e3 / a.epochs
torch.cuda.synchronize()

from torch.profiler import ProfilerActivity, profile  # noqa: E402
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    for _ in range(5):
        epoch()
    torch.cuda.synchronize()
ka = prof.key_averages()
ops = sorted(((e.key, e.count / 5, e.self_cpu_time_total / 5) for e in ka if e.self_cpu_time_total > 0),
             key=lambda t: -t[2])
kernels = [e for e in prof.events() if getattr(e, "device_type", None) is not None and
           str(e.device_type).endswith("CUDA")]
res = {"workload": a.workload, "mode": a.mode, "epoch_wall_ms": round(wall_ms, 3),
       "epoch_host_issue_ms": round(host_ms, 3),
       "gpu_kernels_per_epoch": len(kernels) / 5,
       "top_self_cpu_us": [(k, c, round(t, 1)) for k, c, t in ops[:a.top]]}
print(json.dumps(res), flush=True)
