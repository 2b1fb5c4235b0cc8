"""A/B of one library option on one RGCN layer (forward + training backward) in ONE process:
bit-equality of the outputs and gradients between the settings, then per-kernel-kind µs of
each setting, alternated --rounds times.
usage: python scripts/ab_opt_layer.py --opt 30 --values 0,1 [--workload fb15k237] [--iters 30]"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mpgnn_amd  # noqa: E402
from mpgnn_amd import _lib, data  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="fb15k237")
ap.add_argument("--opt", type=int, required=True)
ap.add_argument("--values", default="0,1")
ap.add_argument("--iters", type=int, default=30)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--feat", type=int, default=None)
a = ap.parse_args()
vals = [int(v) for v in a.values.split(",")]
default = _lib.get_option(a.opt)
g = data.config_graph(a.workload)
dev = torch.device("cuda", 0)
F = a.feat or g.x.shape[1]
torch.manual_seed(10)
conv = mpgnn_amd.RGCNConv(F, F, g.num_relations, flow="target_to_source").to(dev)
x = (g.x[:, :F] if g.x.shape[1] >= F else torch.rand(g.x.shape[0], F)).to(dev).contiguous()
ei, et = g.edge_index.to(dev), g.edge_type.to(dev)
gout = torch.randn(x.shape[0], F, device=dev)


def run(train):
    if train:
        xg = x.clone().requires_grad_(True)
        out = conv(xg, ei, et, activation="relu")
        out.backward(gout)
        return out.detach(), xg.grad, conv.weight.grad.clone(), conv.root.grad.clone(), conv.bias.grad.clone()
    with torch.no_grad():
        return (conv(x, ei, et, activation="relu"),)


res = {"workload": a.workload, "opt": a.opt, "values": vals, "default": default}
outs = {}
plan = mpgnn_amd.get_plan(ei, et, x.shape[0])  # the layer's cached plan: kernel switches are per plan


def setopt(v):
    _lib.set_option(a.opt, v)
    try:
        plan.set_option(a.opt, v)
    except ValueError:  # a process-wide option
        pass


for v in vals:
    setopt(v)
    conv.zero_grad(set_to_none=True)
    outs[v] = run(True)
    torch.cuda.synchronize()
names = ["out", "grad_x", "grad_weight", "grad_root", "grad_bias"]
res["bit_equal"] = {n: all(torch.equal(outs[vals[0]][k], outs[v][k]) for v in vals[1:]) for k, n in enumerate(names)}
res["max_abs_diff"] = {n: max(float((outs[vals[0]][k] - outs[v][k]).abs().max()) for v in vals[1:])
                       for k, n in enumerate(names)}
timing = {v: [] for v in vals}
for r in range(a.rounds):
    for v in vals:
        setopt(v)
        for train in (False, True):
            for _ in range(3):
                conv.zero_grad(set_to_none=True)
                run(train)
        torch.cuda.synchronize()
        rec = {}
        for train in (False, True):
            t0 = time.perf_counter()
            for _ in range(a.iters):
                conv.zero_grad(set_to_none=True)
                run(train)
            torch.cuda.synchronize()
            rec["wall_fwd_us" if not train else "wall_train_us"] = round((time.perf_counter() - t0) / a.iters * 1e6, 1)
        _lib.lib.mpgnn_timing_reset()
        _lib.lib.mpgnn_timing_enable(1)
        for _ in range(a.iters):
            conv.zero_grad(set_to_none=True)
            run(True)
        torch.cuda.synchronize()
        _lib.lib.mpgnn_timing_enable(0)
        for kind in _lib.KERNEL_KINDS:
            ms, n = _lib.kernel_timing(kind)
            if n:
                rec[kind] = round(ms * 1e3 / a.iters, 2)
        timing[v].append(rec)
res["timing"] = {str(v): timing[v] for v in vals}
setopt(default)
print(json.dumps(res), flush=True)
