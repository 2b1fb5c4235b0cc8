#!/usr/bin/env python3
"""A/B backward options on the bench's train step (3-layer RGCN forward + backward, FB15K
shape): ms per fwd+bwd and per-kernel µs per launch (C-ABI timing hook), and the largest
gradient difference against the first setting. Each argument is option=value[,option=value]
(20 = MPGNN_OPT_CHUNK_ROWS, 21 = MPGNN_OPT_OUTER_ROOT_FIRST, 22 = MPGNN_OPT_OUTER_SLICE,
23 = MPGNN_OPT_DGRAD_IDX_AHEAD); the plan is rebuilt per setting
(relation chunks are laid out at plan build); every setting starts from the defaults.

  python scripts/chunk_ab.py 20=128 20=256 20=256,21=0
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402
from mpgnn_amd import _lib, data  # noqa: E402
from mpgnn_amd.plan import plan_cache  # noqa: E402

g = data.config_graph(sys.argv[sys.argv.index("--config") + 1] if "--config" in sys.argv else "fb15k237")
specs = [a for a in sys.argv[1:] if "=" in a] or ["20=128", "20=256"]
DEFAULTS = {20: 192, 21: 1, 22: 16, 23: 1}
torch.manual_seed(10)
net = mpgnn_amd.Net(128, 128, g.num_relations, 128, 2, 3).cuda()
x, ei, et = g.x.cuda(), g.edge_index.cuda(), g.edge_type.cuda()
convs = [net.conv1, net.conv2, net.conv2]


def step():
    h = x
    for conv in convs:
        h = conv(h, ei, et, activation="relu")
    net.zero_grad(set_to_none=False)
    h.sum().backward()


ref = None
for v in specs:
    for k, d in DEFAULTS.items():
        _lib.check(_lib.lib.mpgnn_set_option(k, d), "mpgnn_set_option")
    for kv in v.split(","):
        k, val = (int(t) for t in kv.split("="))
        _lib.check(_lib.lib.mpgnn_set_option(k, val), "mpgnn_set_option")
    plan_cache.clear()  # relation chunks are laid out at plan build
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    grads = torch.cat([p.grad.flatten() for p in net.parameters() if p.grad is not None]).clone()
    err = 0.0 if ref is None else float(((grads - ref).abs() / ref.abs().clamp_min(1e-3)).max())
    ref = grads if ref is None else ref
    t0 = time.perf_counter()
    for _ in range(50):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / 50
    _lib.lib.mpgnn_timing_reset()
    _lib.lib.mpgnn_timing_enable(1)
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    _lib.lib.mpgnn_timing_enable(0)
    kern = {}
    for k in _lib.KERNEL_KINDS:
        t, n = _lib.kernel_timing(k)
        if n:
            kern[k] = [round(t / n * 1e3, 2), round(n / 10, 1)]
    print(json.dumps({"opts": v, "ms_fwd_bwd": round(ms, 4), "max_rel_grad_diff_vs_first": err,
                      "us_per_launch_and_launches_per_step": kern}), flush=True)
for k, d in DEFAULTS.items():
    _lib.lib.mpgnn_set_option(k, d)
