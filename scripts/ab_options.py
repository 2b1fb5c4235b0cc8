#!/usr/bin/env python3
"""A/B the library's tuning options on the bench step (3-layer RGCN forward, FB15K shape):
ms per step (eager, 50 steps) and per-kernel µs per launch (C-ABI timing hook) for each setting.

  python scripts/ab_options.py "7=16" "7=32" "5=0"      # option=value[,option=value...]
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402
from mpgnn_amd import _lib, data  # noqa: E402

g = data.config_graph("fb15k237")
torch.manual_seed(10)
net = mpgnn_amd.Net(128, 128, g.num_relations, 128, 2, 3).cuda()
x, ei, et = g.x.cuda(), g.edge_index.cuda(), g.edge_type.cuda()
convs = [net.conv1, net.conv2, net.conv2]


def step():
    h = x
    for conv in convs:
        h = conv(h, ei, et, activation="relu")
    return h


with torch.no_grad():
    ref = step().clone()
defaults = {}
for spec in sys.argv[1:] or ["7=16"]:
    opts = [tuple(int(v) for v in kv.split("=")) for kv in spec.split(",")]
    for k, v in opts:
        _lib.lib.mpgnn_set_option(k, v)
    with torch.no_grad():
        for _ in range(5):
            out = step()
        torch.cuda.synchronize()
        err = float((out - ref).abs().max())
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
            kern[k] = round(t / n * 1e3, 2)
    print(json.dumps({"opts": spec, "ms_per_step": round(ms, 4), "max_abs_diff_vs_first": err, "us_per_launch": kern}),
          flush=True)
    for k, v in opts:  # back to defaults
        _lib.lib.mpgnn_set_option(k, {7: 16, 5: 1, 6: 0, 4: 0, 0: 0, 8: 0, 9: 2, 10: 0, 12: 0, 14: 0, 15: 0, 16: 1, 17: 0, 18: 0}.get(k, 0))
