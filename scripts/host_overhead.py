#!/usr/bin/env python3
"""Host-side overhead of the eager forward: 3-layer step with / without kernel timing, the
Python path alone per layer, and the HIP-graph replay of the same step."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402
from mpgnn_amd import _lib, data  # noqa: E402

g = data.fb15k237_graph(feat_dim=128, seed=0)
dev = torch.device("cuda", 0)
net = mpgnn_amd.Net(128, 128, g.num_relations, 128, 2, 3).to(dev)
x, ei, et = g.x.to(dev), g.edge_index.to(dev), g.edge_type.to(dev)
convs = [net.conv1, net.conv2, net.conv2]


def step():
    h = x
    for conv in convs:
        h = torch.relu(conv(h, ei, et))
    return h


def timeit(fn, n=100):
    with torch.no_grad():
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6


res = {"eager_us": timeit(step)}
_lib.lib.mpgnn_timing_enable(1)
res["eager_timed_all_us"] = timeit(step)
_lib.lib.mpgnn_timing_reset()
_lib.lib.mpgnn_set_option(3, 1)  # seg_fwd only
res["eager_timed_segfwd_us"] = timeit(step)
_lib.lib.mpgnn_set_option(3, -1)
_lib.lib.mpgnn_timing_enable(0)
_lib.lib.mpgnn_timing_reset()
# host-only: the Python + ctypes path without waiting for the GPU (launch rate)
with torch.no_grad():
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(100):
        step()
    host = (time.perf_counter() - t) / 100 * 1e6
    torch.cuda.synchronize()
res["host_issue_us_per_step"] = host
plan = mpgnn_amd.get_plan(ei, et, g.num_nodes)
h = torch.randn(g.num_nodes, 128, device=dev)


def relu_only():
    y = h
    for _ in range(3):
        y = torch.relu(y)
    return y


res["relu_x3_us"] = timeit(relu_only)
print(json.dumps({k: round(v, 1) for k, v in res.items()}))
