#!/usr/bin/env python3
"""Time mpgnn_adam_step against torch's fused Adam pair on Net(128,128,237,128,2,3)'s parameters
(C3, 7.8 M floats): median of 200 steps each, HIP events. usage: python scripts/adam_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402
from mpgnn_amd import main  # noqa: E402

dev = torch.device("cuda", 0)
out = {}
for kind in ("torch", "hip"):
    net = mpgnn_amd.Net(128, 128, 237, 128, 2, 3).to(dev)
    os.environ["MPGNN_HIP_ADAM"] = "1" if kind == "hip" else "0"
    main._HIP_ADAM = kind == "hip"
    opt = main._adam(net)
    for p in net.parameters():
        p.grad = torch.randn_like(p)
    for _ in range(20):
        opt.step()
    torch.cuda.synchronize()
    ts = []
    for _ in range(200):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        opt.step()
        b.record()
        ts.append((a, b))
    torch.cuda.synchronize()
    v = sorted(x.elapsed_time(y) * 1e3 for x, y in ts)
    out[kind] = {"median_us": round(v[len(v) // 2], 2), "min_us": round(v[0], 2)}
n = sum(p.numel() for p in net.parameters())
out["params"] = n
out["hbm_bytes"] = n * 28
out["hip_TBps"] = round(n * 28 / out["hip"]["median_us"] / 1e6, 2)
out["blocks_env"] = os.environ.get("MPGNN_ADAM_BLOCKS")
print(json.dumps(out))
