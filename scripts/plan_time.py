#!/usr/bin/env python3
"""Plan build time for a named workload: host builder (csrc/plan.cpp, MPGNN_PLAN_TIMING=1 prints
its phases) and, with a GPU, the device builder (csrc/plan_device.hip) from CUDA edge tensors,
plus the digest check that both give the same tables. Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mpgnn_amd  # noqa: E402
from mpgnn_amd import data  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C5"
g = data.config_graph(name)
res = {"workload": name, "edges": int(g.edge_index.shape[1]), "nodes": g.num_nodes}
t = time.time()
ph = mpgnn_amd.GraphPlan(g.edge_index, g.edge_type, g.num_nodes, build="host")
res["host_build_s"] = round(time.time() - t, 3)
if torch.cuda.is_available():
    dev = torch.device("cuda:0")
    t = time.time()
    ph.to_device(dev)
    torch.cuda.synchronize()
    res["host_upload_s"] = round(time.time() - t, 3)
    ei, et = g.edge_index.to(dev), g.edge_type.to(dev)
    torch.cuda.synchronize()
    times = []
    for _ in range(3):
        t = time.time()
        pd = mpgnn_amd.GraphPlan(ei, et, g.num_nodes, build="device")
        torch.cuda.synchronize()
        times.append(round(time.time() - t, 3))
        if _ < 2:
            del pd
    res["device_build_s"] = times
    t = time.time()
    res["digest_equal"] = pd.digest() == ph.digest()
    res["digest_s"] = round(time.time() - t, 3)
print(json.dumps(res), flush=True)
