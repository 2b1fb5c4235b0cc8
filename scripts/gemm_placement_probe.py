"""Does the C3 forward GEMM's time depend on what ran before it? The same no-grad RGCN layer
forward (means, GEMM, combine; kernel times from the library's per-kind HIP events) after:
  idle      - the previous forward only
  write     - a 96 MB fill (lines left dirty in L2 / MALL, like Adam's parameter writes)
  read      - a 96 MB sum (clean lines, the same footprint)
  mfma      - a 4096^3 fp32 matmul (a compute-bound phase: clock / power state)
usage: python scripts/gemm_placement_probe.py [--iters 40] [--rounds 3]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mpgnn_amd  # noqa: E402
from mpgnn_amd import _lib, data  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=40)
ap.add_argument("--rounds", type=int, default=3)
a = ap.parse_args()
g = data.config_graph("fb15k237")
dev = torch.device("cuda", 0)
F = 128
torch.manual_seed(10)
conv = mpgnn_amd.RGCNConv(F, F, g.num_relations, flow="target_to_source").to(dev)
x = g.x[:, :F].contiguous().to(dev)
ei, et = g.edge_index.to(dev), g.edge_type.to(dev)
big = torch.empty(24 * 1024 * 1024, device=dev)  # 96 MB
ma = torch.randn(4096, 4096, device=dev)
pre = {"idle": lambda: None, "write": lambda: big.fill_(1.0), "read": lambda: big.sum(),
       "mfma": lambda: ma @ ma}
res = {k: [] for k in pre}
with torch.no_grad():
    for _ in range(5):
        conv(x, ei, et, activation="relu")
        for f in pre.values():
            f()
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for k, f in pre.items():
            _lib.lib.mpgnn_timing_reset()
            for _ in range(a.iters):
                f()
                _lib.lib.mpgnn_timing_enable(1)
                conv(x, ei, et, activation="relu")
                _lib.lib.mpgnn_timing_enable(0)
            torch.cuda.synchronize()
            rec = {}
            for kind in _lib.KERNEL_KINDS:
                ms, n = _lib.kernel_timing(kind)
                if n:
                    rec[kind] = round(ms * 1e3 / a.iters, 2)
            res[k].append(rec)
print(json.dumps(res), flush=True)
