#!/usr/bin/env python3
"""Minimal driver for rocprofv3: N forward (and optionally backward) passes of one RGCN layer
(mode ALL) on a named workload. Used by scripts/pmc.sh; prints nothing on success."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402
from mpgnn_amd import data  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="fb15k237")
ap.add_argument("--feat", type=int, default=128)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--backward", action="store_true")
args = ap.parse_args()
g = data.config_graph(args.config)
x = torch.rand(g.num_nodes, args.feat, device="cuda", requires_grad=args.backward)
ei, et = g.edge_index.cuda(), g.edge_type.cuda()
torch.manual_seed(0)
conv = mpgnn_amd.RGCNConv(args.feat, args.feat, g.num_relations, flow="target_to_source").cuda()
for _ in range(args.iters):
    if args.backward:
        o = conv(x, ei, et)
        o.backward(torch.ones_like(o))
    else:
        with torch.no_grad():
            conv(x, ei, et)
torch.cuda.synchronize()
