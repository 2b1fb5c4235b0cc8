"""A/B of MPGNN_OPT_FLAT_WG_PER_CU (persistent gather-sum grid) on the C3 forward / backward
layer: per-kernel HIP-event times, outputs compared bit for bit across settings."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402
from mpgnn_amd import _lib, data  # noqa: E402

g = data.fb15k237_graph(feat_dim=128, seed=0, recipe="survey")
x = g.x.cuda().requires_grad_(True)
ei, et = g.edge_index.cuda(), g.edge_type.cuda()
torch.manual_seed(0)
conv = mpgnn_amd.RGCNConv(128, 128, g.num_relations, flow="target_to_source").cuda()
gout = torch.randn(g.num_nodes, 128, device="cuda")
ref = None
for wg in [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,2,4,8,16").split(",")]:
    _lib.set_option(26, wg)
    for _ in range(3):
        x.grad = None
        o = conv(x, ei, et, activation="relu")
        o.backward(gout)
    torch.cuda.synchronize()
    _lib.lib.mpgnn_timing_reset()
    _lib.lib.mpgnn_timing_enable(1)
    it = 20
    for _ in range(it):
        x.grad = None
        o = conv(x, ei, et, activation="relu")
        o.backward(gout)
    torch.cuda.synchronize()
    _lib.lib.mpgnn_timing_enable(0)
    k = {}
    for kind in ("mean", "seg_fwd", "row_fwd", "seg_dgrad", "row_dx", "outer", "reduce", "final"):
        ms, n = _lib.kernel_timing(kind)
        if n:
            k[kind] = round(ms * 1e3 / it, 2)
    res = (o.detach().clone(), x.grad.clone())
    same = None if ref is None else (torch.equal(res[0], ref[0]) and torch.equal(res[1], ref[1]))
    ref = ref or res
    print("wg_per_cu", wg, json.dumps(k), "bit-identical to the first setting:", same, flush=True)
