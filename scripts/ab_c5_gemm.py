"""A/B of the C5 (F = 256) transform GEMM variants on one mode-ALL layer: fp32 MFMA
(MPGNN_OPT_GEMM_BF3=0) vs the split-K bf16 kernel (rel_gemm_bf3w_kernel); forward and
backward kernel times from the library's HIP-event timing, outputs compared across variants."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402
from mpgnn_amd import _lib, data  # noqa: E402

g = data.config_graph(sys.argv[1] if len(sys.argv) > 1 else "C5")
F = 256
x = torch.rand(g.num_nodes, F, generator=torch.Generator().manual_seed(1)).cuda().requires_grad_(True)
ei, et = g.edge_index.cuda(), g.edge_type.cuda()
torch.manual_seed(0)
conv = mpgnn_amd.RGCNConv(F, F, g.num_relations, flow="target_to_source").cuda()
gout = torch.randn(g.num_nodes, F, device="cuda")
res, outs = {}, {}
for name, bf3 in (("fp32", 0), ("bf3w", 1)):
    _lib.set_option(24, bf3)
    for _ in range(2):
        x.grad = None
        o = conv(x, ei, et)
        o.backward(gout)
    torch.cuda.synchronize()
    _lib.lib.mpgnn_timing_reset()
    _lib.lib.mpgnn_timing_enable(1)
    iters = 3
    for _ in range(iters):
        x.grad = None
        o = conv(x, ei, et)
        o.backward(gout)
    torch.cuda.synchronize()
    _lib.lib.mpgnn_timing_enable(0)
    k = {}
    for kind in ("mean", "seg_fwd", "row_fwd", "seg_dgrad", "row_dx", "outer", "reduce"):
        ms, n = _lib.kernel_timing(kind)
        if n:
            k[kind] = round(ms / iters, 3)
    res[name] = k
    outs[name] = (o.detach().clone(), x.grad.detach().clone())
    print(name, json.dumps(k), flush=True)
ref_o, ref_g = outs["fp32"]
for name, (o, gx) in outs.items():
    eo = float(((o - ref_o).norm() / ref_o.norm()))
    eg = float(((gx - ref_g).norm() / ref_g.norm()))
    print(name, "normwise vs fp32: out %.2e dx %.2e" % (eo, eg), flush=True)
