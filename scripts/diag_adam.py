"""Diagnostic: MPNetm step-0 root gradient of layer 2 — reduction error (vs float64 of the GPU's
own inputs) separated from upstream error (GPU inputs vs the float64 truth's)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mpgnn_amd  # noqa: E402
from mpgnn_amd import data  # noqa: E402

g = data.config_graph("C1")
torch.manual_seed(30)
net = mpgnn_amd.MPNetm(128, 64, 3, 64, 3, 2, [[1, 0], [2]]).eval().cuda()
y = torch.randint(0, 3, (1000,), generator=torch.Generator().manual_seed(1))
train_idx = torch.arange(0, 1000, 2)
conv = net.layers_list[0][1]
cap = {}
conv.register_forward_hook(lambda m, i, o: cap.update(x=i[2].detach(), out=o))
out = net(g.x.cuda(), g.edge_index.cuda(), g.edge_type.cuda())
cap["out"].retain_grad()
loss = torch.nn.functional.nll_loss(out[train_idx.cuda()], y[train_idx].cuda())
loss.backward()
x64 = cap["x"].double().cpu()
go64 = cap["out"].grad.double().cpu()
truth_from_gpu_inputs = x64.t() @ go64
gr = conv.root.grad.double().cpu()
scale = float(truth_from_gpu_inputs.abs().max())
den = truth_from_gpu_inputs.abs().clamp_min(1e-3 * scale)
print("root grad reduction error (gpu vs f64 of gpu inputs):", float(((gr - truth_from_gpu_inputs).abs() / den).max()))
f32 = (cap["x"].t() @ cap["out"].grad).double().cpu()
print("torch mm on same inputs vs f64:", float(((f32 - truth_from_gpu_inputs).abs() / den).max()))
f32c = (cap["x"].cpu().t() @ cap["out"].grad.cpu()).double()
print("cpu mm on same inputs vs f64:", float(((f32c - truth_from_gpu_inputs).abs() / den).max()))
