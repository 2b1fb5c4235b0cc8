"""mpgnn_rgcn_bwd_accumulate and Net's shared-conv2 gradient stash (functional.GradStash).

The reference's Net applies the SAME conv2 for layers 1..L-1 (model.py:144-146); autograd sums
the per-use parameter gradients (grad of the later use first, then + the earlier one). The
drop-in sums them inside the backward kernels: the accumulating entry point must give exactly
dst + (what mpgnn_rgcn_bwd gives), element for element, and the Net's gradients must be
bit-identical to the same stack run use by use through autograd's accumulation.
"""
import ctypes

import pytest
import torch

import mpgnn_amd
from mpgnn_amd import _lib, data
from mpgnn_amd.functional import MODE_ALL, _workspace, rgcn_conv
from mpgnn_amd.plan import get_plan

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _graph(kind):
    if kind == "c3":
        return data.fb15k237_graph(feat_dim=128, seed=0)
    return data.synthetic_graph(700, 9, 14, feat_dim=128, seed=4)


def _bwd(plan, x, w, root, h_save, gout, bufs, acc):
    N, F = x.shape
    ws = _workspace(plan.workspace_bytes(MODE_ALL, -1, w.shape[0], F, F, 0, N), x.device)
    gx = torch.empty_like(x)
    fn = _lib.lib.mpgnn_rgcn_bwd_accumulate if acc else _lib.lib.mpgnn_rgcn_bwd
    st = fn(plan.handle, MODE_ALL, -1, w.shape[0], x.data_ptr(), F, w.data_ptr(), root.data_ptr(), F,
            None if h_save is None else h_save.data_ptr(), gout.data_ptr(), 0, N, gx.data_ptr(),
            bufs[0].data_ptr(), bufs[1].data_ptr(), bufs[2].data_ptr(), ws.data_ptr(),
            torch.cuda.current_stream().cuda_stream)
    return st, gx


@pytest.mark.parametrize("kind", ["small", "c3"])
def test_bwd_accumulate_is_dst_plus_bwd(kind):
    g = _graph(kind)
    gen = torch.Generator().manual_seed(5)
    R = g.num_relations
    x = g.x.to(DEV)
    w = (torch.randn(R, 128, 128, generator=gen) * 0.05).to(DEV)
    root = (torch.randn(128, 128, generator=gen) * 0.05).to(DEV)
    gout = torch.randn(g.num_nodes, 128, generator=gen).to(DEV)
    plan = get_plan(g.edge_index.to(DEV), g.edge_type.to(DEV), g.num_nodes, device=x.device).to_device(x.device)
    fresh = (torch.empty(R, 128, 128, device=DEV), torch.empty(128, 128, device=DEV), torch.empty(128, device=DEV))
    st, gx0 = _bwd(plan, x, w, root, None, gout, fresh, acc=False)
    _lib.check(st, "mpgnn_rgcn_bwd")
    prev = (torch.randn(R, 128, 128, generator=gen).to(DEV), torch.randn(128, 128, generator=gen).to(DEV),
            torch.randn(128, generator=gen).to(DEV))
    acc = tuple(p.clone() for p in prev)
    st, gx1 = _bwd(plan, x, w, root, None, gout, acc, acc=True)
    _lib.check(st, "mpgnn_rgcn_bwd_accumulate")
    torch.cuda.synchronize()
    assert torch.equal(gx1, gx0)
    for a, p, f, nm in zip(acc, prev, fresh, ("dW", "droot", "dbias")):
        assert torch.equal(a, p + f), nm


def test_bwd_accumulate_unsupported_launches_nothing():
    g = _graph("small")
    x = g.x[:, :64].contiguous().to(DEV)  # F = 64: not the accumulating path
    R = g.num_relations
    w = torch.randn(R, 64, 64, device=DEV)
    root = torch.randn(64, 64, device=DEV)
    gout = torch.randn(g.num_nodes, 64, device=DEV)
    plan = get_plan(g.edge_index.to(DEV), g.edge_type.to(DEV), g.num_nodes, device=x.device).to_device(x.device)
    bufs = (torch.full((R, 64, 64), 3.0, device=DEV), torch.full((64, 64), 3.0, device=DEV),
            torch.full((64,), 3.0, device=DEV))
    st, _ = _bwd(plan, x, w, root, None, gout, bufs, acc=True)
    assert st == _lib.MPGNN_ERR_UNSUPPORTED
    torch.cuda.synchronize()
    assert all(bool((b == 3.0).all()) for b in bufs)


@pytest.mark.parametrize("kind,layers", [("small", 3), ("small", 5), ("c3", 3)])
def test_net_shared_conv2_grads_bit_identical_to_autograd_accumulation(kind, layers):
    g = _graph(kind)
    torch.manual_seed(30)
    net = mpgnn_amd.Net(128, 128, g.num_relations, 128, 2, layers).to(DEV)
    x, ei, et = g.x.to(DEV), g.edge_index.to(DEV), g.edge_type.to(DEV)
    y = torch.randint(0, 2, (g.num_nodes,), generator=torch.Generator().manual_seed(1)).to(DEV)

    def loss_of(out):
        return torch.nn.functional.nll_loss(out, y)

    out = net(x, ei, et)  # the stash path (layers >= 3)
    loss_of(out).backward()
    got = {n: p.grad.clone() for n, p in net.named_parameters()}
    net.zero_grad(set_to_none=True)
    # the same stack use by use without the stash: autograd sums conv2's gradients
    h = x
    for li in range(layers):
        conv = net.conv1 if li == 0 else net.conv2
        h = conv(h, ei, et, activation="relu")
    loss_of(mpgnn_amd.model.head_log_softmax(net.LinearLayer, h)).backward()  # Net's head, as Net runs it
    for n, p in net.named_parameters():
        assert torch.equal(got[n], p.grad), n
