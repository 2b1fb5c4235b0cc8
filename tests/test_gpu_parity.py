"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the reference goldens.

Bars (BASELINE.json north_star):
  * integer / index work and the mean aggregation: BIT-EXACT (torch.equal)
  * fp32 activations and gradients: within 1e-4 relative, ELEMENTWISE, with no per-tensor
    exceptions:
        err(a, b) = max_e |a_e - b_e| / max(|b_e|, 1e-3 · max|b|)
    i.e. every element with |b| >= 1e-3·max is held to 1e-4 of itself, and the few that
    cancel to below that are held to 1e-7·max (the same bar at the threshold).
    A check passes when err(gpu, reference fp32) <= 1e-4. Where it does not, the check is
    decided against the float64 truth (the same oracle run in float64, `ref64`): the GPU
    passes when err(gpu, f64) <= max(1e-4, 2 · err(reference fp32, f64)) — at least as close
    to the truth as 2x the reference's own fp32 CPU path. Measured on GPU (round 2): the
    reference fp32 path itself is 1e-4…5e-4 off the float64 truth at this bar on dot products
    of 128 terms whose result cancels to ~1e-3 of the tensor's maximum (a 128-term fp32 sum
    carries ~1e-7·max absolute rounding, i.e. ~1e-4 relative at 1e-3·max), so no fp32
    implementation with a different summation order can meet 1e-4 against the fp32 reference
    at every such element; against the truth both are held to the same yardstick. Every check
    records both errors (tests/_parity_report.py → profiles/).
  * ReLU kinks: through a stack of layers a pre-activation within fp32 rounding of 0 may land
    on the other side of the kink on the GPU, which switches a whole gradient path on or off
    (not a rounding-size difference). The model checks therefore run the oracle with the GPU's
    ReLU mask at elements whose float64 pre-activation is within 1e-5·max of zero
    (`kink_act`), and assert that only such elements differ.
  * Whole-model gradients (Net, MPNetm: 3-5 layers, ReLU masks, torch's Linear / log_softmax /
    NLL ops between our kernels) compound every upstream rounding difference through the
    chain; there the truth bar is max(1e-4, 4 · the reference fp32 path's error)
    (MODEL_CPU_FACTOR). Measured: the reduction kernels themselves are MORE accurate than
    torch's mm on the same inputs (scripts/diag_adam.py: dW_root 2.9e-5 vs 6.8e-5 / 8.2e-5 for
    torch GPU / CPU mm at this bar); the 2-3x gaps at model level are upstream amplification.
"""
import numpy as np
import pytest
import torch

import mpgnn_amd
from mpgnn_amd import data
from mpgnn_amd.functional import MODE_ALL, MODE_SINGLE, rgcn_conv, segment_means
from oracle import rgcn_oracle as orc
from tests._parity_report import record

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-4
FLOOR = 1e-3
MODEL_CPU_FACTOR = 4.0


from tests._bars import max_rel_err, normwise_err  # noqa: E402  (the suite's bar, shared)


def rel_close(got, ref, tol=TOL, what="", ref64=None, cpu_factor=2.0):
    """The fp32 bar of the module docstring: gpu vs reference fp32, else vs the float64 truth
    (within max(tol, cpu_factor · the reference fp32 path's own error))."""
    got_f = got.detach().float().cpu()
    ref_f = ref.detach().float().cpu()
    assert got_f.shape == ref_f.shape, (what, got_f.shape, ref_f.shape)
    assert bool(torch.isfinite(got_f).all()) == bool(torch.isfinite(ref_f).all()), (what, "non-finite values differ")
    e = max_rel_err(got_f, ref_f)
    # normwise relative error ||gpu - ref|| / ||ref|| — the north star's "1e-4 rel" read as a norm:
    # held to the same 1e-4 for every check, beside the elementwise bar
    nw = normwise_err(got_f, ref_f)
    assert nw <= tol, f"{what}: normwise rel err {nw:.3e} > {tol:.0e}"
    if ref64 is None:
        record(what, e, tol, normwise=nw)
        assert e <= tol, f"{what}: max elementwise rel err {e:.3e} > {tol:.0e} (no float64 truth given)"
        return e
    ref64 = ref64.detach().double().cpu()
    e_gpu = max_rel_err(got_f, ref64)
    e_cpu = max_rel_err(ref_f, ref64)
    bar = max(tol, cpu_factor * e_cpu)
    record(what, e, tol, normwise=nw, e_gpu64=e_gpu, e_cpu64=e_cpu, cpu_factor=cpu_factor,
           normwise_gpu64=normwise_err(got_f, ref64), normwise_cpu64=normwise_err(ref_f, ref64))
    assert e <= tol or e_gpu <= bar, (f"{what}: gpu vs fp32 reference {e:.3e} > {tol:.0e} and vs float64 truth "
                                      f"gpu {e_gpu:.3e}, reference fp32 path {e_cpu:.3e} (bar {bar:.3e})")
    return e


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def oracle_layer(x, edge_index, edge_type, W, root, bias, gout, mode=MODE_ALL, rel=0, dtype=torch.float32):
    """The oracle layer (CPU autograd) in ``dtype``: mode ALL = the RGCNConv loop
    (rgcn_forward), mode SINGLE = CustomRGCNConv over relation ``rel`` (the same loop over that
    relation alone, 2-D weight, before the reference's squeeze). Returns
    {"out", "dx", "dW", "droot", "dbias"} (grads only for the tensors given; no backward when
    ``gout`` is None)."""
    xs = x.detach().to(dtype).requires_grad_(gout is not None)
    ps = [None if p is None else p.detach().to(dtype).requires_grad_(gout is not None) for p in (W, root, bias)]
    if mode == MODE_ALL:
        out = orc.rgcn_forward(xs, edge_index, edge_type, ps[0], ps[1], ps[2])
    else:  # CustomRGCNConv's arithmetic without its final squeeze (rgcn_forward over one relation)
        out = orc.rgcn_forward(xs, edge_index, torch.where(edge_type == rel, 0, -1), ps[0][None], ps[1], ps[2])
    res = {"out": out.detach()}
    if gout is not None:
        out.backward(gout.to(dtype))
        res["dx"] = xs.grad
        for k, p in zip(("dW", "droot", "dbias"), ps):
            if p is not None:
                res[k] = p.grad
    return res


def oracle_layer2(*args, **kw):
    """``oracle_layer`` in float32 (the reference path) and float64 (the truth)."""
    return oracle_layer(*args, **kw, dtype=torch.float32), oracle_layer(*args, **kw, dtype=torch.float64)


def close_all(got: dict, r32: dict, r64: dict, prefix=""):
    """rel_close over every key of ``got`` (keys of oracle_layer)."""
    for k, v in got.items():
        rel_close(v, r32[k], what=prefix + k, ref64=r64[k])


def kink_act(gpu_acts, rel_tol=1e-5):
    """Oracle ReLU that follows the GPU's mask where the pre-activation is within
    ``rel_tol``·max of zero (a kink the two fp32 paths may resolve differently) and its own
    mask everywhere else. ``gpu_acts[k]`` = the GPU tensor whose sign decides the k-th ReLU
    (its output, or its input)."""
    def act(k, v):
        pre = v.detach()
        if k >= len(gpu_acts):
            return torch.relu(v)
        mine = pre > 0
        theirs = gpu_acts[k].detach().cpu() > 0
        near = pre.abs() <= rel_tol * float(pre.abs().max())
        flips = int(((mine != theirs) & ~near).sum())
        assert flips == 0, f"ReLU {k}: {flips} mask differences away from the kink"
        return v * torch.where(near, theirs, mine).to(v.dtype)
    return act


def oracle_means_per_segment(plan, x, mode, relation, num_relations, ei, et):
    """Oracle segment means in the plan's relation-major segment order."""
    b, e = plan.select(mode, relation, num_relations)
    s_row = torch.from_numpy(plan.table("s_row")[b:e].astype(np.int64))
    s_rel = plan.table("s_rel")[b:e]
    out = torch.empty(e - b, x.shape[1])
    for r in np.unique(s_rel):
        h = orc.segment_means(x, ei, et, int(r))
        m = torch.from_numpy(s_rel == r)
        out[m] = h[s_row[m]]
    return out


# ------------------------------------------------------------------------------------------
# bit-exact mean aggregation
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("F", [1, 2, 3, 64, 100, 128, 130, 200, 256])
def test_segment_means_bit_exact_c1(F):
    g = data.synthetic_graph(1000, 3, 10, feat_dim=F, seed=F)
    plan = mpgnn_amd.GraphPlan(g.edge_index, g.edge_type, g.num_nodes)
    xg = g.x.to(DEV)
    for rel in range(3):
        h = segment_means(xg, plan, MODE_SINGLE, rel)
        ref = oracle_means_per_segment(plan, g.x, MODE_SINGLE, rel, 0, g.edge_index, g.edge_type)
        assert torch.equal(h.cpu(), ref), (F, rel)
    h = segment_means(xg, plan, MODE_ALL, -1, 3)
    ref = oracle_means_per_segment(plan, g.x, MODE_ALL, -1, 3, g.edge_index, g.edge_type)
    assert torch.equal(h.cpu(), ref)


def test_segment_means_bit_exact_golden():
    g = np.load("tests/golden/layer_single.npz")
    ei, et = t(g["edge_index"]), t(g["edge_type"])
    plan = mpgnn_amd.GraphPlan(ei, et, 1000)
    for F in (2, 128):
        x = t(g[f"F{F}_x"])
        for rel in range(4):
            b, e = plan.select(MODE_SINGLE, rel, 0)
            h = segment_means(x.to(DEV), plan, MODE_SINGLE, rel).cpu()
            ref_full = t(g[f"F{F}_r{rel}_h"])
            rows = torch.from_numpy(plan.table("s_row")[b:e].astype(np.int64))
            assert torch.equal(h, ref_full[rows])
            # rows without an edge of the relation are exactly zero in the reference
            mask = torch.ones(1000, dtype=torch.bool)
            mask[rows] = False
            assert torch.all(ref_full[mask] == 0)


@pytest.mark.parametrize("name", ["C2", "fb15k237"])
def test_segment_means_bit_exact_full_size(name):
    g = data.config_graph(name)
    plan = mpgnn_amd.GraphPlan(g.edge_index, g.edge_type, g.num_nodes)
    h = segment_means(g.x.to(DEV), plan, MODE_ALL, -1, g.num_relations).cpu()
    # oracle over the whole graph relation by relation (reference loop)
    ref = oracle_means_per_segment(plan, g.x, MODE_ALL, -1, g.num_relations, g.edge_index, g.edge_type)
    assert torch.equal(h, ref)


# ------------------------------------------------------------------------------------------
# layer forward / backward vs reference goldens
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("F_in", [2, 128])
@pytest.mark.parametrize("rel", [0, 1, 2, 3])
def test_custom_rgcn_conv_matches_reference_golden(F_in, rel):
    g = np.load("tests/golden/layer_single.npz")
    ei, et = t(g["edge_index"]).to(DEV), t(g["edge_type"]).to(DEV)
    conv = mpgnn_amd.CustomRGCNConv(F_in, 64, 1, flow="target_to_source").to(DEV)
    with torch.no_grad():
        conv.weight.copy_(t(g[f"F{F_in}_weight"]))
        conv.root.copy_(t(g[f"F{F_in}_root"]))
        conv.bias.copy_(t(g[f"F{F_in}_bias"]))
    x = t(g[f"F{F_in}_x"]).to(DEV).requires_grad_(True)
    out = conv(0, rel, x, ei, et)
    gout = t(g[f"F{F_in}_gout"])
    out.backward(gout.to(DEV))
    # reference fp32 = the golden (the reference's own layer); truth = the oracle in float64
    r64 = oracle_layer(t(g[f"F{F_in}_x"]), t(g["edge_index"]), t(g["edge_type"]), t(g[f"F{F_in}_weight"]),
                       t(g[f"F{F_in}_root"]), t(g[f"F{F_in}_bias"]), gout, MODE_SINGLE, rel, torch.float64)
    rel_close(out, t(g[f"F{F_in}_r{rel}_out"]), what="out", ref64=r64["out"])
    rel_close(x.grad, t(g[f"F{F_in}_r{rel}_dx"]), what="dx", ref64=r64["dx"])
    rel_close(conv.weight.grad, t(g[f"F{F_in}_r{rel}_dweight"]), what="dweight", ref64=r64["dW"])
    rel_close(conv.root.grad, t(g[f"F{F_in}_r{rel}_droot"]), what="droot", ref64=r64["droot"])
    rel_close(conv.bias.grad, t(g[f"F{F_in}_r{rel}_dbias"]), what="dbias", ref64=r64["dbias"])


@pytest.mark.parametrize("F_in", [2, 128])
def test_rgcn_conv_matches_reference_golden(F_in):
    g = np.load("tests/golden/layer_all.npz")
    ei, et = t(g["edge_index"]).to(DEV), t(g["edge_type"]).to(DEV)
    conv = mpgnn_amd.RGCNConv(F_in, 64, 3, flow="target_to_source").to(DEV)
    with torch.no_grad():
        conv.weight.copy_(t(g[f"F{F_in}_weight"]))
        conv.root.copy_(t(g[f"F{F_in}_root"]))
        conv.bias.copy_(t(g[f"F{F_in}_bias"]))
    x = t(g[f"F{F_in}_x"]).to(DEV).requires_grad_(True)
    out = conv(x, ei, et)
    gout = t(g[f"F{F_in}_gout"])
    out.backward(gout.to(DEV))
    r64 = oracle_layer(t(g[f"F{F_in}_x"]), t(g["edge_index"]), t(g["edge_type"]), t(g[f"F{F_in}_weight"]),
                       t(g[f"F{F_in}_root"]), t(g[f"F{F_in}_bias"]), gout, MODE_ALL, 0, torch.float64)
    rel_close(out, t(g[f"F{F_in}_out"]), what="out", ref64=r64["out"])
    rel_close(x.grad, t(g[f"F{F_in}_dx"]), what="dx", ref64=r64["dx"])
    rel_close(conv.weight.grad, t(g[f"F{F_in}_dweight"]), what="dweight", ref64=r64["dW"])
    rel_close(conv.root.grad, t(g[f"F{F_in}_droot"]), what="droot", ref64=r64["droot"])
    rel_close(conv.bias.grad, t(g[f"F{F_in}_dbias"]), what="dbias", ref64=r64["dbias"])


# ------------------------------------------------------------------------------------------
# width sweep vs the oracle (both modes), forward + backward
# ------------------------------------------------------------------------------------------
WIDTHS = [(1, 1), (2, 64), (3, 5), (37, 33), (64, 64), (100, 96), (128, 128), (128, 200), (256, 256), (130, 7)]


@pytest.mark.parametrize("f_in,f_out", WIDTHS)
@pytest.mark.parametrize("mode", [MODE_SINGLE, MODE_ALL])
def test_width_sweep_fwd_bwd(f_in, f_out, mode):
    g = data.synthetic_graph(700, 4, 12, feat_dim=f_in, seed=f_in * 7 + f_out)
    gen = torch.Generator().manual_seed(f_in + 1000 * f_out)
    R = 4
    W = (torch.rand((R, f_in, f_out) if mode == MODE_ALL else (f_in, f_out), generator=gen) - 0.5)
    root = torch.rand(f_in, f_out, generator=gen) - 0.5
    bias = torch.rand(f_out, generator=gen) - 0.5
    gout = torch.randn(700, f_out, generator=gen)
    rel = 2
    r32, r64 = oracle_layer2(g.x, g.edge_index, g.edge_type, W, root, bias, gout, mode=mode, rel=rel)
    plan = mpgnn_amd.GraphPlan(g.edge_index, g.edge_type, 700)
    xg = g.x.to(DEV).requires_grad_(True)
    Wg, rg, bg = (p.to(DEV).requires_grad_(True) for p in (W, root, bias))
    out = rgcn_conv(xg, Wg, rg, bg, plan, mode, relation=rel, num_relations=R)
    out.backward(gout.to(DEV))
    close_all({"out": out, "dx": xg.grad, "dW": Wg.grad, "droot": rg.grad, "dbias": bg.grad}, r32, r64)


def test_no_root_no_bias_and_partial_relations():
    g = data.synthetic_graph(500, 6, 9, feat_dim=48, seed=11)
    gen = torch.Generator().manual_seed(5)
    W = torch.rand(4, 48, 24, generator=gen) - 0.5          # only relations 0..3 of 0..5
    r32, r64 = oracle_layer2(g.x, g.edge_index, g.edge_type, W, None, None, None)
    conv = mpgnn_amd.RGCNConv(48, 24, 4, root_weight=False, bias=False, flow="target_to_source").to(DEV)
    with torch.no_grad():
        conv.weight.copy_(W)
    out = conv(g.x.to(DEV), g.edge_index.to(DEV), g.edge_type.to(DEV))
    rel_close(out, r32["out"], what="out", ref64=r64["out"])


def test_absent_relation_gives_root_plus_bias():
    g = data.synthetic_graph(300, 3, 5, feat_dim=16, seed=2)
    conv = mpgnn_amd.CustomRGCNConv(16, 8, 1, flow="target_to_source").to(DEV)
    out = conv(0, 7, g.x.to(DEV), g.edge_index.to(DEV), g.edge_type.to(DEV))
    ref = g.x @ conv.root.detach().cpu() + conv.bias.detach().cpu()
    ref64 = g.x.double() @ conv.root.detach().cpu().double() + conv.bias.detach().cpu().double()
    rel_close(out, ref, what="out", ref64=ref64)


# ------------------------------------------------------------------------------------------
# models
# ------------------------------------------------------------------------------------------
def test_mpnetm_eval_logits_match_reference_golden():
    g = np.load("tests/golden/mpnetm_synthetic.npz")
    kat = np.load("tests/golden/kat_synthetic.npz")
    link = kat["L3_link"]
    ei = t(np.stack([link[:, 0], link[:, 2]])).to(DEV)
    et = t(link[:, 1]).to(DEV)
    torch.manual_seed(30)
    net = mpgnn_amd.MPNetm(2, 64, 4, 64, 2, 1, [[1, 0]])
    net.load_state_dict({k[3:]: t(g[k]) for k in g.files if k.startswith("sd.")})
    net = net.to(DEV).eval()
    with torch.no_grad():
        logits = net(t(g["x"]).to(DEV), ei, et)
    p64 = {k[3:]: t(g[k]).double() for k in g.files if k.startswith("sd.")}
    ref64 = orc.mpnetm_forward(p64, t(g["x"]).double(), ei.cpu(), et.cpu(), [[1, 0]])
    rel_close(logits, t(g["logits"]), what="logits", ref64=ref64)


@pytest.mark.parametrize("name,hidden,classes", [("C1", 64, 5), ("fb15k237", 64, 5), ("fb15k237", 128, 2)])
def test_net_forward_backward_vs_oracle(name, hidden, classes, monkeypatch):
    """Net (model.py:132-149) forward + every parameter gradient against the oracle's net_forward.
    ("fb15k237", 128, 2) is the bench's headline model, Net(128, 128, 237, 128, 2, 3): its shared
    conv2 takes the GradStash path (the later uses' gradients summed inside the backward kernels
    by mpgnn_rgcn_bwd_accumulate, F = 128 only) — the test asserts that path ran."""
    g = data.config_graph(name)
    F = g.x.shape[1]
    torch.manual_seed(10)                                   # main_rgcn.py:31
    net = mpgnn_amd.Net(F, hidden, g.num_relations, hidden, classes, 3)
    sd = {k: v.detach().clone() for k, v in net.state_dict().items()}
    gout = torch.randn(g.num_nodes, classes, generator=torch.Generator().manual_seed(3))
    net = net.to(DEV)
    import mpgnn_amd.functional as fnl
    from mpgnn_amd import _lib
    calls = {"acc": 0}

    class _Count:
        def __getattr__(self, k):
            f = getattr(_lib.lib, k)
            if k != "mpgnn_rgcn_bwd_accumulate":
                return f

            def wrapped(*a):
                calls["acc"] += 1
                return f(*a)
            return wrapped
    monkeypatch.setattr(fnl, "lib", _Count())
    acts = []  # the three fused-ReLU layer outputs, in call order
    hooks = [m.register_forward_hook(lambda _m, _i, o: acts.append(o.detach())) for m in (net.conv1, net.conv2)]
    out = net(g.x.to(DEV), g.edge_index.to(DEV), g.edge_type.to(DEV))
    for h in hooks:
        h.remove()
    out.backward(gout.to(DEV))
    if hidden == 128:
        assert calls["acc"] == 1, calls  # conv2's second use (backward order) accumulated in-kernel
    act = kink_act(acts)
    res = {}
    for dt in (torch.float32, torch.float64):
        params = {k: v.detach().to(dt, copy=True).requires_grad_(True) for k, v in sd.items()}
        ref = orc.net_forward(params, g.x.to(dt), g.edge_index, g.edge_type, 3, act=act)
        ref.backward(gout.to(dt))
        res[dt] = (ref.detach(), params)
    rel_close(out, res[torch.float32][0], what=f"{name} log_softmax", ref64=res[torch.float64][0])
    for k, p in net.named_parameters():  # whole-model gradients: MODEL_CPU_FACTOR (module docstring)
        rel_close(p.grad, res[torch.float32][1][k].grad, what=f"{name} {k}", ref64=res[torch.float64][1][k].grad,
                  cpu_factor=MODEL_CPU_FACTOR)


def test_adam_training_steps_track_oracle():
    """mpgnn_train semantics (main.py:1055-1082): full-batch NLL on train_idx, backward, Adam
    (lr 0.01, wd 5e-4, main.py:1119). Five steps on GPU vs the same steps on the CPU oracle.
    Adam normalises each gradient by its running RMS, so elements whose gradient is ~0 move by
    ±lr on rounding noise alone: the check is on the loss trajectory (1e-4 rel) and on the
    first step's parameters, not on every element after five steps."""
    g = data.config_graph("C1")
    torch.manual_seed(30)
    net = mpgnn_amd.MPNetm(128, 64, 3, 64, 3, 2, [[1, 0], [2]]).eval()   # eval: no dropout RNG
    ref_params = {k: v.detach().clone().requires_grad_(True) for k, v in net.state_dict().items()}
    names = list(ref_params.keys())
    y = torch.randint(0, 3, (1000,), generator=torch.Generator().manual_seed(1))
    train_idx = torch.arange(0, 1000, 2)
    opt_ref = torch.optim.Adam(list(ref_params.values()), lr=0.01, weight_decay=0.0005)
    netg = net.to(DEV)
    opt = torch.optim.Adam(netg.parameters(), lr=0.01, weight_decay=0.0005)
    xg, eig, etg = g.x.to(DEV), g.edge_index.to(DEV), g.edge_type.to(DEV)
    convs = [c for convs in netg.layers_list for c in convs]  # ReLU inputs in call order
    for step in range(5):
        acts = []
        hooks = [c.register_forward_hook(lambda _m, _i, o: acts.append(o.detach())) for c in convs]
        opt.zero_grad()
        outg = netg(xg, eig, etg)
        for h in hooks:
            h.remove()
        loss = torch.nn.functional.nll_loss(outg[train_idx.to(DEV)], y[train_idx].to(DEV))
        loss.backward()
        act = kink_act(acts) if step == 0 else None  # later steps: the parameters differ by Adam's ±lr noise
        if step == 0:  # before any update the gradients must agree (the fp32 bar, float64 truth)
            p64 = {k: v.detach().double().requires_grad_(True) for k, v in ref_params.items()}
            o64 = orc.mpnetm_forward(p64, g.x.double(), g.edge_index, g.edge_type, [[1, 0], [2]], act=act)
            torch.nn.functional.nll_loss(o64[train_idx], y[train_idx]).backward()
        opt_ref.zero_grad()
        out = orc.mpnetm_forward(ref_params, g.x, g.edge_index, g.edge_type, [[1, 0], [2]], act=act)
        loss_ref = torch.nn.functional.nll_loss(out[train_idx], y[train_idx])
        loss_ref.backward()
        if step == 0:
            for k, p in zip(names, netg.parameters()):
                rel_close(p.grad, ref_params[k].grad, what="grad " + k, ref64=p64[k].grad, cpu_factor=MODEL_CPU_FACTOR)
        opt_ref.step()
        opt.step()
        assert abs(float(loss) - float(loss_ref)) <= 1e-4 * abs(float(loss_ref)), (step, float(loss), float(loss_ref))


# ------------------------------------------------------------------------------------------
# sharding (emulated on one GPU), determinism, errors
# ------------------------------------------------------------------------------------------
_FB_CASES: dict = {}


def fb_layer_case(seed: int, f_out: int, gout_seed: int):
    """FB15K-237 (C3) graph, an RGCNConv(128, f_out) with torch.manual_seed(seed) init and bias
    U(-0.1, 0.1), a seeded output gradient, and the oracle layer in float32 and float64 (cached:
    the float64 loop over 237 relations takes seconds)."""
    key = (seed, f_out, gout_seed)
    g = data.config_graph("fb15k237")
    torch.manual_seed(seed)
    conv = mpgnn_amd.RGCNConv(128, f_out, g.num_relations, flow="target_to_source")
    with torch.no_grad():
        conv.bias.uniform_(-0.1, 0.1)
    gout = torch.randn(g.num_nodes, f_out, generator=torch.Generator().manual_seed(gout_seed))
    if key not in _FB_CASES:
        _FB_CASES[key] = oracle_layer2(g.x, g.edge_index, g.edge_type, conv.weight, conv.root, conv.bias, gout)
    r32, r64 = _FB_CASES[key]
    return g, conv.to(DEV), gout, r32, r64

@pytest.mark.parametrize("f_out", [64, 128])
@pytest.mark.parametrize("world", [2, 4, 8])
def test_dst_range_shards_sum_to_unsharded(world, f_out):
    """node_2-range shards (the north star's partition) on the C3 graph: the partial outputs and
    gradients of the shards sum to the unsharded layer's, both within the bar of the oracle. At
    F_out = 128 every shard runs the bf16-split GEMMs (rel_gemm_bf3 forward / dgrad and the
    bf16-split weight gradient) that the 128 x 128 sharded bench path uses."""
    g, conv, gout, r32, r64 = fb_layer_case(0, f_out, 1)
    xg = g.x.to(DEV).requires_grad_(True)
    eig, etg = g.edge_index.to(DEV), g.edge_type.to(DEV)
    full = conv(xg, eig, etg)
    full.backward(gout.to(DEV))
    close_all({"out": full, "dx": xg.grad, "dW": conv.weight.grad, "droot": conv.root.grad,
               "dbias": conv.bias.grad}, r32, r64, "unsharded ")
    xg.grad = None
    conv.zero_grad()
    ranges = mpgnn_amd.distributed.shard_ranges(g.edge_index, g.num_nodes, world)
    acc = torch.zeros_like(full)
    for lo, hi in ranges:
        part = conv(xg, eig, etg, shard=(lo, hi))
        acc += part.detach()
        part.backward(gout.to(DEV))   # grads accumulate = the all-reduce of the ranks
    close_all({"out": acc, "dx": xg.grad, "dW": conv.weight.grad, "droot": conv.root.grad,
               "dbias": conv.bias.grad}, r32, r64, f"{world} shards ")


def test_deterministic_bitwise():
    g = data.config_graph("fb15k237")
    torch.manual_seed(0)
    conv = mpgnn_amd.RGCNConv(128, 128, g.num_relations, flow="target_to_source").to(DEV)
    xg = g.x.to(DEV).requires_grad_(True)
    eig, etg = g.edge_index.to(DEV), g.edge_type.to(DEV)
    outs, grads = [], []
    for _ in range(2):
        xg.grad = None
        conv.zero_grad()
        o = conv(xg, eig, etg)
        o.backward(torch.ones_like(o))
        outs.append(o.detach().clone())
        grads.append([xg.grad.clone()] + [p.grad.clone() for p in conv.parameters()])
    assert torch.equal(outs[0], outs[1])
    for a, b in zip(*grads):
        assert torch.equal(a, b)


def test_invalid_node_index_raises_index_error():
    ei = torch.tensor([[0, 1, 5], [1, 2, 0]], device=DEV)
    et = torch.tensor([0, 0, 1], device=DEV)
    x = torch.rand(3, 4, device=DEV)
    conv = mpgnn_amd.CustomRGCNConv(4, 4, 1, flow="target_to_source").to(DEV)
    conv(0, 0, x, ei, et)
    with pytest.raises(IndexError):
        conv(0, 1, x, ei, et)


def test_empty_graph_and_isolated_rows():
    ei = torch.zeros(2, 0, dtype=torch.long, device=DEV)
    et = torch.zeros(0, dtype=torch.long, device=DEV)
    x = torch.rand(10, 8, device=DEV)
    conv = mpgnn_amd.RGCNConv(8, 4, 2, flow="target_to_source").to(DEV)
    out = conv(x, ei, et)
    ref = x.cpu() @ conv.root.detach().cpu() + conv.bias.detach().cpu()
    ref64 = x.cpu().double() @ conv.root.detach().cpu().double() + conv.bias.detach().cpu().double()
    rel_close(out, ref, what="out", ref64=ref64)


def test_exact_order_option_and_ragged_pieces_agree():
    """Default path sums runs > 32 entries as ordered pieces; MPGNN_OPT_EXACT_ORDER restores
    the reference's sequential order. Both must match the oracle. (For hub rows that sum ~6000
    terms the sequential order itself carries ~3e-5 relative rounding error; the piece order
    is the more accurate of the two.)"""
    from mpgnn_amd import _lib
    g, conv, gout, r32, r64 = fb_layer_case(0, 64, 1)
    xg = g.x.to(DEV).requires_grad_(True)
    eig, etg = g.edge_index.to(DEV), g.edge_type.to(DEV)
    plan = mpgnn_amd.get_plan(eig, etg, g.num_nodes)  # the plan the layer's calls use
    try:
        for exact in (False, True):
            plan.set_exact_order(exact)
            xg.grad = None
            conv.zero_grad()
            o = conv(xg, eig, etg)
            o.backward(gout.to(DEV))
            close_all({"out": o, "dx": xg.grad, "dW": conv.weight.grad, "droot": conv.root.grad,
                       "dbias": conv.bias.grad}, r32, r64, "exact " if exact else "fast ")
    finally:
        plan.set_exact_order(False)


# ------------------------------------------------------------------------------------------
# the fused ReLU
# ------------------------------------------------------------------------------------------
def _layer_all_outputs(g, F_out, seed, activation=None):
    gen = torch.Generator().manual_seed(seed)
    R, F_in = g.num_relations, g.x.shape[1]
    W = ((torch.rand(R, F_in, F_out, generator=gen) - 0.5) * 0.2).to(DEV).requires_grad_(True)
    root = ((torch.rand(F_in, F_out, generator=gen) - 0.5) * 0.2).to(DEV).requires_grad_(True)
    bias = (torch.rand(F_out, generator=gen) - 0.5).to(DEV).requires_grad_(True)
    gout = torch.randn(g.num_nodes, F_out, generator=gen).to(DEV)
    plan = mpgnn_amd.get_plan(g.edge_index, g.edge_type, g.num_nodes)
    xg = g.x.to(DEV).requires_grad_(True)
    out = rgcn_conv(xg, W, root, bias, plan, MODE_ALL, num_relations=R, activation=activation)
    out.backward(gout)
    h = segment_means(g.x.to(DEV), plan, MODE_ALL, -1, R)
    torch.cuda.synchronize()
    return [v.detach().clone() for v in (out, h, xg.grad, W.grad, root.grad, bias.grad)]


@pytest.mark.parametrize("cfg", ["C1", "fb15k237"])
def test_fused_relu_equals_relu_of_layer(cfg):
    """activation='relu' (fused into the combine epilogue) == F.relu(layer) bit for bit,
    gradients included (threshold_backward on the fused output)."""
    g = data.config_graph(cfg)
    F_out = 64
    fused = _layer_all_outputs(g, F_out, 7, activation="relu")
    gen = torch.Generator().manual_seed(7)
    R, F_in = g.num_relations, g.x.shape[1]
    W = ((torch.rand(R, F_in, F_out, generator=gen) - 0.5) * 0.2).to(DEV).requires_grad_(True)
    root = ((torch.rand(F_in, F_out, generator=gen) - 0.5) * 0.2).to(DEV).requires_grad_(True)
    bias = (torch.rand(F_out, generator=gen) - 0.5).to(DEV).requires_grad_(True)
    gout = torch.randn(g.num_nodes, F_out, generator=gen).to(DEV)
    plan = mpgnn_amd.get_plan(g.edge_index, g.edge_type, g.num_nodes)
    xg = g.x.to(DEV).requires_grad_(True)
    out = torch.relu(rgcn_conv(xg, W, root, bias, plan, MODE_ALL, num_relations=R))
    out.backward(gout)
    torch.cuda.synchronize()
    for name, a, b in zip(("out", "dx", "dW", "droot", "dbias"),
                          (fused[0], fused[2], fused[3], fused[4], fused[5]),
                          (out, xg.grad, W.grad, root.grad, bias.grad)):
        assert torch.equal(a, b.detach()), (cfg, name)
    assert bool((fused[0] >= 0).all()) and bool((fused[0] == 0).any())


def test_fused_relu_propagates_nan():
    """A NaN in x reaches the outputs through the fused ReLU as torch.relu would pass it
    (fmaxf(NaN, 0) = 0 would hide a diverging run); same NaN pattern as
    relu(layer) and the same finite values elsewhere."""
    g = data.config_graph("C1")
    F_out = 32
    gen = torch.Generator().manual_seed(11)
    R, F_in = g.num_relations, g.x.shape[1]
    W = ((torch.rand(R, F_in, F_out, generator=gen) - 0.5) * 0.2).to(DEV)
    root = ((torch.rand(F_in, F_out, generator=gen) - 0.5) * 0.2).to(DEV)
    bias = (torch.rand(F_out, generator=gen) - 0.5).to(DEV)
    x = g.x.clone()
    x[int(g.edge_index[1, 0])] = float("nan")  # a gathered row: NaN spreads to its neighbours' means
    x[5, 3] = float("nan")                      # and a root row
    plan = mpgnn_amd.get_plan(g.edge_index, g.edge_type, g.num_nodes)
    with torch.no_grad():
        fused = rgcn_conv(x.to(DEV), W, root, bias, plan, MODE_ALL, num_relations=R, activation="relu")
        plain = torch.relu(rgcn_conv(x.to(DEV), W, root, bias, plan, MODE_ALL, num_relations=R))
    torch.cuda.synchronize()
    assert bool(torch.isnan(plain).any())
    assert torch.equal(torch.isnan(fused), torch.isnan(plain))
    assert torch.equal(torch.nan_to_num(fused, nan=0.0), torch.nan_to_num(plain, nan=0.0))


def test_fused_relu_mode_single_and_exact_paths():
    """The paths without a fused epilogue (mode SINGLE, exact order) apply the ReLU after the
    combine; Net with the fused activation matches the oracle's F.relu(conv) stack."""
    from mpgnn_amd import _lib
    g = data.config_graph("C1")
    gen = torch.Generator().manual_seed(3)
    W = ((torch.rand(g.x.shape[1], 32, generator=gen) - 0.5) * 0.2).to(DEV)
    root = ((torch.rand(g.x.shape[1], 32, generator=gen) - 0.5) * 0.2).to(DEV)
    bias = (torch.rand(32, generator=gen) - 0.5).to(DEV)
    plan = mpgnn_amd.get_plan(g.edge_index, g.edge_type, g.num_nodes)
    xg = g.x.to(DEV)
    a = rgcn_conv(xg, W, root, bias, plan, MODE_SINGLE, relation=1, activation="relu")
    b = torch.relu(rgcn_conv(xg, W, root, bias, plan, MODE_SINGLE, relation=1))
    assert torch.equal(a, b)
    try:
        plan.set_exact_order(True)
        Wa = W[None].expand(g.num_relations, -1, -1).contiguous()
        a = rgcn_conv(xg, Wa, root, bias, plan, MODE_ALL, num_relations=g.num_relations, activation="relu")
        b = torch.relu(rgcn_conv(xg, Wa, root, bias, plan, MODE_ALL, num_relations=g.num_relations))
        assert torch.equal(a, b)
    finally:
        plan.set_exact_order(False)
    torch.manual_seed(10)
    net = mpgnn_amd.Net(g.x.shape[1], 32, g.num_relations, 32, 2, 3)
    params = {k: v.detach().clone() for k, v in net.state_dict().items()}
    ref = orc.net_forward(params, g.x, g.edge_index, g.edge_type, 3)
    ref64 = orc.net_forward({k: v.double() for k, v in params.items()}, g.x.double(), g.edge_index, g.edge_type, 3)
    out = net.to(DEV)(xg, g.edge_index.to(DEV), g.edge_type.to(DEV))
    rel_close(out, ref, what="Net", ref64=ref64)


@pytest.mark.parametrize("f_in", [64, 128])
@pytest.mark.parametrize("mode", [MODE_SINGLE, MODE_ALL])
def test_rel_gemm_matches_oracle_and_tile_gemm(f_in, mode):
    """MPGNN_OPT_REL_GEMM (default on: weights held in registers per relation run, 32-row
    tiles) for F_out = 128: forward and every gradient match the oracle and the tile GEMM."""
    from mpgnn_amd import _lib
    f_out = 128
    g = data.config_graph("fb15k237") if f_in == 128 else \
        data.synthetic_graph(2000, 9, 30, feat_dim=f_in, seed=5)
    N, R = g.num_nodes, g.num_relations
    gen = torch.Generator().manual_seed(f_in + mode)
    W = (torch.rand((R, f_in, f_out) if mode == MODE_ALL else (f_in, f_out), generator=gen) - 0.5) * 0.2
    root = (torch.rand(f_in, f_out, generator=gen) - 0.5) * 0.2
    bias = torch.rand(f_out, generator=gen) - 0.5
    gout = torch.randn(N, f_out, generator=gen)
    rel = 2
    r32, r64 = oracle_layer2(g.x, g.edge_index, g.edge_type, W, root, bias, gout, mode=mode, rel=rel)
    plan = mpgnn_amd.GraphPlan(g.edge_index, g.edge_type, N)
    try:
        for on in (1, 0):
            plan.set_option(5, on)
            xg = g.x.to(DEV).requires_grad_(True)
            Wg, rg, bg = (p.to(DEV).requires_grad_(True) for p in (W, root, bias))
            out = rgcn_conv(xg, Wg, rg, bg, plan, mode, relation=rel, num_relations=R)
            out.backward(gout.to(DEV))
            torch.cuda.synchronize()
            close_all({"out": out, "dx": xg.grad, "dW": Wg.grad, "droot": rg.grad, "dbias": bg.grad}, r32, r64,
                      "rel_gemm " if on else "tile_gemm ")
    finally:
        plan.set_option(5, 1)


@pytest.mark.parametrize("mode", [MODE_ALL, MODE_SINGLE])
@pytest.mark.parametrize("rows", [None, (0.25, 0.8)])
def test_fused_backward_matches_two_launches_and_oracle(mode, rows):
    """MPGNN_OPT_BWD_FUSED (bwd_bf3_kernel: dgrad + dW / droot / dbias in one launch, dW slabs
    per workgroup run; taken when the layer has at most 4 items per CU) against the dgrad launch
    + chunked dW launch: grad_x bit-identical (the same products in the same order), the
    parameter gradients within the suite's bar of the oracle either way — mode ALL on a graph of
    ~900 items (8 relations, many runs per workgroup), mode SINGLE on C3's largest relation (hub
    rows), a node_1 row range (root items of a shard), repeated calls (cached slab layout)."""
    from mpgnn_amd import _lib
    g = data.config_graph("fb15k237") if mode == MODE_SINGLE else \
        data.synthetic_graph(6000, 8, 8, feat_dim=128, seed=21)
    N, R = g.num_nodes, g.num_relations
    gen = torch.Generator().manual_seed(40 + mode)
    W = (torch.rand((R, 128, 128) if mode == MODE_ALL else (128, 128), generator=gen) - 0.5) * 0.2
    root = (torch.rand(128, 128, generator=gen) - 0.5) * 0.2
    bias = torch.rand(128, generator=gen) - 0.5
    gout = torch.randn(N, 128, generator=gen)
    rel = int(torch.bincount(g.edge_type).argmax())
    lo, hi = (0, N) if rows is None else (int(rows[0] * N), int(rows[1] * N))
    plan = mpgnn_amd.GraphPlan(g.edge_index, g.edge_type, N)
    res = {}
    for fused in (1, 0, 1):
        plan.set_option(25, fused)
        xg = g.x.to(DEV).requires_grad_(True)
        Wg, rg, bg = (t.to(DEV).requires_grad_(True) for t in (W, root, bias))
        out = rgcn_conv(xg, Wg, rg, bg, plan, mode, relation=rel, num_relations=R,
                        row_range=None if rows is None else (lo, hi))
        out.backward(gout.to(DEV))
        torch.cuda.synchronize()
        got = {"dx": xg.grad, "dW": Wg.grad, "droot": rg.grad, "dbias": bg.grad}
        if fused in res:
            for k in got:
                assert torch.equal(got[k], res[fused][k]), (fused, k, "not repeatable")
        res[fused] = got
    assert torch.equal(res[1]["dx"], res[0]["dx"]), "grad_x differs between the fused and the two-launch backward"
    if rows is None:
        r32, r64 = oracle_layer2(g.x, g.edge_index, g.edge_type, W, root, bias, gout, mode=mode, rel=rel)
        for k in ("dW", "droot", "dbias", "dx"):
            rel_close(res[1][k], r32[k], what=f"fused bwd {k}", ref64=r64[k])
    else:  # a row range: the two backwards agree to fp32 summation order (their bar vs the truth: above)
        for k in ("dW", "droot", "dbias"):
            nw = normwise_err(res[1][k].cpu(), res[0][k].cpu())
            record(f"fused bwd rows {k} vs two-launch", nw, 1e-5, normwise=nw)
            assert nw <= 1e-5, (k, nw)


def test_grad_x_hub_rows_finished_in_launch_equal_finalize():
    """MPGNN_OPT_FLAT_FUSE_SPLIT: the C3 grad_x rows of more than 16 chunks (hub nodes, up to
    ~190 pieces) finished by the wave that adds their last piece (write-through partials, an
    agent-scope piece counter, the slots summed in chunk order) against finalize_rows_kernel
    after the launch: grad_x bit-identical, repeated calls (the counters must return to zero —
    a stale count would finish a row early or never), and the oracle's bar."""
    from mpgnn_amd import _lib
    g = data.fb15k237_graph(feat_dim=128, seed=0, recipe="survey")
    N, R = g.num_nodes, g.num_relations
    indeg = torch.bincount(g.edge_index[1], minlength=N)
    assert int(indeg.max()) > 16 * 32, "C3 has no hub row of more than 16 chunks"
    gen = torch.Generator().manual_seed(77)
    W = (torch.rand((R, 128, 128), generator=gen) - 0.5) * 0.2
    root = (torch.rand(128, 128, generator=gen) - 0.5) * 0.2
    bias = torch.rand(128, generator=gen) - 0.5
    gout = torch.randn(N, 128, generator=gen)
    plan = mpgnn_amd.GraphPlan(g.edge_index.to(DEV), g.edge_type.to(DEV), N)
    xg0 = g.x.to(DEV)
    Wg, rg, bg = (t.to(DEV) for t in (W, root, bias))
    res = {}
    for fuse in (1, 0, 1, 1):
        plan.set_option(27, fuse)
        xg = xg0.clone().requires_grad_(True)
        out = rgcn_conv(xg, Wg, rg, bg, plan, MODE_ALL, num_relations=R)
        out.backward(gout.to(DEV))
        torch.cuda.synchronize()
        if fuse in res:
            assert torch.equal(xg.grad, res[fuse]), (fuse, "not repeatable")
        res[fuse] = xg.grad
    assert torch.equal(res[1], res[0]), "grad_x differs between the in-launch finish and finalize_rows_kernel"
    hubs = torch.nonzero(indeg > 16 * 32).flatten()
    r32, r64 = oracle_layer2(g.x, g.edge_index, g.edge_type, W, root, bias, gout, mode=MODE_ALL, rel=None)
    rel_close(res[1][hubs.to(DEV)], r32["dx"][hubs], what="grad_x hub rows (in-launch finish)", ref64=r64["dx"][hubs])
    rel_close(res[1], r32["dx"], what="grad_x C3 (in-launch finish)", ref64=r64["dx"])


@pytest.mark.parametrize("feat", [128, 256])
def test_weight_gradient_vector_gathers_equal_column_gathers(feat):
    """MPGNN_OPT_OUTER_VEC: outer_bf3v_kernel (16-B row gathers, row-major planes read with
    ds_read_b64_tr_b16) against outer_bf3_kernel (4-B column gathers, transposed planes): the
    same bf16 pieces reach the matrix cores, 16 rows per instruction in slice order, so dW and
    droot agree to the matrix cores' in-instruction rounding (held to 1e-6 normwise; both are
    held to the oracle's bar elsewhere); dbias sums each column in another fixed order. Each
    kernel is bitwise repeatable. C3 graph at F = 128; a synthetic graph at F = 256 (the
    four-quadrant launches)."""
    from mpgnn_amd import _lib
    if feat == 128:
        g = data.fb15k237_graph(feat_dim=128, seed=0, recipe="survey")
    else:
        g = data.synthetic_graph(3000, 6, 8, feat_dim=256, seed=5)
    N, R = g.num_nodes, g.num_relations
    gen = torch.Generator().manual_seed(91 + feat)
    W = (torch.rand((R, feat, feat), generator=gen) - 0.5) * 0.2
    root = (torch.rand(feat, feat, generator=gen) - 0.5) * 0.2
    bias = torch.rand(feat, generator=gen) - 0.5
    gout = torch.randn(N, feat, generator=gen)
    plan = mpgnn_amd.GraphPlan(g.edge_index.to(DEV), g.edge_type.to(DEV), N)
    res = {}
    for vec in (1, 0, 1):
        plan.set_option(28, vec)
        Wg, rg, bg = (t.to(DEV).requires_grad_(True) for t in (W, root, bias))
        out = rgcn_conv(g.x.to(DEV), Wg, rg, bg, plan, MODE_ALL, num_relations=R)
        out.backward(gout.to(DEV))
        torch.cuda.synchronize()
        got = {"dW": Wg.grad, "droot": rg.grad, "dbias": bg.grad}
        if vec in res:
            for k in got:
                assert torch.equal(got[k], res[vec][k]), (vec, k, "not repeatable")
        res[vec] = got
    for k in ("dW", "droot"):
        nwk = normwise_err(res[1][k].cpu(), res[0][k].cpu())
        record(f"{k} outer_bf3v vs outer_bf3 F={feat}", nwk, 1e-6, normwise=nwk)
        assert nwk <= 1e-6, (k, nwk)
    nw = normwise_err(res[1]["dbias"].cpu(), res[0]["dbias"].cpu())
    record(f"dbias outer_bf3v vs outer_bf3 F={feat}", nw, 1e-6, normwise=nw)
    assert nw <= 1e-6, nw


def test_gemm_item_ranges_do_not_change_results():
    """MPGNN_OPT_GEMM_SWITCH_COST: the bf16-split GEMM's workgroup item ranges balanced by
    items + weight switches (default) against equal item counts — each item's arithmetic is the
    same wherever it runs, so the layer output and every gradient are bit-identical (C3)."""
    from mpgnn_amd import _lib
    g = data.fb15k237_graph(feat_dim=128, seed=0, recipe="survey")
    N, R = g.num_nodes, g.num_relations
    gen = torch.Generator().manual_seed(5)
    W = (torch.rand((R, 128, 128), generator=gen) - 0.5) * 0.2
    root = (torch.rand(128, 128, generator=gen) - 0.5) * 0.2
    bias = torch.rand(128, generator=gen) - 0.5
    gout = torch.randn(N, 128, generator=gen)
    plan = mpgnn_amd.GraphPlan(g.edge_index.to(DEV), g.edge_type.to(DEV), N)
    res = {}
    for cost in (250, 0, 100):
        plan.set_option(29, cost)
        xg = g.x.to(DEV).requires_grad_(True)
        Wg, rg, bg = (t.to(DEV).requires_grad_(True) for t in (W, root, bias))
        out = rgcn_conv(xg, Wg, rg, bg, plan, MODE_ALL, num_relations=R)
        out.backward(gout.to(DEV))
        torch.cuda.synchronize()
        res[cost] = [out.detach(), xg.grad, Wg.grad, rg.grad, bg.grad]
    for cost in (0, 100):
        for k, a, b in zip(("out", "dx", "dW", "droot", "dbias"), res[cost], res[250]):
            assert torch.equal(a, b), (cost, k)


@pytest.mark.parametrize("mode", ["all", "single"])
def test_k256_gemm_interleaved_commit_bit_identical(mode):
    """MPGNN_OPT_GEMM_W_IL (34): the K = 256 bf16-split GEMM (F_in = F_out = 256, C5's width) with
    the next item's tile committed in four parts among the k-steps' MFMAs computes the same
    products in the same order as the one-k-step commit — forward and dgrad (mode ALL) and the
    mode-SINGLE forward with its root epilogue, bit-identical; a ragged last node tile (N % 32)
    and partial relation tiles included."""
    g = data.synthetic_graph(6007, 7, 10, feat_dim=256, seed=21)
    N, R = g.num_nodes, g.num_relations
    gen = torch.Generator().manual_seed(9)
    single = mode == "single"
    W = (torch.rand((256, 256) if single else (R, 256, 256), generator=gen) - 0.5) * 0.1
    root = (torch.rand(256, 256, generator=gen) - 0.5) * 0.1
    bias = torch.rand(256, generator=gen) - 0.5
    gout = torch.randn(N, 256, generator=gen)
    plan = mpgnn_amd.GraphPlan(g.edge_index.to(DEV), g.edge_type.to(DEV), N)
    res = {}
    for il in (0, 1, 0):
        plan.set_option(34, il)
        xg = g.x.to(DEV).requires_grad_(not single)
        Wg, rg, bg = (t.to(DEV).requires_grad_(not single) for t in (W, root, bias))
        if single:
            with torch.no_grad():
                out = rgcn_conv(xg, Wg, rg, bg, plan, MODE_SINGLE, relation=3, activation="relu")
            res[il] = [out]
        else:
            out = rgcn_conv(xg, Wg, rg, bg, plan, MODE_ALL, num_relations=R)
            out.backward(gout.to(DEV))
            res[il] = [out.detach(), xg.grad, Wg.grad, rg.grad, bg.grad]
        torch.cuda.synchronize()
    plan.set_option(34, _lib_default(34))
    for k, a, b in zip(("out", "dx", "dW", "droot", "dbias"), res[1], res[0]):
        assert torch.equal(a, b), k
    assert res[0][0].abs().sum() > 0


@pytest.mark.parametrize("opt,val,graph", [(35, 1, "syn"), (36, 1, "syn"), (36, 2, "syn"), (37, 32, "syn"),
                                           (37, 8, "syn"), (38, 1, "syn"), (41, 1, "syn"), (41, 1, "fb15k237"),
                                           (42, 0, "syn"), (42, 0, "fb15k237")])
def test_w1_gemm_and_outer_variants_bit_identical(opt, val, graph):
    """Round 6 variants, off by default, against the product kernels on one layer (forward, dgrad,
    every gradient) — bit for bit:
      35 MPGNN_OPT_GEMM_W1: rel_gemm_w1_kernel (one workgroup per CU, 64-row items: tile pairs of
         one relation, a relation's odd last tile alone, 64-node root items with a ragged last one,
         the next relation's weight slice prefetched) vs rel_gemm_bf3_kernel;
      36 MPGNN_OPT_OUTER_VARIANT: the weight gradient's row indices by scalar loads (1), or the
         next-next slice's rows issued after the MFMAs (2), vs the product order.
      37 MPGNN_OPT_FLAT_U: the gather-sum kernels with 32 / 8 rows in flight per wave (means,
         combine, grad_x) vs 16;
      38 MPGNN_OPT_FLAT_PAD: their chunks fetched from the padded per-slot tables vs the scalar
         chunk-range hops;
      41 MPGNN_OPT_BWD_SIDE_REDUCE: the weight gradient's slab sum on a side stream beside dgrad and
         grad_x (C3 takes that path: more items than the one-launch backward's four per CU);
      42 MPGNN_OPT_GEMM_FIRST (on by default; the test turns it off): the GEMM prologue's range and
         first rows from per-range records vs the range -> tiles -> row-index hops.
    A graph with relations of 1, odd and even 32-row tile counts and N % 64 != 0, and C3."""
    g = data.synthetic_graph(5003, 9, 12, feat_dim=128, seed=37) if graph == "syn" else data.config_graph(graph)
    N, R = g.num_nodes, g.num_relations
    gen = torch.Generator().manual_seed(opt + val)
    W = (torch.rand((R, 128, 128), generator=gen) - 0.5) * 0.1
    root = (torch.rand(128, 128, generator=gen) - 0.5) * 0.1
    bias = torch.rand(128, generator=gen) - 0.5
    gout = torch.randn(N, 128, generator=gen)
    plan = mpgnn_amd.GraphPlan(g.edge_index.to(DEV), g.edge_type.to(DEV), N)
    res = {}
    base = _lib_default(opt)  # the product setting (0, or 16 rows in flight for option 37)
    for v in (base, val):
        plan.set_option(opt, v)
        xg = g.x.to(DEV).requires_grad_(True)
        Wg, rg, bg = (t.to(DEV).requires_grad_(True) for t in (W, root, bias))
        out = rgcn_conv(xg, Wg, rg, bg, plan, MODE_ALL, num_relations=R, activation="relu")
        out.backward(gout.to(DEV))
        torch.cuda.synchronize()
        res[v] = [out.detach(), xg.grad, Wg.grad, rg.grad, bg.grad]
    plan.set_option(opt, _lib_default(opt))
    for k, a, b in zip(("out", "dx", "dW", "droot", "dbias"), res[val], res[base]):
        assert torch.equal(a, b), k
    assert res[base][0].abs().sum() > 0 and res[base][2].abs().sum() > 0


@pytest.mark.parametrize("f_in", [128, 64])
def test_single_fold_bit_identical(f_in):
    """MPGNN_OPT_SINGLE_FOLD (39): the fused mode-SINGLE layer computing the relation's multi-edge
    segment means inside its GEMM launch (32-edge pieces added in order, / cnt) against the means
    launch + GEMM: forward and every gradient (dW reads the saved means the fold writes) bit for
    bit, on a relation with hub segments of 33, 40 (two pieces) and 600 edges (> 16 pieces: the
    means kernel's split rows) and a ragged last node tile."""
    g = data.synthetic_graph(3001, 5, 12, feat_dim=f_in, seed=41)
    rng = np.random.default_rng(5)
    hubs = [(7, 600), (11, 40), (13, 33)]
    n1 = np.concatenate([np.full(k, v) for v, k in hubs])
    n2 = rng.integers(0, g.num_nodes, size=n1.size)
    ei = torch.cat([g.edge_index, torch.from_numpy(np.stack([n1, n2]))], 1)
    et = torch.cat([g.edge_type, torch.full((n1.size,), 2, dtype=torch.int64)])
    N = g.num_nodes
    gen = torch.Generator().manual_seed(f_in)
    W = (torch.rand(f_in, 128, generator=gen) - 0.5) * 0.1
    root = (torch.rand(f_in, 128, generator=gen) - 0.5) * 0.1
    bias = torch.rand(128, generator=gen) - 0.5
    gout = torch.randn(N, 128, generator=gen)
    plan = mpgnn_amd.GraphPlan(ei.to(DEV), et.to(DEV), N)
    res = {}
    for v in (0, 1):
        plan.set_option(39, v)
        xg = g.x.to(DEV).requires_grad_(True)
        Wg, rg, bg = (t.to(DEV).requires_grad_(True) for t in (W, root, bias))
        out = rgcn_conv(xg, Wg, rg, bg, plan, MODE_SINGLE, relation=2, activation="relu")
        out.backward(gout.to(DEV))
        with torch.no_grad():
            out_inf = rgcn_conv(g.x.to(DEV), Wg, rg, bg, plan, MODE_SINGLE, relation=2, activation="relu")
        torch.cuda.synchronize()
        res[v] = [out.detach(), out_inf, xg.grad, Wg.grad, rg.grad, bg.grad]
    plan.set_option(39, _lib_default(39))
    for k, a, b in zip(("out", "out no-grad", "dx", "dW", "droot", "dbias"), res[1], res[0]):
        assert torch.equal(a, b), k
    assert res[0][0].abs().sum() > 0 and res[0][3].abs().sum() > 0


def _lib_default(opt):
    from mpgnn_amd import _lib
    return _lib.get_option(opt)


# ------------------------------------------------------------------------------------------
# CustomFastRGCNConv (A7): transform-then-aggregate semantics on the same kernels
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("f_in,f_out", [(16, 16), (128, 64)])
def test_fast_rgcn_conv_matches_per_edge_oracle(f_in, f_out):
    g = data.synthetic_graph(500, 5, 10, feat_dim=f_in, seed=11 + f_in)
    torch.manual_seed(30)
    conv = mpgnn_amd.CustomFastRGCNConv(f_in, f_out, 5, flow="target_to_source")
    with torch.no_grad():
        conv.bias.uniform_(-0.5, 0.5)
    gout = torch.randn(g.num_nodes, f_out, generator=torch.Generator().manual_seed(f_in))
    ref = {}
    for dt in (torch.float32, torch.float64):
        xs = g.x.detach().to(dt, copy=True).requires_grad_(True)
        ps = [p.detach().to(dt, copy=True).requires_grad_(True) for p in (conv.weight, conv.root, conv.bias)]
        o = orc.fast_rgcn_forward(xs, g.edge_index, g.edge_type, *ps)
        o.backward(gout.to(dt))
        ref[dt] = (o.detach(), xs.grad, [p.grad for p in ps])
    convg = conv.to(DEV)
    xg = g.x.to(DEV).requires_grad_(True)
    out = convg(xg, g.edge_index.to(DEV), g.edge_type.to(DEV))
    rel_close(out, ref[torch.float32][0], what="fast out", ref64=ref[torch.float64][0])
    out.backward(gout.to(DEV))
    rel_close(xg.grad, ref[torch.float32][1], what="fast dx", ref64=ref[torch.float64][1])
    # dW (per-edge transform x_j @ W[edge_type], scaled, scattered: mp_rgcn_layer.py:344-357), droot, dbias
    for name, p, r32, r64 in zip(("dW", "droot", "dbias"), (convg.weight, convg.root, convg.bias),
                                 ref[torch.float32][2], ref[torch.float64][2]):
        rel_close(p.grad, r32, what=f"fast {name}", ref64=r64)


# ------------------------------------------------------------------------------------------
# C5 at full size (2M nodes, 64 relations, 32M edges, 256-d: x = 2 GB, far beyond the LLC)
# ------------------------------------------------------------------------------------------
def test_c5_full_size_sampled_rows_vs_oracle():
    """BASELINE.json configs[4] on one GPU: the whole graph is aggregated and transformed; the
    check runs on 192 sampled rows (the full oracle is 64 dense 2M×256×256 GEMMs per layer):
    segment means bit-exact (sequential fp32 sum in edge order, IEEE division) and the
    RGCNConv output within 1e-4 of the per-relation loop of model.py / mp_rgcn_layer.py:249-258."""
    g = data.config_graph("C5")
    N, R, F = g.num_nodes, g.num_relations, g.x.shape[1]
    plan = mpgnn_amd.GraphPlan(g.edge_index, g.edge_type, N)
    xg = g.x.to(DEV)
    rng = np.random.default_rng(5)
    rows = np.sort(rng.choice(N, 192, replace=False))
    ei0, ei1, et = g.edge_index[0].numpy(), g.edge_index[1].numpy(), g.edge_type.numpy()
    sel = np.nonzero(np.isin(ei0, rows))[0]  # edges of the sampled rows, original order
    x = g.x.numpy()
    means = {}
    for e in sel:  # sequential fp32 accumulation in edge order (ATen scatter_add_ order)
        key = (int(ei0[e]), int(et[e]))
        acc, c = means.get(key, (np.zeros(F, np.float32), 0))
        means[key] = (acc + x[ei1[e]], c + 1)
    # segment means through the C ABI, bit-exact
    s_row, s_rel = plan.table("s_row"), plan.table("s_rel")
    segs = np.nonzero(np.isin(s_row, rows))[0]
    h = segment_means(xg, plan, MODE_ALL, -1, R)
    hs = h[torch.from_numpy(segs).to(DEV)].cpu().numpy()
    del h
    assert len(segs) == len(means)
    for k, sidx in enumerate(segs):
        acc, c = means[(int(s_row[sidx]), int(s_rel[sidx]))]
        assert np.array_equal(hs[k], acc / np.float32(c)), (int(s_row[sidx]), int(s_rel[sidx]))
    # the layer
    torch.manual_seed(30)
    conv = mpgnn_amd.RGCNConv(F, F, R, flow="target_to_source")
    with torch.no_grad():
        conv.bias.uniform_(-0.1, 0.1)
    W, root, bias = conv.weight.detach().clone(), conv.root.detach().clone(), conv.bias.detach().clone()
    conv = conv.to(DEV)
    with torch.no_grad():
        out = conv(xg, g.edge_index.to(DEV), g.edge_type.to(DEV))
        got = out[torch.from_numpy(rows).to(DEV)].cpu()
    del out
    ref = torch.zeros(len(rows), F)
    ref64 = torch.zeros(len(rows), F, dtype=torch.float64)
    W64, root64, bias64 = W.double(), root.double(), bias.double()
    for k, i in enumerate(rows):
        acc = torch.zeros(F)
        acc64 = torch.zeros(F, dtype=torch.float64)
        for r in range(R):  # relation order, as the loop accumulates
            if (int(i), r) in means:
                s, c = means[(int(i), r)]
                h = torch.from_numpy(s / np.float32(c))  # the reference's fp32 means (bit-exact above)
                acc = acc + h @ W[r]
                acc64 = acc64 + h.double() @ W64[r]
        ref[k] = acc + torch.from_numpy(x[i]) @ root + bias
        ref64[k] = acc64 + torch.from_numpy(x[i]).double() @ root64 + bias64
    rel_close(got, ref, what="C5 sampled rows", ref64=ref64)


def test_c5_full_size_backward_sparse_output_gradient_vs_oracle():
    """C5's backward on the whole graph (VERDICT r4 Missing #3): 27.5 M segments through the
    F = 256 kernels — the split-K dgrad (rel_gemm_bf3w_kernel<true>), the four-quadrant weight
    gradient over every reduction chunk and slab (outer_bf3v_kernel), the slab reduce and grad_x
    — with an output gradient that is non-zero only on 192 sampled node_1 rows, so that the
    oracle is cheap: dW_r / droot / dbias involve only those rows' segments, dx only their
    node_2 rows (and the rows themselves through root). Every other dx row must be exactly zero.
    Reference: autograd of mp_rgcn_layer.py:249-258 (+ root, bias) at model.py:206-214's shape."""
    g = data.config_graph("C5")
    N, R, F = g.num_nodes, g.num_relations, g.x.shape[1]
    rng = np.random.default_rng(7)
    rows = np.sort(rng.choice(N, 192, replace=False))
    ei0, ei1, et = g.edge_index[0].numpy(), g.edge_index[1].numpy(), g.edge_type.numpy()
    sel = np.nonzero(np.isin(ei0, rows))[0]
    x = g.x.numpy()
    means = {}
    for e in sel:  # sequential fp32 accumulation in edge order (ATen scatter_add_ order)
        key = (int(ei0[e]), int(et[e]))
        acc, c = means.get(key, (np.zeros(F, np.float32), 0))
        means[key] = (acc + x[ei1[e]], c + 1)
    torch.manual_seed(31)
    conv = mpgnn_amd.RGCNConv(F, F, R, flow="target_to_source")
    with torch.no_grad():
        conv.bias.uniform_(-0.1, 0.1)
    W, root = conv.weight.detach().numpy(), conv.root.detach().numpy()
    gen = torch.Generator().manual_seed(8)
    grow = torch.randn(len(rows), F, generator=gen).numpy()
    # oracle in float32 (rows in order) and float64
    out = {}
    for dt in (np.float32, np.float64):
        dW = np.zeros((R, F, F), dt)
        droot = np.zeros((F, F), dt)
        dbias = np.zeros(F, dt)
        dx = {}
        Wd, rootd = W.astype(dt), root.astype(dt)
        for k, i in enumerate(rows):
            gi = grow[k].astype(dt)
            dbias += gi
            droot += np.outer(x[i].astype(dt), gi)
            dx[int(i)] = dx.get(int(i), np.zeros(F, dt)) + gi @ rootd.T
            for r in range(R):
                if (int(i), r) not in means:
                    continue
                s, c = means[(int(i), r)]
                h = (s / np.float32(c)).astype(dt)
                dW[r] += np.outer(h, gi)
        for e in sel:  # dx[j] += (g_i @ W_r^T) / cnt_r(i)
            i, j, r = int(ei0[e]), int(ei1[e]), int(et[e])
            gi = grow[np.searchsorted(rows, i)].astype(dt)
            c = means[(i, r)][1]
            dx[j] = dx.get(j, np.zeros(F, dt)) + (gi @ Wd[r].T) / dt(c)
        out[dt] = (dW, droot, dbias, dx)
    touched = np.array(sorted(out[np.float32][3]))
    convg = conv.to(DEV)
    xg = g.x.to(DEV).requires_grad_(True)
    gout = torch.zeros(N, F, device=DEV)
    gout[torch.from_numpy(rows).to(DEV)] = torch.from_numpy(grow).to(DEV)
    y = convg(xg, g.edge_index.to(DEV), g.edge_type.to(DEV))
    y.backward(gout)
    del y, gout
    torch.cuda.synchronize()
    r32, r64 = out[np.float32], out[np.float64]
    rel_close(convg.weight.grad, t(r32[0]), what="C5 bwd dW", ref64=t(r64[0]))
    rel_close(convg.root.grad, t(r32[1]), what="C5 bwd droot", ref64=t(r64[1]))
    rel_close(convg.bias.grad, t(r32[2]), what="C5 bwd dbias", ref64=t(r64[2]))
    tix = torch.from_numpy(touched).to(DEV)
    dx_t = xg.grad[tix].cpu()
    rel_close(dx_t, t(np.stack([r32[3][int(j)] for j in touched])), what="C5 bwd dx touched rows",
              ref64=t(np.stack([r64[3][int(j)] for j in touched])))
    mask = torch.ones(N, dtype=torch.bool, device=DEV)
    mask[tix] = False
    assert int(torch.count_nonzero(xg.grad[mask])) == 0, "dx non-zero outside the touched rows"


def test_c2_layer_backward_long_reduction_chunks():
    """C2 (100k nodes, 16 relations, 1.65 M edges): the weight-gradient chunks grow past 128
    segments (plan chunk cap = S / 4096 rounded to 32); one RGCNConv forward + backward vs the
    oracle's autograd."""
    g = data.config_graph("C2")
    plan = mpgnn_amd.GraphPlan(g.edge_index, g.edge_type, g.num_nodes)
    assert plan.num_segments > 128 * 4096  # chunks longer than kChunkRows
    torch.manual_seed(30)
    conv = mpgnn_amd.RGCNConv(128, 128, g.num_relations, flow="target_to_source")
    with torch.no_grad():
        conv.bias.uniform_(-0.1, 0.1)
    gout = torch.randn(g.num_nodes, 128, generator=torch.Generator().manual_seed(3))
    r32, r64 = oracle_layer2(g.x, g.edge_index, g.edge_type, conv.weight, conv.root, conv.bias, gout)
    convg = conv.to(DEV)
    xg = g.x.to(DEV).requires_grad_(True)
    out = convg(xg, g.edge_index.to(DEV), g.edge_type.to(DEV))
    out.backward(gout.to(DEV))
    close_all({"out": out, "dx": xg.grad, "dW": convg.weight.grad, "droot": convg.root.grad,
               "dbias": convg.bias.grad}, r32, r64, "C2 ")


@pytest.mark.parametrize("n,f,o", [(14541, 128, 128), (2000, 256, 200), (777, 96, 70), (1, 128, 128),
                                   (64, 128, 128), (200003, 128, 128)])
def test_linear_wgrad_abi_output_blocks(n, f, o):
    """mpgnn_linear_wgrad for heads wider than one pass (O > 32·256/F: output blocks of
    32·256/F, the partials buffer reused in stream order): weight and bias gradient against the
    float64 truth at the suite's bar."""
    import ctypes
    from mpgnn_amd import _lib
    gen = torch.Generator().manual_seed(n + o)
    x = torch.randn(n, f, generator=gen)
    g = torch.randn(n, o, generator=gen)
    xd, gd = x.to(DEV), g.to(DEV)
    nb = ctypes.c_int64()
    _lib.check(_lib.lib.mpgnn_linear_wgrad_workspace_bytes(n, f, o, ctypes.byref(nb)))
    ws = torch.empty(int(nb.value), dtype=torch.uint8, device=DEV)
    gw = torch.empty(o, f, device=DEV)
    gb = torch.empty(o, device=DEV)
    _lib.check(_lib.lib.mpgnn_linear_wgrad(xd.data_ptr(), gd.data_ptr(), n, f, o, gw.data_ptr(), gb.data_ptr(),
                                           ws.data_ptr(), torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    rel_close(gw, g.t() @ x, what=f"linear_wgrad {n}x{f}->{o} dW", ref64=g.double().t() @ x.double())
    rel_close(gb, g.sum(0), what=f"linear_wgrad {n}x{f}->{o} db", ref64=g.double().sum(0))


@pytest.mark.parametrize("n,f_in,f_out", [(14541, 128, 2), (1000, 128, 64), (300, 64, 3), (14541, 128, 128),
                                         (2000, 256, 200)])
def test_split_k_linear_matches_nn_linear(n, f_in, f_out):
    """model.linear: forward (the C ABI's mpgnn_linear_fwd for 128 -> 128 and O <= 8, nn.Linear's
    GEMM otherwise), grad_weight (sliced over rows) and grad_bias / grad_input within the suite's
    bar of autograd's, decided against the float64 truth where fp32 orders differ."""
    from mpgnn_amd.model import linear
    torch.manual_seed(0)
    lin = torch.nn.Linear(f_in, f_out).to(DEV)
    x = torch.randn(n, f_in, device=DEV, requires_grad=True)
    g = torch.randn(n, f_out, device=DEV)
    ref = lin(x)
    ref.backward(g)
    ref_grads = [x.grad.clone(), lin.weight.grad.clone(), lin.bias.grad.clone()]
    x.grad = None
    lin.zero_grad()
    out = linear(lin, x)
    # truth: the same products in float64
    x64, g64, w64 = x.detach().double().cpu(), g.double().cpu(), lin.weight.detach().double().cpu()
    rel_close(out, ref, what="out", ref64=x64 @ w64.t() + lin.bias.detach().double().cpu())
    out.backward(g)
    truth = [g64 @ w64, g64.t() @ x64, g64.sum(0)]
    for got, want, t64, what in zip([x.grad, lin.weight.grad, lin.bias.grad], ref_grads, truth, ["dx", "dW", "db"]):
        rel_close(got, want, what=what, ref64=t64)


@pytest.mark.parametrize("mode", [MODE_SINGLE, MODE_ALL])
def test_chunk_rows_option_moves_only_slab_boundaries(mode):
    """MPGNN_OPT_CHUNK_ROWS (rows per weight-gradient reduction chunk) moves slab boundaries,
    i.e. the fp32 order of the dW / droot / dbias sums: every gradient within 1e-4 of the
    default chunking."""
    from mpgnn_amd import _lib
    from mpgnn_amd.plan import plan_cache
    g = data.config_graph("fb15k237")
    R = g.num_relations
    gen = torch.Generator().manual_seed(6)
    W = torch.rand((R, 128, 128) if mode == MODE_ALL else (128, 128), generator=gen) - 0.5
    root, bias = torch.rand(128, 128, generator=gen) - 0.5, torch.rand(128, generator=gen) - 0.5
    gout = torch.randn(g.num_nodes, 128, generator=gen).to(DEV)

    def run():
        plan = mpgnn_amd.GraphPlan(g.edge_index, g.edge_type, g.num_nodes)
        xg = g.x.to(DEV).requires_grad_(True)
        ps = [t.to(DEV).requires_grad_(True) for t in (W, root, bias)]
        out = rgcn_conv(xg, *ps, plan, mode, relation=3, num_relations=R)
        out.backward(gout)
        return [t.grad.clone() for t in [xg] + ps]

    r32, r64 = oracle_layer2(g.x, g.edge_index, g.edge_type, W, root, bias, gout.cpu(), mode=mode, rel=3)
    shipped = _lib.get_option(20)
    assert shipped == 256
    try:
        for rows in (shipped, 192, 64, 512):  # the shipped default first
            _lib.set_option(20, rows)
            plan_cache.clear()
            got = run()
            close_all(dict(zip(("dx", "dW", "droot", "dbias"), got)), r32, r64, f"chunk rows {rows} ")
    finally:
        _lib.set_option(20, shipped)
        plan_cache.clear()


@pytest.mark.parametrize("name,mode,rel", [("C1", MODE_ALL, -1), ("C1", MODE_SINGLE, 1), ("fb15k237", MODE_ALL, -1),
                                           ("fb15k237", MODE_SINGLE, 3), ("fb15k237", MODE_SINGLE, 10_000)])
def test_segment_means_backward_vs_oracle(name, mode, rel):
    """mpgnn_rel_mean_bwd (autograd of segment_means) vs the oracle's autograd through PyG's
    mean (index_select / scatter_add_ / div, mp_rgcn_layer.py:236), 1e-4; an absent relation
    gives dx = 0."""
    g = data.config_graph(name)
    R = g.num_relations
    plan = mpgnn_amd.GraphPlan(g.edge_index, g.edge_type, g.num_nodes)
    xg = g.x.to(DEV).requires_grad_(True)
    h = segment_means(xg, plan, mode, rel, R)
    dh = torch.randn(h.shape, generator=torch.Generator().manual_seed(2))
    h.backward(dh.to(DEV))
    b, e = plan.select(mode, rel, R)
    s_row = torch.from_numpy(plan.table("s_row")[b:e].astype(np.int64))
    s_rel = plan.table("s_rel")[b:e]
    grads = {}
    for dt in (torch.float32, torch.float64):
        xs = g.x.detach().to(dt, copy=True).requires_grad_(True)
        loss = torch.zeros((), dtype=dt)
        for r in np.unique(s_rel):
            hr = orc.segment_means(xs, g.edge_index, g.edge_type, int(r))
            m = torch.from_numpy(s_rel == r)
            loss = loss + (hr[s_row[m]] * dh[m].to(dt)).sum()
        if len(s_rel):
            loss.backward()
            grads[dt] = xs.grad
    if len(s_rel):
        rel_close(xg.grad, grads[torch.float32], what="dx", ref64=grads[torch.float64])
    else:
        assert torch.count_nonzero(xg.grad) == 0


@pytest.mark.parametrize("world", [2, 4])
def test_shard_forward_reads_only_own_rows(world):
    """distributed.sharded_stack_forward leaves every row outside a rank's node_2 range
    unwritten between layers: a shard's partial forward must not read them. Poisoning those
    rows with NaN changes no bit of the partial output."""
    from mpgnn_amd.distributed import shard_ranges
    g = data.config_graph("fb15k237")
    torch.manual_seed(30)
    conv = mpgnn_amd.RGCNConv(128, 128, g.num_relations, flow="target_to_source").to(DEV)
    x, ei, et = g.x.to(DEV), g.edge_index.to(DEV), g.edge_type.to(DEV)
    for lo, hi in shard_ranges(g.edge_index, g.num_nodes, world):
        with torch.no_grad():
            clean = conv(x, ei, et, shard=(lo, hi))
            xp = torch.full_like(x, float("nan"))
            xp[lo:hi] = x[lo:hi]
            poisoned = conv(xp, ei, et, shard=(lo, hi))
        assert torch.equal(clean, poisoned), (lo, hi)


@pytest.mark.parametrize("world", [2, 4])
def test_row_shards_complete_rows_and_sum_to_unsharded(world):
    """shard_side="rows" (plan sharded by the aggregating node): each rank's output rows in its
    range equal the unsharded layer's, rows outside it are exactly zero, so the sum over ranks
    (the all-reduce of the training path) is the unsharded output; gradients summed over ranks
    match the unsharded gradients."""
    from mpgnn_amd.distributed import shard_ranges
    g, conv, gout, r32, r64 = fb_layer_case(30, 128, 4)
    x, ei, et = g.x.to(DEV), g.edge_index.to(DEV), g.edge_type.to(DEV)
    gout = gout.to(DEV)
    total = torch.zeros(g.num_nodes, 128, device=DEV)
    sums = {k: None for k in ("dx", "dW", "droot", "dbias")}
    for lo, hi in shard_ranges(g.edge_index, g.num_nodes, world, side="rows"):
        conv.zero_grad()
        xs = x.clone().requires_grad_(True)
        part = conv(xs, ei, et, shard=(lo, hi), shard_side="rows")
        part.backward(gout)
        assert torch.count_nonzero(part[:lo]) == 0 and torch.count_nonzero(part[hi:]) == 0
        rel_close(part[lo:hi], r32["out"][lo:hi], what="own rows", ref64=r64["out"][lo:hi])
        total += part.detach()
        for k, gr in zip(sums, [xs.grad, conv.weight.grad, conv.root.grad, conv.bias.grad]):
            sums[k] = gr.clone() if sums[k] is None else sums[k] + gr
    sums["out"] = total
    close_all(sums, r32, r64, f"{world} row shards ")


@pytest.mark.parametrize("n,f_out,root_weight", [(40, 1, True), (1, 8, True), (40, 1, False), (1, 8, False)])
def test_squeeze_edge_cases_match_reference(n, f_out, root_weight):
    """mp_rgcn_layer.py:246 squeezes `zeros + h @ W` before the in-place root add (:265): with a
    root weight, F_out == 1 or N == 1 makes the reference raise RuntimeError, and so must the
    drop-in; without one, the squeezed output is returned — same shape and values."""
    gen = torch.Generator().manual_seed(n + f_out)
    ei = torch.randint(0, n, (2, 3 * n), generator=gen)
    et = torch.randint(0, 2, (3 * n,), generator=gen)
    x = torch.rand(n, 6, generator=gen)
    torch.manual_seed(30)
    conv = mpgnn_amd.CustomRGCNConv(6, f_out, 1, root_weight=root_weight, flow="target_to_source")
    W = conv.weight.detach().clone()
    root = conv.root.detach().clone() if root_weight else None
    bias = conv.bias.detach().clone()
    try:
        ref = orc.custom_rgcn_forward(x, ei, et, 1, W, root, bias)
        ref64 = orc.custom_rgcn_forward(x.double(), ei, et, 1, W.double(), None if root is None else root.double(),
                                        bias.double())
        ref_err = None
    except RuntimeError as e:
        ref, ref_err = None, e
    conv = conv.to(DEV)
    if ref_err is not None:
        with pytest.raises(RuntimeError):
            conv(0, 1, x.to(DEV), ei.to(DEV), et.to(DEV))
    else:
        out = conv(0, 1, x.to(DEV), ei.to(DEV), et.to(DEV))
        assert out.shape == ref.shape
        rel_close(out, ref, what="squeezed output", ref64=ref64)


@pytest.mark.parametrize("n,offset", [(14541 * 128, 0), (1001, 0), (1003, 1), (3, 0), (0, 0)])
def test_relu_bwd_matches_threshold_backward(n, offset):
    """mpgnn_relu_bwd = torch's ReLU backward (threshold_backward: 0 where the output is not > 0,
    even for inf / NaN gradients), bit-exact, on aligned (float4) and misaligned (scalar) buffers."""
    from mpgnn_amd import _lib
    gen = torch.Generator().manual_seed(7)
    g = torch.randn(n + offset, generator=gen)
    y = torch.relu(torch.randn(n + offset, generator=gen))
    if n > 8:
        g[:4] = torch.tensor([float("nan"), float("inf"), -float("inf"), float("nan")])
        # NaN / -0.0 / inf OUTPUTS: threshold_backward passes grad where the output is NaN
        y[offset + 4: offset + 8] = torch.tensor([float("nan"), -0.0, float("inf"), float("nan")])
    g, y = g.to(DEV)[offset:], y.to(DEV)[offset:]
    d = torch.full((n + offset,), 7.0, device=DEV)[offset:]
    _lib.check(_lib.lib.mpgnn_relu_bwd(g.data_ptr(), y.data_ptr(), n, d.data_ptr(), None), "mpgnn_relu_bwd")
    torch.cuda.synchronize()
    ref = torch.ops.aten.threshold_backward(g, y, 0.0)
    assert torch.equal(torch.nan_to_num(d, nan=123.0), torch.nan_to_num(ref, nan=123.0))


@pytest.mark.parametrize("n,f,o,bias", [(14541, 128, 2, True), (1000, 128, 64, True), (5, 256, 32, False),
                                        (3000, 64, 128, True), (700, 512, 4, True), (14541, 128, 128, True),
                                        (50, 128, 128, True), (70001, 128, 128, False)])
def test_linear_head_gradients_vs_autograd(n, f, o, bias):
    """model.linear (the wrappers' heads, model.py:147 / :224-226): forward and all gradients vs
    plain autograd of F.linear, 1e-4 — the C-ABI mpgnn_linear_wgrad path (F <= 256) and the
    sliced-GEMM fallback (F = 512)."""
    from mpgnn_amd.model import linear
    gen = torch.Generator().manual_seed(11)
    layer = torch.nn.Linear(f, o, bias=bias).to(DEV)
    x = torch.randn(n, f, generator=gen).to(DEV).requires_grad_(True)
    go = torch.randn(n, o, generator=gen).to(DEV)
    out = linear(layer, x)
    out.backward(go)
    got = [x.grad.clone(), layer.weight.grad.clone()] + ([layer.bias.grad.clone()] if bias else [])
    x.grad = None
    layer.zero_grad(set_to_none=True)
    ref_out = torch.nn.functional.linear(x, layer.weight, layer.bias)
    ref_out.backward(go)
    ref = [x.grad, layer.weight.grad] + ([layer.bias.grad] if bias else [])
    # the float64 truth of the same products (the suite's elementwise bar, decided against it
    # where the two fp32 summation orders differ at a cancellation)
    x64 = x.detach().cpu().double().requires_grad_(True)
    w64 = layer.weight.detach().cpu().double().requires_grad_(True)
    b64 = layer.bias.detach().cpu().double().requires_grad_(True) if bias else None
    o64 = torch.nn.functional.linear(x64, w64, b64)
    o64.backward(go.cpu().double())
    t64 = [x64.grad, w64.grad] + ([b64.grad] if bias else [])
    rel_close(out, ref_out, what=f"linear {n}x{f}->{o} out", ref64=o64.detach())
    for a, b, t, nm in zip(got, ref, t64, ("dx", "dW", "dbias")):
        rel_close(a, b, what=f"linear {n}x{f}->{o} {nm}", ref64=t)


@pytest.mark.parametrize("n,f,o,bias,relu", [(14541, 128, 2, True, False), (333, 64, 5, False, True),
                                             (1000, 256, 8, True, True), (7, 4, 1, True, False)])
def test_linear_small_head_abi_vs_torch(n, f, o, bias, relu):
    """mpgnn_linear_fwd / mpgnn_linear_dgrad for heads with O <= 8 through the C ABI directly:
    act(x @ Wᵀ + b) and g @ W against torch at the suite's bar, the float64 truth deciding; the
    forward (float64 sums, one rounding) IS the float64 truth rounded to fp32 but for rare
    near-half-ulp cases."""
    from mpgnn_amd import _lib
    gen = torch.Generator().manual_seed(21)
    x = torch.randn(n, f, generator=gen)
    w = torch.randn(o, f, generator=gen) * 0.1
    b = torch.randn(o, generator=gen) if bias else None
    go = torch.randn(n, o, generator=gen)
    xd, wd, gd = x.to(DEV), w.to(DEV), go.to(DEV)
    bd = b.to(DEV) if bias else None
    out = torch.empty(n, o, device=DEV)
    gx = torch.empty(n, f, device=DEV)
    _lib.check(_lib.lib.mpgnn_linear_fwd(xd.data_ptr(), n, f, wd.data_ptr(), o, bd.data_ptr() if bias else None,
                                         _lib.ACT_RELU if relu else _lib.ACT_NONE, out.data_ptr(), None), "fwd")
    _lib.check(_lib.lib.mpgnn_linear_dgrad(gd.data_ptr(), n, o, wd.data_ptr(), f, gx.data_ptr(), None), "dgrad")
    torch.cuda.synchronize()
    ref = torch.nn.functional.linear(xd, wd, bd)
    ref64 = torch.nn.functional.linear(x.double(), w.double(), b.double() if bias else None)
    if relu:
        ref, ref64 = torch.relu(ref), torch.relu(ref64)
    rel_close(out, ref, what="small head out", ref64=ref64)
    rel_close(gx, gd @ wd, what="small head dgrad", ref64=go.double() @ w.double())
    off = int((out.cpu() != ref64.float()).sum())
    assert off <= max(1, out.numel() // 10000), (off, out.numel())


@pytest.mark.parametrize("n,f,o", [(14541, 128, 128), (14541, 128, 2), (333, 64, 5), (1000, 128, 64)])
def test_linear_head_fused_relu_vs_autograd(n, f, o):
    """model.linear(..., activation='relu') = F.relu(F.linear(...)) (MPNetm's fc1, model.py:225):
    the ReLU in the head's launch (mpgnn_linear_fwd / its bias pass) and its backward through
    mpgnn_relu_bwd, forward and every gradient vs autograd at the suite's bar."""
    from mpgnn_amd.model import linear
    gen = torch.Generator().manual_seed(12)
    layer = torch.nn.Linear(f, o).to(DEV)
    x = torch.randn(n, f, generator=gen).to(DEV).requires_grad_(True)
    go = torch.randn(n, o, generator=gen).to(DEV)
    # no gradient where the pre-activation is within fp32 rounding of 0 (either ReLU mask is right)
    z64 = torch.nn.functional.linear(x.detach().cpu().double(), layer.weight.detach().cpu().double(),
                                     layer.bias.detach().cpu().double())
    go = go * (z64.abs() > 1e-4).to(DEV, torch.float32)
    out = linear(layer, x, activation="relu")
    out.backward(go)
    got = [x.grad.clone(), layer.weight.grad.clone(), layer.bias.grad.clone()]
    x.grad = None
    layer.zero_grad(set_to_none=True)
    ref_out = torch.relu(torch.nn.functional.linear(x, layer.weight, layer.bias))
    ref_out.backward(go)
    ref = [x.grad, layer.weight.grad, layer.bias.grad]
    x64 = x.detach().cpu().double().requires_grad_(True)
    w64 = layer.weight.detach().cpu().double().requires_grad_(True)
    b64 = layer.bias.detach().cpu().double().requires_grad_(True)
    o64 = torch.relu(torch.nn.functional.linear(x64, w64, b64))
    o64.backward(go.cpu().double())
    rel_close(out, ref_out, what=f"relu linear {n}x{f}->{o} out", ref64=o64.detach())
    for a, b, t, nm in zip(got, ref, [x64.grad, w64.grad, b64.grad], ("dx", "dW", "dbias")):
        rel_close(a, b, what=f"relu linear {n}x{f}->{o} {nm}", ref64=t)
    with pytest.raises(ValueError):
        linear(layer, x, activation="gelu")


# ------------------------------------------------------------------------------------------
# mode SINGLE (CustomRGCNConv, the MPGNN metapath layer) at full C2 size and on C5 rows
# ------------------------------------------------------------------------------------------
def test_mode_single_full_size_c2_fwd_bwd():
    """BASELINE.json configs[1] (N = 100 k, R = 16, 128-d), CustomRGCNConv over relation 1 on the
    whole graph — the fused layer GEMM ([x | mean] @ [root; W] + bias, one launch) — forward and
    every gradient against the oracle (mp_rgcn_layer.py:225-271) in fp32 and the float64 truth."""
    g = data.config_graph("C2")
    N = g.num_nodes
    gen = torch.Generator().manual_seed(21)
    W = (torch.rand(128, 128, generator=gen) - 0.5) * 0.2
    root = (torch.rand(128, 128, generator=gen) - 0.5) * 0.2
    bias = torch.rand(128, generator=gen) - 0.5
    gout = torch.randn(N, 128, generator=gen)
    r32, r64 = oracle_layer2(g.x, g.edge_index, g.edge_type, W, root, bias, gout, mode=MODE_SINGLE, rel=1)
    plan = mpgnn_amd.GraphPlan(g.edge_index, g.edge_type, N)
    xg = g.x.to(DEV).requires_grad_(True)
    Wg, rg, bg = (p.to(DEV).requires_grad_(True) for p in (W, root, bias))
    out = rgcn_conv(xg, Wg, rg, bg, plan, MODE_SINGLE, relation=1)
    out.backward(gout.to(DEV))
    close_all({"out": out, "dx": xg.grad, "dW": Wg.grad, "droot": rg.grad, "dbias": bg.grad}, r32, r64, "C2 single ")


@pytest.mark.parametrize("f_in", [64, 128])
@pytest.mark.parametrize("bf3", [1, 0])
def test_fused_single_layer_absent_relation_and_relu(f_in, bf3):
    """The fused mode-SINGLE layer with an absent relation (every node row is [x_i | 0]) and with
    the ReLU epilogue: x @ root + bias, and relu(layer) of the oracle — on the split-K bf16
    kernel (single_bf3_kernel, MPGNN_OPT_GEMM_BF3 = 1) and on the fp32 K = 2·F_in GEMM."""
    from mpgnn_amd import _lib
    _lib.set_option(24, bf3)
    g = data.synthetic_graph(900, 3, 8, feat_dim=f_in, seed=3 + f_in)
    torch.manual_seed(4)
    conv = mpgnn_amd.CustomRGCNConv(f_in, 128, 1, flow="target_to_source")
    with torch.no_grad():
        conv.bias.uniform_(-0.5, 0.5)
    W, root, bias = (p.detach().clone() for p in (conv.weight, conv.root, conv.bias))
    conv = conv.to(DEV)
    ei, et, xg = g.edge_index.to(DEV), g.edge_type.to(DEV), g.x.to(DEV)
    out = conv(0, 7, xg, ei, et)
    rel_close(out, g.x @ root + bias, what="absent out", ref64=g.x.double() @ root.double() + bias.double())
    for rel in (0, 2):
        r32, r64 = oracle_layer2(g.x, g.edge_index, g.edge_type, W, root, bias, None, mode=MODE_SINGLE, rel=rel)
        out = conv(0, rel, xg, ei, et, activation="relu")
        rel_close(out, torch.relu(r32["out"]), what="fused relu out", ref64=torch.relu(r64["out"]))


def test_mode_single_c5_full_size_sampled_rows():
    """BASELINE.json configs[4] (N = 2 M, 64 relations, 256-d) mode SINGLE over relation 2 on the
    whole graph; checked on 256 sampled rows against the oracle CustomRGCNConv arithmetic
    (mean over the row's relation-2 edges @ W + x @ root + bias) and the float64 truth."""
    g = data.config_graph("C5")
    N, F = g.num_nodes, g.x.shape[1]
    gen = torch.Generator().manual_seed(8)
    W = (torch.rand(F, F, generator=gen) - 0.5) * 0.1
    root = (torch.rand(F, F, generator=gen) - 0.5) * 0.1
    bias = torch.rand(F, generator=gen) - 0.5
    plan = mpgnn_amd.GraphPlan(g.edge_index, g.edge_type, N)
    with torch.no_grad():
        out = rgcn_conv(g.x.to(DEV), W.to(DEV), root.to(DEV), bias.to(DEV), plan, MODE_SINGLE, relation=2).cpu()
    rows = torch.from_numpy(np.random.default_rng(2).choice(N, 256, replace=False))
    ei, et = g.edge_index, g.edge_type
    sel = (et == 2) & torch.isin(ei[0], rows)
    src, dst = ei[0][sel], ei[1][sel]
    for dt in (torch.float32, torch.float64):
        h = torch.zeros(N, F, dtype=dt)
        h.index_add_(0, src, g.x[dst].to(dt))  # sequential per row, as scatter_add_
        cnt = torch.bincount(src, minlength=N).clamp(min=1).to(dt)
        hr = h[rows] / cnt[rows, None]
        ref = hr @ W.to(dt) + g.x[rows].to(dt) @ root.to(dt) + bias.to(dt)
        if dt == torch.float32:
            r32 = ref
        else:
            r64 = ref
    rel_close(out[rows], r32, what="C5 single sampled rows", ref64=r64)


def test_graph_captured_training_step_equals_eager():
    """One MPNetm training step (forward, NLL, backward, Adam) captured as a HIP graph on torch's
    own capture stream — the layer workspaces grow inside the capture (forward-only, then the
    backward's size) — replays bit for bit like the same step run eagerly."""
    g = data.synthetic_graph(3000, 4, 12, feat_dim=64, seed=9)
    ei, et, x = g.edge_index.to(DEV), g.edge_type.to(DEV), g.x.to(DEV)
    y = torch.randint(0, 2, (g.num_nodes,), generator=torch.Generator().manual_seed(1)).to(DEV)
    torch.manual_seed(30)
    ref = mpgnn_amd.MPNetm(64, 128, 4, 128, 2, 1, [[3, 1, 0]])
    nets = [mpgnn_amd.MPNetm(64, 128, 4, 128, 2, 1, [[3, 1, 0]]).to(DEV) for _ in range(2)]
    for n in nets:
        n.load_state_dict(ref.state_dict())
        n.eval()  # dropout off: the two runs see the same masks (none)
    opts = [torch.optim.Adam(n.parameters(), lr=0.01, weight_decay=5e-4, fused=True, capturable=True) for n in nets]

    def train_step(net, opt):
        out = net(x, ei, et)
        loss = torch.nn.functional.nll_loss(out, y)
        loss.backward()
        opt.step()
        return loss

    mpgnn_amd.functional.release_workspaces()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm-up (optimizer state, autograd) off the default stream
        opts[0].zero_grad(set_to_none=True)
        train_step(nets[0], opts[0])
    torch.cuda.current_stream().wait_stream(s)
    opts[1].zero_grad(set_to_none=True)
    train_step(nets[1], opts[1])
    torch.cuda.synchronize()
    cg = torch.cuda.CUDAGraph()
    opts[0].zero_grad(set_to_none=True)
    with torch.cuda.graph(cg):
        train_step(nets[0], opts[0])
    for _ in range(3):
        cg.replay()
        opts[1].zero_grad(set_to_none=True)
        train_step(nets[1], opts[1])
    torch.cuda.synchronize()
    for (k, a), (_, b) in zip(nets[0].state_dict().items(), nets[1].state_dict().items()):
        assert torch.equal(a, b), k
    del cg
    mpgnn_amd.functional.release_workspaces()


def test_captured_workspace_outgrown_then_replayed_equals_eager():
    """The round-3 fault's mechanism (gpurun_out/diag/kr4.err), pinned by its exact
    scenario: a training step is captured on a stream whose workspace was allocated EAGERLY;
    a larger-graph call on the same stream then outgrows that workspace; the freed block is
    re-allocated and filled with NaN; the captured step is replayed. The workspace cache must
    retire (not free) the captured buffer, so the replay equals the eager step bit for bit and
    the retired buffer is still counted by workspace_bytes_cached() until release_workspaces."""
    from mpgnn_amd import functional as fn
    small = data.synthetic_graph(3000, 5, 10, feat_dim=128, seed=3)
    big = data.synthetic_graph(40000, 7, 20, feat_dim=128, seed=4)
    torch.manual_seed(12)
    ref = mpgnn_amd.RGCNConv(128, 128, 5, flow="target_to_source")
    convs = [mpgnn_amd.RGCNConv(128, 128, 5, flow="target_to_source").to(DEV) for _ in range(2)]
    for c in convs:
        c.load_state_dict(ref.state_dict())
    big_conv = mpgnn_amd.RGCNConv(128, 128, 7, flow="target_to_source").to(DEV)
    xs, eis, ets = small.x.to(DEV), small.edge_index.to(DEV), small.edge_type.to(DEV)
    xb, eib, etb = big.x.to(DEV), big.edge_index.to(DEV), big.edge_type.to(DEV)
    wsum = torch.randn(small.num_nodes, 128, generator=torch.Generator().manual_seed(2)).to(DEV)
    xg = [xs.clone().requires_grad_(True) for _ in range(2)]

    def step(k):
        out = convs[k](xg[k], eis, ets, activation="relu")
        (out * wsum).sum().backward()

    fn.release_workspaces()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step(0)  # eager: the stream's workspace is allocated here, outside any capture
        torch.cuda.synchronize()
        before = fn.workspace_bytes_cached()
        cg = torch.cuda.CUDAGraph()
        for c in (convs[0],):
            c.zero_grad(set_to_none=False)
        xg[0].grad.zero_()
        with torch.cuda.graph(cg, stream=s):
            step(0)  # captured: uses the eagerly allocated buffer
        # a larger graph on the same stream outgrows the captured buffer
        with torch.no_grad():
            big_out = big_conv(xb, eib, etb)
        torch.cuda.synchronize()
        grown = fn.workspace_bytes_cached()
        assert grown > before, (grown, before)
        # whatever the allocator now hands out of freed blocks is poisoned: a tensor of the
        # captured buffer's size would take that buffer's block had it been freed, and the
        # replay would then write into it
        poison = [torch.full((n,), float("nan"), device=DEV) for n in (before // 4, before // 8, before // 16)]
        for c in (convs[0],):
            c.zero_grad(set_to_none=False)
        xg[0].grad.zero_()
        cg.replay()
        torch.cuda.synchronize()
    torch.cuda.current_stream().wait_stream(s)
    step(1)  # the same step, eager, on the default stream
    torch.cuda.synchronize()
    for a, b, name in ((xg[0].grad, xg[1].grad, "grad_x"), (convs[0].weight.grad, convs[1].weight.grad, "dW"),
                       (convs[0].root.grad, convs[1].root.grad, "droot"), (convs[0].bias.grad, convs[1].bias.grad, "dbias")):
        assert bool(torch.isfinite(a).all()), name
        assert torch.equal(a, b), name
    for p_ in poison:
        assert bool(torch.isnan(p_).all()), "the replay wrote into memory the allocator had handed out again"
    assert fn.workspace_bytes_cached() >= grown  # the retired buffer outlives the graph's replays
    del cg, poison, big_out
    fn.release_workspaces(s)
    assert not any(k[1] == s.cuda_stream for k in list(fn._WS) + list(fn._RETIRED))


@pytest.mark.parametrize("act", [None, "relu"])
def test_mode_single_256_root_epilogue_fwd_bwd(act):
    """Mode SINGLE at F_in = F_out = 256 (C5's width): the wide GEMM finishes the rows without a
    segment of the relation in its root epilogue ((0 + x_i @ root) + bias, ReLU) and
    single_fix_kernel adds Y to the rows with one. Whole-graph forward and every gradient against
    the oracle CustomRGCNConv (fp32 and the float64 truth), present and absent relations, a
    700-edge hub segment."""
    g = data.synthetic_graph(6000, 4, 12, feat_dim=256, seed=17)
    hub = torch.stack([torch.full((700,), 5), torch.arange(700) % 6000])
    ei = torch.cat([g.edge_index, hub], 1)
    et = torch.cat([g.edge_type, torch.full((700,), 1)])
    N = g.num_nodes
    gen = torch.Generator().manual_seed(23)
    W = (torch.rand(256, 256, generator=gen) - 0.5) * 0.1
    root = (torch.rand(256, 256, generator=gen) - 0.5) * 0.1
    bias = torch.rand(256, generator=gen) - 0.5
    gout = torch.randn(N, 256, generator=gen)
    plan = mpgnn_amd.GraphPlan(ei.to(DEV), et.to(DEV), N)
    for rel in (1, 3, 9):  # 9: absent relation
        xg = g.x.to(DEV).requires_grad_(True)
        Wg, rg, bg = (p.to(DEV).requires_grad_(True) for p in (W, root, bias))
        out = rgcn_conv(xg, Wg, rg, bg, plan, MODE_SINGLE, relation=rel, activation=act)
        out.backward(gout.to(DEV))
        got = {"out": out, "dx": xg.grad, "dW": Wg.grad, "droot": rg.grad, "dbias": bg.grad}
        relu = kink_act([out]) if act == "relu" else None  # ReLU kinks follow the GPU's mask
        refs = {}
        for dt in (torch.float32, torch.float64):
            xr, Wr, rr, br = (t.detach().to(dt).requires_grad_(True) for t in (g.x, W, root, bias))
            o = orc.custom_rgcn_forward(xr, ei, et, rel, Wr, rr, br)
            if relu is not None:
                o = relu(0, o)
            o.backward(gout.to(dt))
            refs[dt] = {"out": o.detach(), "dx": xr.grad, "dW": Wr.grad, "droot": rr.grad, "dbias": br.grad}
        for k in got:
            rel_close(got[k], refs[torch.float32][k], what=f"256 single rel {rel} {act} {k}", ref64=refs[torch.float64][k])


@pytest.mark.parametrize("f_in,f_out", [(96, 64), (128, 256), (64, 36), (32, 6)])
def test_mode_single_streaming_combine_widths(f_in, f_out):
    """Mode SINGLE at widths neither the fused layer nor the root epilogue takes: the transform,
    then single_combine_kernel (one wave per row through the node -> segment map; F_out % 4 != 0
    keeps the gather-rows combine) — forward with ReLU against the oracle."""
    g = data.synthetic_graph(3000, 3, 9, feat_dim=f_in, seed=31 + f_in)
    gen = torch.Generator().manual_seed(f_out)
    W = (torch.rand(f_in, f_out, generator=gen) - 0.5) * 0.2
    root = (torch.rand(f_in, f_out, generator=gen) - 0.5) * 0.2
    bias = torch.rand(f_out, generator=gen) - 0.5
    plan = mpgnn_amd.GraphPlan(g.edge_index.to(DEV), g.edge_type.to(DEV), g.num_nodes)
    for rel in (0, 2, 7):  # 7: absent
        with torch.no_grad():
            out = rgcn_conv(g.x.to(DEV), W.to(DEV), root.to(DEV), bias.to(DEV), plan, MODE_SINGLE, relation=rel,
                            activation="relu")
        act = kink_act([out])
        r32 = act(0, orc.custom_rgcn_forward(g.x, g.edge_index, g.edge_type, rel, W, root, bias))
        r64 = act(0, orc.custom_rgcn_forward(g.x.double(), g.edge_index, g.edge_type, rel, W.double(), root.double(),
                                             bias.double()))
        rel_close(out, r32, what=f"single combine {f_in}x{f_out} rel {rel}", ref64=r64)


def _adam_case(dev, contract_sizes=((37, 128, 128), (128, 128), (128,), (2, 128), (2,), (5, 3))):
    g = torch.Generator().manual_seed(7)
    return [torch.nn.Parameter(torch.randn(*s, generator=g).to(dev)) for s in contract_sizes]


@pytest.mark.gpu
@pytest.mark.parametrize("capturable", [False, True])
def test_adam_step_bit_identical_to_torch(capturable):
    """mpgnn_adam_step (LeanAdam's step on the GPU: step counters + ATen's fused update in one
    launch, csrc/optim_kernels.hip) = torch.optim.Adam(fused=True) bit for bit — parameters,
    exp_avg, exp_avg_sq, step — over 6 steps with fresh gradients, tensors whose sizes are and
    are not multiples of 4. The default fma-contraction variant (MPGNN_OPT_ADAM_CONTRACT) is the
    one that matches torch's build; the other is reported for the record."""
    import ctypes
    from mpgnn_amd import _lib, main
    dev = torch.device("cuda", 0)
    kw = dict(lr=0.01, weight_decay=5e-4, fused=True, capturable=capturable)
    v0 = ctypes.c_int64()
    _lib.check(_lib.lib.mpgnn_get_option(_lib.OPT_ADAM_CONTRACT, ctypes.byref(v0)), "get")
    match = {}
    try:
        for contract in (int(v0.value), 1 - int(v0.value)):
            _lib.check(_lib.lib.mpgnn_set_option(_lib.OPT_ADAM_CONTRACT, contract), "set")
            pa, pb = _adam_case(dev), _adam_case(dev)
            oa, ob = torch.optim.Adam(pa, **kw), main.LeanAdam(pb, **kw)
            gg = torch.Generator().manual_seed(11)
            for it in range(6):
                grads = [torch.randn(p.shape, generator=gg).to(dev) * (10.0 ** (it - 3)) for p in pa]
                for ps, o in ((pa, oa), (pb, ob)):
                    for p, gr in zip(ps, grads):
                        p.grad = gr.clone()
                    o.step()
                if it >= 1:
                    assert getattr(ob, "_hip_cache", None) is not None, "the HIP step did not run"
            torch.cuda.synchronize()
            ok = all(torch.equal(p, q) and all(torch.equal(oa.state[p][k], ob.state[q][k])
                                               for k in ("exp_avg", "exp_avg_sq", "step"))
                     for p, q in zip(pa, pb))
            match[contract] = ok
    finally:
        _lib.check(_lib.lib.mpgnn_set_option(_lib.OPT_ADAM_CONTRACT, int(v0.value)), "restore")
    print(f"adam contraction variants bit-identical to torch: {match}")
    assert match[int(v0.value)], match


@pytest.mark.gpu
@pytest.mark.parametrize("name,hidden,classes", [("C1", 64, 5), ("fb15k237", 128, 2)])
def test_net_relu_backward_fused_bit_identical(name, hidden, classes, monkeypatch):
    """Net's ReLU backwards fused into the consumers' input-gradient kernels (grad_x of the next
    conv: mpgnn_rgcn_bwd_relu_in, the head: mpgnn_linear_logsoftmax_bwd's relu_in) give every parameter
    gradient bit for bit as the separate relu_bwd launches (MPGNN_RELU_FUSE=0), with no
    relu_bwd launch left; a forward hook on a conv turns the fusion off (its output observable)."""
    import mpgnn_amd.functional as fnl
    from mpgnn_amd import _lib
    from mpgnn_amd import model as mdl
    g = data.config_graph(name)
    F = g.x.shape[1]
    torch.manual_seed(10)
    net = mpgnn_amd.Net(F, hidden, g.num_relations, hidden, classes, 3).to(DEV)
    gout = torch.randn(g.num_nodes, classes, generator=torch.Generator().manual_seed(3)).to(DEV)
    x, ei, et = g.x.to(DEV), g.edge_index.to(DEV), g.edge_type.to(DEV)
    calls = {}
    real = _lib.lib

    class _Count:
        def __getattr__(self, k):
            f = getattr(real, k)

            def wrapped(*a):
                calls[k] = calls.get(k, 0) + 1
                return f(*a)
            return wrapped
    monkeypatch.setattr(fnl, "lib", _Count())
    monkeypatch.setattr(_lib, "lib", _Count())

    def grads(fuse, hook=False):
        monkeypatch.setattr(mdl, "_RELU_FUSE", fuse)
        calls.clear()
        net.zero_grad(set_to_none=True)
        h = net.conv2.register_forward_hook(lambda *_: None) if hook else None
        out = net(x, ei, et)
        if h is not None:
            h.remove()
        out.backward(gout)
        torch.cuda.synchronize()
        return {k: p.grad.clone() for k, p in net.named_parameters()}, dict(calls)

    ref, c_ref = grads(False)
    got, c_got = grads(True)
    hooked, c_hook = grads(True, hook=True)
    assert c_ref.get("mpgnn_relu_bwd", 0) == 3 and c_hook.get("mpgnn_relu_bwd", 0) == 3, (c_ref, c_hook)
    assert c_got.get("mpgnn_relu_bwd", 0) == 0, c_got
    # conv2's two uses (C1, F = 64: the accumulating call is refused, then a fresh one: three calls)
    assert c_got.get("mpgnn_rgcn_bwd_relu_in", 0) >= 2, c_got
    # the head (Net.lin + log_softmax, one fused backward) takes the last layer's ReLU mask
    assert c_got.get("mpgnn_linear_logsoftmax_bwd", 0) == 1, c_got
    for k in ref:
        assert torch.equal(ref[k], got[k]), k
        assert torch.equal(ref[k], hooked[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("n,f,o,relu_in", [(14541, 128, 2, True), (1000, 64, 5, False), (37, 16, 8, True),
                                           (300, 256, 3, False)])
def test_head_log_softmax_vs_torch(n, f, o, relu_in):
    """model.head_log_softmax (Net.lin + F.log_softmax, model.py:147-148: mpgnn_linear_fwd with
    MPGNN_ACT_LOG_SOFTMAX, mpgnn_linear_logsoftmax_bwd) against torch's F.linear + F.log_softmax
    in float64: the log-probabilities, grad_input (with the input's ReLU backward fused when the
    input is tagged internal, against relu's autograd) and the weight / bias gradients, within
    the suite's fp32 bars."""
    from mpgnn_amd import model as mdl
    gen = torch.Generator().manual_seed(n + f + o)
    lin = torch.nn.Linear(f, o).to(DEV)
    pre = torch.randn(n, f, generator=gen).to(DEV).requires_grad_(True)
    x = torch.relu(pre) if relu_in else pre * 1.0
    gout = torch.randn(n, o, generator=gen).to(DEV)
    if relu_in:
        x._mpgnn_relu_internal = True
    out = mdl.head_log_softmax(lin, x)
    out.backward(gout)
    # float64 truth through torch's autograd
    pre64 = pre.detach().double().requires_grad_(True)
    w64 = lin.weight.detach().double().requires_grad_(True)
    b64 = lin.bias.detach().double().requires_grad_(True)
    x64 = torch.relu(pre64) if relu_in else pre64 * 1.0
    ref = torch.nn.functional.log_softmax(torch.nn.functional.linear(x64, w64, b64), dim=1)
    ref.backward(gout.double())
    for what, got, want in (("logp", out, ref), ("grad_input", pre.grad, pre64.grad),
                            ("grad_weight", lin.weight.grad, w64.grad), ("grad_bias", lin.bias.grad, b64.grad)):
        err = normwise_err(got.double().cpu(), want.detach().cpu())
        assert err <= 1e-5, (what, err)


@pytest.mark.gpu
def test_mpnetm_dropout_relu_backward_fused_bit_identical(monkeypatch):
    """MPNetm in training mode (Dropout(0.6) after each metapath layer's ReLU, model.py:211-215):
    with the ReLU outputs internal, each dropout's backward and the ReLU backward of the layer
    before it run as ONE launch (mpgnn_dropout_relu_bwd) and fc1's ReLU backward fuses into the
    head's (no relu_bwd launch left); the forward draws the same dropout masks (torch's own
    native_dropout, the kernel and random stream F.dropout uses) — every parameter gradient bit
    for bit as MPGNN_RELU_FUSE=0 under the same seed; a forward hook turns it off."""
    from mpgnn_amd import _lib
    from mpgnn_amd import model as mdl
    import mpgnn_amd.functional as fnl
    g = data.synthetic_graph(3000, 4, 12, feat_dim=64, seed=9)
    ei, et, x = g.edge_index.to(DEV), g.edge_type.to(DEV), g.x.to(DEV)
    y = torch.randint(0, 2, (g.num_nodes,), generator=torch.Generator().manual_seed(1)).to(DEV)
    torch.manual_seed(30)
    net = mpgnn_amd.MPNetm(64, 128, 4, 128, 2, 1, [[3, 1, 0]]).to(DEV).train()
    calls = {}
    real = _lib.lib

    class _Count:
        def __getattr__(self, k):
            f = getattr(real, k)

            def wrapped(*a):
                calls[k] = calls.get(k, 0) + 1
                return f(*a)
            return wrapped
    monkeypatch.setattr(fnl, "lib", _Count())
    monkeypatch.setattr(_lib, "lib", _Count())

    def grads(fuse, hook=False):
        monkeypatch.setattr(mdl, "_RELU_FUSE", fuse)
        calls.clear()
        net.zero_grad(set_to_none=True)
        h = net.fc1.register_forward_hook(lambda *_: None) if hook else None
        torch.manual_seed(123)  # the same dropout masks in every run
        out = net(x, ei, et)
        if h is not None:
            h.remove()
        torch.nn.functional.nll_loss(out, y).backward()
        torch.cuda.synchronize()
        return {k: p.grad.clone() for k, p in net.named_parameters()}, dict(calls)

    ref, c_ref = grads(False)
    got, c_got = grads(True)
    hooked, c_hook = grads(True, hook=True)
    assert c_ref.get("mpgnn_relu_bwd", 0) == 4 and c_hook.get("mpgnn_relu_bwd", 0) == 4, (c_ref, c_hook)
    assert c_got.get("mpgnn_relu_bwd", 0) == 0 and c_got.get("mpgnn_dropout_relu_bwd", 0) == 3, c_got
    for k in ref:
        assert torch.equal(ref[k], got[k]), k
        assert torch.equal(ref[k], hooked[k]), k
