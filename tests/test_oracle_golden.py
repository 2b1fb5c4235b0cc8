"""CPU: pin the oracle (oracle/rgcn_oracle.py) against the reference's own outputs.

* layer_single.npz / layer_all.npz / mpnetm_synthetic.npz were produced by running the
  reference mp_rgcn_layer.py / model.py (tests/golden/make_golden.py).
* kat_synthetic.npz holds the planted ground truth the reference ships with its synthetic
  graphs (embedding.dat / label.dat): it pins the edge direction of
  flow='target_to_source', the relation masking and "rows without edges aggregate to 0".
"""
import numpy as np
import pytest
import torch

from oracle import rgcn_oracle as orc


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def close(a, b, tol=1e-6):
    """Reductions over N rows (dW, droot) depend on the BLAS thread count; compare with a
    scale-aware tolerance |a-b| <= tol*|b| + tol*max|b|."""
    scale = float(b.abs().max()) if b.numel() else 0.0
    torch.testing.assert_close(a, b, rtol=tol, atol=tol * max(scale, 1e-30))


@pytest.mark.parametrize("F_in", [2, 128])
@pytest.mark.parametrize("rel", [0, 1, 2, 3])
def test_single_forward_and_grads_match_reference(golden, F_in, rel):
    g = golden("layer_single.npz")
    ei, et = t(g["edge_index"]), t(g["edge_type"])
    x = t(g[f"F{F_in}_x"]).requires_grad_(True)
    W = t(g[f"F{F_in}_weight"]).requires_grad_(True)
    root = t(g[f"F{F_in}_root"]).requires_grad_(True)
    bias = t(g[f"F{F_in}_bias"]).requires_grad_(True)
    out = orc.custom_rgcn_forward(x, ei, et, rel, W, root, bias)
    # bit-exact: same ATen ops in the same order as the reference
    assert torch.equal(out.detach(), t(g[f"F{F_in}_r{rel}_out"]))
    h = orc.segment_means(x.detach(), ei, et, rel)
    assert torch.equal(h, t(g[f"F{F_in}_r{rel}_h"]))
    assert np.array_equal(orc.masked_edge_index(ei, et == rel).numpy(), g[f"F{F_in}_r{rel}_masked"])
    out.backward(t(g[f"F{F_in}_gout"]))
    for name, p in (("dx", x), ("dweight", W), ("droot", root), ("dbias", bias)):
        close(p.grad, t(g[f"F{F_in}_r{rel}_{name}"]))


@pytest.mark.parametrize("F_in", [2, 128])
def test_all_forward_and_grads_match_reference(golden, F_in):
    g = golden("layer_all.npz")
    ei, et = t(g["edge_index"]), t(g["edge_type"])
    x = t(g[f"F{F_in}_x"]).requires_grad_(True)
    W = t(g[f"F{F_in}_weight"]).requires_grad_(True)
    root = t(g[f"F{F_in}_root"]).requires_grad_(True)
    bias = t(g[f"F{F_in}_bias"]).requires_grad_(True)
    out = orc.rgcn_forward(x, ei, et, W, root, bias)
    assert torch.equal(out.detach(), t(g[f"F{F_in}_out"]))
    out.backward(t(g[f"F{F_in}_gout"]))
    for name, p in (("dx", x), ("dweight", W), ("droot", root), ("dbias", bias)):
        close(p.grad, t(g[f"F{F_in}_{name}"]))


def test_mpnetm_logits_match_reference(golden):
    g = golden("mpnetm_synthetic.npz")
    kat = golden("kat_synthetic.npz")
    link = kat["L3_link"]
    ei = t(np.stack([link[:, 0], link[:, 2]]))
    et = t(link[:, 1])
    params = {k[3:]: t(g[k]) for k in g.files if k.startswith("sd.")}
    logits = orc.mpnetm_forward(params, t(g["x"]), ei, et, [[1, 0]])
    assert torch.equal(logits, t(g["logits"]))


@pytest.mark.parametrize("tag", ["L3", "L4"])
def test_planted_metapath_kat(golden, tag):
    """SURVEY §4 KAT: x = [colour == blue]; aggregate over relation 1 into edge_index[0];
    (>0) AND red == embedding column 1; aggregate that over relation 0, (>0) == column 2 ==
    label.dat."""
    kat = golden("kat_synthetic.npz")
    link, node = kat[f"{tag}_link"], kat[f"{tag}_node"]
    emb, label = kat[f"{tag}_embedding"], kat[f"{tag}_label"]
    N = node.shape[0]
    ei = t(np.stack([link[:, 0], link[:, 2]]))
    et = t(link[:, 1])
    red, blue = node[:, 1] == 1, node[:, 2] == 1
    rel_first, rel_second = kat[f"{tag}_metapath_rel"]          # "1 0"
    x = t(blue.astype(np.float32)[:, None])
    h1 = orc.propagate_mean(orc.masked_edge_index(ei, et == rel_first), x, (N, N)).numpy()[:, 0]
    hop1 = (h1 > 0) & red
    assert np.array_equal(hop1.astype(np.int64), emb[:, 1])
    h2 = orc.propagate_mean(orc.masked_edge_index(ei, et == rel_second),
                            t(hop1.astype(np.float32)[:, None]), (N, N)).numpy()[:, 0]
    hop2 = h2 > 0
    assert np.array_equal(hop2.astype(np.int64), emb[:, 2])
    assert np.array_equal(hop2.astype(np.int64)[label[:, 0]], label[:, 1])
    # rows with no edge of the relation aggregate to exactly 0 (count clamped to 1)
    deg = np.bincount(link[link[:, 1] == rel_first, 0], minlength=N)
    assert np.all(h1[deg == 0] == 0.0)


def test_seeded_init_matches_reference_state_dict(golden):
    """Drop-in property: MPNetm built from our layers with torch.manual_seed(30) (main.py:31)
    has the reference's exact parameters (same shapes, names, order and glorot draws)."""
    import mpgnn_amd
    g = golden("mpnetm_synthetic.npz")
    torch.manual_seed(30)
    net = mpgnn_amd.MPNetm(2, 64, 4, 64, 2, 1, [[1, 0]])
    sd = net.state_dict()
    ref_keys = [k[3:] for k in g.files if k.startswith("sd.")]
    assert list(sd.keys()) == ref_keys
    for k in ref_keys:
        assert torch.equal(sd[k], t(g["sd." + k])), k


def test_seeded_init_single_layer(golden):
    import mpgnn_amd
    g = golden("layer_single.npz")
    for F_in in (2, 128):
        torch.manual_seed(30)
        conv = mpgnn_amd.CustomRGCNConv(F_in, 64, 1, flow="target_to_source")
        assert torch.equal(conv.weight.detach(), t(g[f"F{F_in}_weight"]))
        assert torch.equal(conv.root.detach(), t(g[f"F{F_in}_root"]))
        assert torch.equal(conv.bias.detach(), t(g[f"F{F_in}_bias"]))


def test_fast_rgcn_oracle_equals_loop_oracle():
    """CustomFastRGCNConv's transform-then-aggregate arithmetic
    (mp_rgcn_layer.py:324-357, 3-D weight) equals the RGCNConv loop (A6) up to summation order;
    rows without edges get x@root + bias only."""
    from mpgnn_amd import data
    g = data.synthetic_graph(400, 4, 8, feat_dim=24, seed=5)
    torch.manual_seed(0)
    w, root, bias = torch.randn(4, 24, 16), torch.randn(24, 16), torch.randn(16)
    a = orc.rgcn_forward(g.x, g.edge_index, g.edge_type, w, root, bias)
    b = orc.fast_rgcn_forward(g.x, g.edge_index, g.edge_type, w, root, bias)
    assert torch.allclose(a, b, rtol=1e-5, atol=1e-5)
    # one relation absent from the graph, one isolated row
    keep = (g.edge_type != 2) & (g.edge_index[0] != 7)
    ei, et = g.edge_index[:, keep], g.edge_type[keep]
    a = orc.rgcn_forward(g.x, ei, et, w, root, bias)
    b = orc.fast_rgcn_forward(g.x, ei, et, w, root, bias)
    assert torch.allclose(a, b, rtol=1e-5, atol=1e-5)
    assert torch.allclose(b[7], g.x[7] @ root + bias, rtol=1e-6, atol=1e-6)
