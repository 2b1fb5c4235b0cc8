"""Training-loop drop-in: the native link.dat reader, the device-side
scores against scikit-learn, the loop's host logic with a CPU oracle model, and (GPU) the
loops of main.py / main_rgcn.py against the same loop run on the CPU oracle."""
import os

import numpy as np
import pytest
import torch
from sklearn.metrics import f1_score
from sklearn.utils import class_weight as skl_class_weight

import mpgnn_amd
from mpgnn_amd import data, main, main_rgcn, metrics
from oracle import rgcn_oracle as orc

DEV = "cuda"


# ------------------------------------------------------------------------------------------
# native link.dat reader (main.py:150-151,366-372)
# ------------------------------------------------------------------------------------------
def _write(path, text):
    with open(path, "w", newline="") as f:
        f.write(text)


@pytest.mark.parametrize("graph", ["L3", "L4"])
def test_load_links_matches_reference_layout_on_kat_graphs(tmp_path, golden, graph):
    """The reference's own link.dat rows (KAT fixture) parse to the tensors
    get_edge_index_and_type_no_reverse builds: row 0 = node_1, row 1 = node_2, file order."""
    rows = golden("kat_synthetic.npz")[f"{graph}_link"]
    p = tmp_path / "link.dat"
    np.savetxt(p, rows, fmt="%d", delimiter="\t")
    ei, et = data.load_links(str(p))
    assert ei.dtype == torch.int64 and et.dtype == torch.int64
    assert np.array_equal(ei.numpy(), np.stack([rows[:, 0], rows[:, 2]]))
    assert np.array_equal(et.numpy(), rows[:, 1])
    # and the pandas path of the reference (load_files + get_edge_index_and_type_no_reverse)
    import pandas as pd
    links = pd.read_csv(p, sep="\t", header=None).rename(columns={0: "node_1", 1: "relation_type", 2: "node_2"})
    ei2, et2 = main.get_edge_index_and_type_no_reverse(links)
    assert torch.equal(ei, ei2) and torch.equal(et, et2)


def test_load_links_edge_cases(tmp_path):
    p = str(tmp_path / "l.dat")
    _write(p, "")
    ei, et = data.load_links(p)
    assert ei.shape == (2, 0) and et.shape == (0,)
    # CRLF, blank lines, spaces, no trailing newline, integral floats, negative ids kept
    _write(p, "1\t2\t3\r\n\n  4 5\t6  \n\t\n7\t8\t9.0\n-1\t0\t2")
    ei, et = data.load_links(p)
    assert ei.tolist() == [[1, 4, 7, -1], [3, 6, 9, 2]] and et.tolist() == [2, 5, 8, 0]
    for bad in ("1\t2\n", "1\t2\t3\t4\n", "1\tx\t3\n", "1\t2\t3.5\n"):
        _write(p, "0\t0\t0\n" + bad)
        with pytest.raises(ValueError):
            data.load_links(p)
    with pytest.raises(ValueError):
        data.load_links(str(tmp_path / "missing.dat"))


def test_load_links_large_file_multithreaded(tmp_path):
    """> 1 MiB so the reader splits the file over several threads; boundaries are exact."""
    rng = np.random.default_rng(3)
    rows = np.stack([rng.integers(0, 10**6, 200_000), rng.integers(0, 237, 200_000),
                     rng.integers(0, 10**6, 200_000)], 1)
    p = tmp_path / "big.dat"
    np.savetxt(p, rows, fmt="%d", delimiter="\t")
    assert os.path.getsize(p) > (3 << 20)
    ei, et = data.load_links(str(p))
    assert np.array_equal(ei.numpy(), np.stack([rows[:, 0], rows[:, 2]])) and np.array_equal(et.numpy(), rows[:, 1])


@pytest.mark.parametrize("graph", ["L3", "L4"])
def test_node_features_column_order_per_reference_driver(tmp_path, golden, graph):
    """main.py:347-355 keeps get_dummies' column order (its flip, main.py:353, is commented
    out); main_rgcn.py:345-353 reverses the columns (main_rgcn.py:351). Run both loaders on
    the reference's own node.dat rows (KAT fixture) through load_files, as the drivers do."""
    node = golden("kat_synthetic.npz")[f"{graph}_node"]
    label = golden("kat_synthetic.npz")[f"{graph}_label"]
    link = golden("kat_synthetic.npz")[f"{graph}_link"]
    for name, rows in (("node.dat", node), ("label.dat", label), ("link.dat", link)):
        np.savetxt(tmp_path / name, rows, fmt="%d", delimiter="\t")
    labels, features, links, _, nrel = main.load_files(str(tmp_path / "node.dat"), str(tmp_path / "link.dat"),
                                                       str(tmp_path / "label.dat"))
    cols = node[:, 1:].astype(np.float32)
    x_mpgnn = main.get_node_features(features)
    x_rgcn = main_rgcn.get_node_features(features)
    assert x_mpgnn.dtype == torch.float32 and x_rgcn.dtype == torch.float32
    assert np.array_equal(x_mpgnn.numpy(), cols)
    assert np.array_equal(x_rgcn.numpy(), cols[:, ::-1])
    assert not np.array_equal(x_mpgnn.numpy(), x_rgcn.numpy())  # the two drivers really differ here
    # native readers (csrc/io.cpp) give the same matrices and labels
    assert torch.equal(data.load_node_features(str(tmp_path / "node.dat")), x_mpgnn)
    assert torch.equal(data.load_node_features(str(tmp_path / "node.dat"), flip=True), x_rgcn)
    ids, y = data.load_labels(str(tmp_path / "label.dat"))
    assert np.array_equal(ids.numpy(), label[:, 0]) and torch.equal(y, labels)
    assert nrel == np.unique(link[:, 1]).size


def test_tsv_reader_edge_cases(tmp_path):
    p = str(tmp_path / "n.dat")
    _write(p, "")
    assert data.read_tsv_numeric(p).shape == (0, 0)
    # ragged rows pad with NaN (pandas read_csv), floats / exponents / signs, CRLF, blank lines,
    # an empty middle field and a trailing tab (NaN fields in place: the split is on single tabs,
    # as read_csv(sep='\t') of main.py:140-147 cuts them), spaces around a number
    _write(p, "0\t1.5\t-2e3\t\r\n\n1\t\t+4\n2\t 0.25 \t7\t\n")
    a = data.read_tsv_numeric(p)
    assert a.shape == (3, 4)
    assert a[0, 2] == -2000 and np.isnan(a[1, 1]) and a[1, 2] == 4 and a[2, 1] == 0.25 and a[2, 2] == 7
    assert np.isnan(a[:, 3]).all()
    import pandas as pd
    ref = pd.read_csv(p, sep="\t", header=None).to_numpy(dtype=np.float64)
    assert np.array_equal(np.isnan(a), np.isnan(ref)) and np.array_equal(np.nan_to_num(a), np.nan_to_num(ref))
    for bad in ("0\tred\n", "1\t2x\n", "1\t2 3\n"):  # a space never separates fields
        _write(p, bad)
        with pytest.raises(ValueError):
            data.read_tsv_numeric(p)
    _write(p, "0\t1.5\n")
    with pytest.raises(ValueError):
        data.load_labels(p)
    with pytest.raises(ValueError):
        data.read_tsv_numeric(str(tmp_path / "missing.dat"))


def test_tsv_reader_large_file_multithreaded(tmp_path):
    rng = np.random.default_rng(5)
    a = np.concatenate([np.arange(150_000)[:, None], rng.random((150_000, 4)) * 100], 1)
    p = tmp_path / "big.dat"
    np.savetxt(p, a, fmt=["%d"] + ["%.17g"] * 4, delimiter="\t")
    assert os.path.getsize(p) > (3 << 20)
    assert np.array_equal(data.read_tsv_numeric(str(p)), a)  # %.17g round-trips float64 exactly


# ------------------------------------------------------------------------------------------
# scores and loss weights (main.py:1062-1098, main_rgcn.py:376-415)
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("seed", range(8))
def test_f1_macro_identical_to_sklearn(seed):
    rng = np.random.default_rng(seed)
    c = int(rng.integers(2, 12))
    n = int(rng.integers(1, 400))
    y = rng.integers(0, c, n)
    pred = rng.integers(0, c, n) if seed % 2 else np.where(rng.random(n) < 0.7, y, rng.integers(0, c, n))
    if seed == 3:
        pred[:] = 0  # a class predicted nowhere / present nowhere
    ref = f1_score(pred.tolist(), y.tolist(), average="macro")  # the reference's argument order
    got = metrics.f1_macro(torch.from_numpy(pred), torch.from_numpy(y), c)
    assert got == ref, (got, ref)
    many = metrics.f1_macro_many([(torch.from_numpy(pred), torch.from_numpy(y)),
                                  (torch.from_numpy(y), torch.from_numpy(pred))], c)
    assert many == [ref, f1_score(y.tolist(), pred.tolist(), average="macro")]


def _rows_case(seed, c, n_rows):
    """Log-probability-like scores with ties and NaN rows, label lists with out-of-range labels
    and repeated rows."""
    g = torch.Generator().manual_seed(seed)
    s = torch.randn(n_rows, c, generator=g)
    s[::7] = s[::7].round()  # ties: the first maximum wins
    s[5::11, c // 2] = float("nan")  # a NaN wins (torch.argmax)
    if c > 1:
        s[3::13] = 0.0  # a whole row tied
    lists = []
    for k, n in enumerate((n_rows // 2, 1, 0, n_rows + 5)):
        idx = torch.randint(0, n_rows, (n,), generator=g)
        y = torch.randint(-1, c + 1, (n,), generator=g)  # -1 and c count in no class
        lists.append((idx.to(torch.int32) if k == 1 else idx, y))
    return s, lists


@pytest.mark.parametrize("seed,c", [(0, 2), (1, 3), (2, 1), (3, 40)])
def test_confusion_counts_rows_cpu_equals_argmax_counts(seed, c):
    s, lists = _rows_case(seed, c, 300)
    got = metrics.confusion_counts_rows(s, lists)
    ref = metrics.confusion_counts_many([(torch.argmax(s[i.long()], 1), y) for i, y in lists], c)
    assert torch.equal(got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,c", [(0, 2), (1, 3), (2, 1), (3, 40), (4, 700)])
def test_confusion_counts_rows_kernel_equals_torch(seed, c):
    """mpgnn_confusion_counts (one launch) = torch.argmax over the listed rows + the per-class
    counts of metrics.confusion_counts_many, integer-exact; and the macro F1 from them equals
    scikit-learn's on the same predictions (main.py:1094-1098)."""
    s, lists = _rows_case(seed, c, 3000)
    dev = torch.device("cuda", 0)
    sd = s.to(dev)
    ld = [(i.to(dev), y.to(dev)) for i, y in lists]
    got = metrics.confusion_counts_rows(sd, ld)
    ref = metrics.confusion_counts_many([(torch.argmax(sd[i.long()], 1), y) for i, y in ld], c)
    assert got.is_cuda and torch.equal(got, ref)
    pred = torch.argmax(s[lists[0][0]], 1)
    y = lists[0][1]
    keep = (y >= 0) & (y < c)
    if keep.any():
        assert metrics.f1_from_counts(metrics.confusion_counts_rows(sd, [(ld[0][0][keep.to(dev)],
                                                                          ld[0][1][keep.to(dev)])]))[0] == \
            f1_score(pred[keep].tolist(), y[keep].tolist(), average="macro")


def test_confusion_counts_rows_range_check():
    """a row list with an out-of-range entry fails the one-time check, so the GPU path
    hands it to torch's ops (whose indexing rejects it like the reference's pred[idx]); a list
    in range is remembered per object and version."""
    idx = torch.tensor([0, 4, 9])
    assert metrics._rows_valid(idx, 10)
    assert not metrics._rows_valid(torch.tensor([0, 10]), 10)
    assert not metrics._rows_valid(torch.tensor([-1, 3]), 10)
    idx[1] = 12  # in-place change: the cached verdict no longer applies
    assert not metrics._rows_valid(idx, 10)
    assert metrics._rows_valid(torch.empty(0, dtype=torch.int64), 0)


@pytest.mark.gpu
def test_confusion_counts_rows_wide_classes_take_torch():
    """C above the kernel's LDS histograms (4096) runs torch's counts (same values) instead of
    failing the launch."""
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(6)
    wide = torch.randn(300, 5000, generator=g).to(dev)
    idx = torch.randperm(300, generator=g)[:200].to(dev)
    y = torch.randint(0, 5000, (200,), generator=g).to(dev)
    got = metrics.confusion_counts_rows(wide, [(idx, y)])
    ref = metrics.confusion_counts_many([(torch.argmax(wide[idx], 1), y)], 5000)
    assert torch.equal(got, ref)


def _nll_case(seed, rows, c, n, dup=False, ignore=False):
    """log_softmax rows (requires grad through the softmax input), a row list (repeated rows when
    dup) and targets (some ignore_index -100 when ignore)."""
    g = torch.Generator().manual_seed(seed)
    h = torch.randn(rows, c, generator=g) * 3
    idx = torch.randint(0, rows, (n,), generator=g) if dup else torch.randperm(rows, generator=g)[:n]
    y = torch.randint(0, c, (n,), generator=g)
    if ignore and n:
        y[torch.rand(n, generator=g) < 0.2] = -100
    return h, idx, y


def test_nll_loss_rows_cpu_is_torch():
    h, idx, y = _nll_case(0, 50, 3, 20)
    logp = torch.log_softmax(h, 1)
    assert torch.equal(metrics.nll_loss_rows(logp, idx, y), torch.nn.functional.nll_loss(logp[idx], y))


@pytest.mark.gpu
@pytest.mark.parametrize("seed,rows,c,n,dup,ignore", [(0, 14541, 2, 4847, False, False), (1, 3000, 5, 2500, True, True),
                                                      (2, 70, 2, 0, False, False), (3, 9, 3, 9, False, True),
                                                      (4, 5000, 40, 4000, True, False)])
def test_nll_loss_rows_kernel_vs_torch(seed, rows, c, n, dup, ignore):
    """metrics.nll_loss_rows on the GPU (mpgnn_nll_rows_fwd / _bwd) against torch's
    F.nll_loss(log_softmax(h)[idx], y) (main.py:1065, 1088): the loss within a few ulp (summation
    order), the gradient of the softmax input bit for bit — repeated rows, ignore_index entries
    and the empty list (NaN loss, zero gradient) included."""
    h, idx, y = _nll_case(seed, rows, c, n, dup, ignore)
    dev = torch.device("cuda", 0)
    hd, idx_d, y_d = h.to(dev), idx.to(dev), y.to(dev)
    ha = hd.clone().requires_grad_(True)
    hb = hd.clone().requires_grad_(True)
    la = metrics.nll_loss_rows(torch.log_softmax(ha, 1), idx_d, y_d)
    assert la.grad_fn is not None and "NllRows" in type(la.grad_fn).__name__
    lb = torch.nn.functional.nll_loss(torch.log_softmax(hb, 1).index_select(0, idx_d), y_d)
    la.backward()
    lb.backward()
    if n == 0 or bool((y == -100).all()):
        assert torch.isnan(la) and torch.isnan(lb)
    else:
        assert torch.allclose(la, lb, rtol=4e-7 * max(1.0, n ** 0.5), atol=0), (float(la), float(lb))
    assert torch.equal(ha.grad, hb.grad)
    with torch.no_grad():  # the validation loss: forward only, the same launch
        lv = metrics.nll_loss_rows(torch.log_softmax(hd, 1), idx_d, y_d)
        assert torch.equal(lv, la.detach()) or bool(torch.isnan(la))


@pytest.mark.gpu
@pytest.mark.parametrize("seed,rows,c,n,dup,ignore", [(0, 14541, 2, 4847, False, False), (1, 3000, 5, 2500, True, True),
                                                      (4, 5000, 40, 4000, True, False)])
def test_nll_loss_rows_class_weighted_vs_torch(seed, rows, c, n, dup, ignore):
    """metrics.nll_loss_rows(..., weight=w) on the GPU (mpgnn_nll_rows_fwd_weighted and the dense
    / scatter backward with class weights) against F.nll_loss(..., weight=w) — main_rgcn.py's
    training loss (main_rgcn.py:376-380): the loss within the summation-order bar, the gradient
    of the softmax input within 1e-6 of its largest entry (torch's per-pair value is -(w·(g /
    total_weight)) too; repeated rows are summed in another order)."""
    h, idx, y = _nll_case(seed, rows, c, n, dup, ignore)
    dev = torch.device("cuda", 0)
    w = (torch.rand(c, generator=torch.Generator().manual_seed(seed + 7)) + 0.25).to(dev)
    hd, idx_d, y_d = h.to(dev), idx.to(dev), y.to(dev)
    ha = hd.clone().requires_grad_(True)
    hb = hd.clone().requires_grad_(True)
    la = metrics.nll_loss_rows(torch.log_softmax(ha, 1), idx_d, y_d, weight=w)
    assert la.grad_fn is not None and "NllRows" in type(la.grad_fn).__name__
    lb = torch.nn.functional.nll_loss(torch.log_softmax(hb, 1).index_select(0, idx_d), y_d, weight=w)
    la.backward()
    lb.backward()
    assert torch.allclose(la, lb, rtol=1e-6 * max(1.0, n ** 0.5), atol=0), (float(la), float(lb))
    # repeated rows: torch sums their addends through index_add's atomics, the kernel in row order
    scale = float(hb.grad.abs().max())
    assert torch.allclose(ha.grad, hb.grad, rtol=1e-6, atol=1e-6 * scale), float((ha.grad - hb.grad).abs().max())


@pytest.mark.gpu
def test_nll_loss_rows_out_of_range_lists_take_torchs_path():
    """A row or target outside the matrix fails the one-time list check (the call then runs
    torch's ops, which raise torch's error, instead of the kernels); ignore_index passes."""
    dev = torch.device("cuda", 0)
    logp = torch.log_softmax(torch.randn(10, 3, device=dev), 1)
    idx = torch.tensor([0, 4, 12], device=dev)
    y = torch.tensor([0, 1, 2], device=dev)
    assert not metrics._nll_lists_valid(idx, y, 10, 3)
    assert not metrics._nll_lists_valid(idx[:2], torch.tensor([0, 3], device=dev), 10, 3)
    assert metrics._nll_lists_valid(idx[:2], torch.tensor([0, -100], device=dev), 10, 3)
    assert logp.shape == (10, 3)


def test_nll_loss_rows_fallback_raises_torchs_errors():
    if os.environ.get("MPGNN_LIB_PATH", "").endswith("_asan.so"):
        pytest.skip("a torch C++ exception aborts under the preloaded sanitizer runtime (test_host_sanitizers)")
    logp = torch.log_softmax(torch.randn(10, 3), 1)
    with pytest.raises(IndexError):
        metrics.nll_loss_rows(logp, torch.tensor([0, 4, 12]), torch.tensor([0, 1, 2]))
    with pytest.raises(IndexError):
        metrics.nll_loss_rows(logp, torch.tensor([0, 4]), torch.tensor([0, 3]))


def test_class_weight_balanced_identical_to_sklearn():
    for seed in range(4):
        y = torch.from_numpy(np.random.default_rng(seed).integers(0, 3 + seed, 97))
        ref = skl_class_weight.compute_class_weight("balanced", classes=np.unique(y.numpy()), y=y.tolist())
        assert np.array_equal(metrics.class_weight_balanced(y), ref)
        assert np.array_equal(metrics.class_weight_balanced(y), ref)  # cached answer


def test_class_weight_cache_keyed_on_the_tensor_object():
    """A new label tensor at a recycled address (same numel, _version 0) must not hit the
    previous tensor's cached weights (the cache was keyed on data_ptr)."""
    buf = torch.tensor([0, 0, 0, 1], dtype=torch.int64)
    w1 = metrics.class_weight_balanced(buf)
    alias = buf.view(-1)  # another tensor object over the same storage and address
    alias.copy_(torch.tensor([0, 1, 1, 1]))  # bumps the shared version counter too
    w2 = metrics.class_weight_balanced(alias)
    assert np.array_equal(w2, skl_class_weight.compute_class_weight("balanced", classes=np.array([0, 1]),
                                                                    y=[0, 1, 1, 1]))
    assert not np.array_equal(w1, w2)
    y3 = torch.tensor([1, 1, 1, 0], dtype=torch.int64).as_strided((4,), (1,))
    assert np.array_equal(metrics.class_weight_balanced(y3), w2)  # same class counts as alias


# ------------------------------------------------------------------------------------------
# loop host logic with the CPU oracle as the model (no GPU)
# ------------------------------------------------------------------------------------------
class _OracleNet(torch.nn.Module):
    """model.py:Net restated by the oracle (CPU), with Net's parameter names."""

    def __init__(self, params, layers):
        super().__init__()
        self.p = torch.nn.ParameterDict({k.replace(".", "__"): torch.nn.Parameter(v.clone()) for k, v in params.items()})
        self.layers = layers

    def forward(self, x, edge_index, edge_type):
        params = {k.replace("__", "."): v for k, v in self.p.items()}
        return orc.net_forward(params, x, edge_index, edge_type, self.layers)


def _task(g, classes=3, seed=1):
    gen = torch.Generator().manual_seed(seed)
    y = torch.randint(0, classes, (g.num_nodes,), generator=gen)
    perm = torch.randperm(g.num_nodes, generator=gen)
    n = g.num_nodes
    tr, va, te = perm[: n // 2], perm[n // 2: 3 * n // 4], perm[3 * n // 4:]
    return main.Data(x=g.x, edge_index=g.edge_index, edge_type=g.edge_type, train_idx=tr, train_y=y[tr],
                     val_idx=va, val_y=y[va], test_idx=te, test_y=y[te])


def _net_params(g, f_in, hidden, classes, seed=30):
    torch.manual_seed(seed)
    r = g.num_relations
    gl = lambda *s: torch.nn.init.xavier_uniform_(torch.empty(*s)) if len(s) == 2 else \
        torch.stack([torch.nn.init.xavier_uniform_(torch.empty(*s[1:])) for _ in range(s[0])])  # noqa: E731
    return {"conv1.weight": gl(r, f_in, hidden), "conv1.root": gl(f_in, hidden), "conv1.bias": torch.zeros(hidden),
            "conv2.weight": gl(r, hidden, hidden), "conv2.root": gl(hidden, hidden), "conv2.bias": torch.zeros(hidden),
            "LinearLayer.weight": gl(classes, hidden), "LinearLayer.bias": torch.zeros(classes)}


def test_rgcn_loop_functions_on_cpu_oracle_model():
    g = data.synthetic_graph(300, 3, 6, feat_dim=16, seed=2)
    d = _task(g)
    net = _OracleNet(_net_params(g, 16, 32, 3), 2)
    opt = torch.optim.Adam(net.parameters(), lr=0.01, weight_decay=0.0005)
    losses = []
    for _ in range(4):
        loss, w = main_rgcn.mpgnn_train(net, opt, d)
        losses.append(loss)
        f1_tr, f1_v, f1_v2, lv = main_rgcn.mpgnn_validation(net, d, w)
        assert 0.0 <= f1_tr <= 1.0 and f1_v == f1_v2 and torch.is_tensor(lv)
        # scores equal scikit-learn on the reference's list path
        pred = net(d.x, d.edge_index, d.edge_type)
        ref = f1_score(torch.argmax(pred[d.val_idx], 1).tolist(), d.val_y.tolist(), average="macro")
        assert f1_v == ref
    assert np.array_equal(w, skl_class_weight.compute_class_weight("balanced", classes=np.unique(d.train_y.numpy()),
                                                                   y=d.train_y.tolist()))
    assert losses[-1] < losses[0]
    lt, f1_t = main_rgcn.mpgnn_test(net, d, w)
    assert 0.0 <= f1_t <= 1.0


# ------------------------------------------------------------------------------------------
# GPU: the loops vs the same loop on the CPU oracle
# ------------------------------------------------------------------------------------------
@pytest.mark.gpu
def test_rgcn_epochs_track_oracle_loop():
    """main_rgcn.py:456-461 epochs (weighted NLL, Adam) with Net on the GPU vs _OracleNet on
    the CPU from the same parameters: the loss trajectory agrees to 1e-4 relative for the
    first epochs (Adam amplifies rounding noise of ~0 gradients later, see test_gpu_parity)."""
    g = data.config_graph("C1")
    d = _task(g)
    torch.manual_seed(30)
    net = mpgnn_amd.Net(128, 64, g.num_relations, 64, 3, 2)
    ref = _OracleNet({k: v.detach() for k, v in net.state_dict().items()}, 2)
    netg = net.to(DEV)
    dg = d.to(DEV)
    opt = torch.optim.Adam(netg.parameters(), lr=0.01, weight_decay=0.0005)
    opt_ref = torch.optim.Adam(ref.parameters(), lr=0.01, weight_decay=0.0005)
    for epoch in range(3):
        loss, w = main_rgcn.mpgnn_train(netg, opt, dg)
        loss_ref, w_ref = main_rgcn.mpgnn_train(ref, opt_ref, d)
        assert np.array_equal(w, w_ref)
        assert abs(loss - loss_ref) <= 1e-4 * abs(loss_ref), (epoch, loss, loss_ref)
        _, _, _, lv = main_rgcn.mpgnn_validation(netg, dg, w)
        _, _, _, lv_ref = main_rgcn.mpgnn_validation(ref, d, w_ref)
        assert abs(float(lv) - float(lv_ref)) <= 1e-4 * abs(float(lv_ref))


@pytest.mark.gpu
def test_mpgnn_parallel_multiple_x_learns_planted_metapath(golden, capsys):
    """main.py:1138-1160 on the reference's planted synthetic graph (KAT fixture, metapath
    length 3): training MPNetm over the planted metapath reaches a high test macro F1, and the
    reference's printed line is produced."""
    z = golden("kat_synthetic.npz")
    link, node, label = z["L3_link"], z["L3_node"], z["L3_label"]
    ei = torch.from_numpy(np.stack([link[:, 0], link[:, 2]]))
    et = torch.from_numpy(link[:, 1].copy())
    n = node.shape[0]
    x = torch.from_numpy(node[:, 1:].astype(np.float32))  # one-hot colours (red, blue)
    y = torch.zeros(n, dtype=torch.int64)
    y[torch.from_numpy(label[:, 0])] = torch.from_numpy(label[:, 1])
    perm = torch.randperm(n, generator=torch.Generator().manual_seed(0))
    tr, va, te = perm[: n * 6 // 10], perm[n * 6 // 10: n * 8 // 10], perm[n * 8 // 10:]
    d = main.Data(x=x, edge_index=ei, edge_type=et, train_idx=tr, train_y=y[tr], val_idx=va, val_y=y[va],
                  test_idx=te, test_y=y[te]).to(DEV)
    torch.manual_seed(30)
    mp = [int(r) for r in z["L3_metapath_rel"]]  # layer 0 aggregates over mp[0] (model.py:210)
    f1 = main.mpgnn_parallel_multiple_x(d, x.shape[1], 64, int(et.max()) + 1, 64, 2, mp, True, epochs=200)
    out = capsys.readouterr().out
    assert "test loss" in out
    print(out, f1)
    assert f1 > 0.9, f1
    val = main.mpgnn_parallel_multiple(d, x.shape[1], 64, int(et.max()) + 1, 64, 2, [mp], epochs=3)
    assert 0.0 <= val <= 1.0


@pytest.mark.gpu
def test_metapath_fanout_single_rank_trains_each_candidate(golden):
    """main.py:1430-1452 on one rank: every candidate metapath is trained with
    mpgnn_parallel_multiple and scored; the planted metapath is among the best."""
    from mpgnn_amd import distributed as mdist
    z = golden("kat_synthetic.npz")
    link, node, label = z["L3_link"], z["L3_node"], z["L3_label"]
    n = node.shape[0]
    y = torch.zeros(n, dtype=torch.int64)
    y[torch.from_numpy(label[:, 0])] = torch.from_numpy(label[:, 1])
    perm = torch.randperm(n, generator=torch.Generator().manual_seed(0))
    tr, va, te = perm[: n * 6 // 10], perm[n * 6 // 10: n * 8 // 10], perm[n * 8 // 10:]
    d = main.Data(x=torch.from_numpy(node[:, 1:].astype(np.float32)),
                  edge_index=torch.from_numpy(np.stack([link[:, 0], link[:, 2]])),
                  edge_type=torch.from_numpy(link[:, 1].copy()), train_idx=tr, train_y=y[tr], val_idx=va,
                  val_y=y[va], test_idx=te, test_y=y[te]).to(DEV)
    planted = [int(r) for r in z["L3_metapath_rel"]]
    cands = [planted, [0, 0], [2, 1], [1]]
    torch.manual_seed(30)
    scores = mdist.metapath_fanout(d, 2, 64, int(link[:, 1].max()) + 1, 64, 2, cands, epochs=150)
    assert set(scores) == {str(c) for c in cands}
    assert all(0.0 <= v <= 1.0 for v in scores.values())
    best = mdist.best_metapaths(scores, k=1)
    assert scores[str(planted)] == max(scores.values()), scores
    assert list(best) == [str(planted)] or scores[list(best)[0]] == scores[str(planted)]


@pytest.mark.gpu
def test_rgcn_loop_graph_replay_equals_eager(capsys, monkeypatch):
    """mpgnn_parallel_multiple (main_rgcn.py:452-472) replays one captured HIP graph per epoch
    after three eager ones (main._epochs): Net has no dropout, so the replayed epochs compute
    exactly what the eager loop computes — the printed losses / scores and the returned test F1
    are identical with MPGNN_LOOP_GRAPH=0 and =1."""
    g = data.config_graph("C1")
    d = _task(g).to(DEV)
    outs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("MPGNN_LOOP_GRAPH", flag)
        torch.manual_seed(30)
        f1 = main_rgcn.mpgnn_parallel_multiple(d, 128, 64, g.num_relations, 64, 3, 2, epochs=30)
        outs.append((f1, capsys.readouterr().out))
    assert outs[0] == outs[1], outs
    assert outs[0][1].count("train loss") == 3


@pytest.mark.gpu
def test_loops_release_their_workspace_between_calls():
    """Each drop-in loop owns the scratch buffers of its side stream (main._epochs releases
    them once its HIP graph is gone): calling main.mpgnn_parallel_multiple and
    main_rgcn.mpgnn_parallel_multiple again and again leaves torch.cuda.memory_allocated and the
    workspace cache where the first call left them (main.py:1371-1373 trains one model per
    metapath candidate in one process; a buffer kept per call would grow without bound)."""
    from mpgnn_amd.functional import workspace_bytes_cached
    g = data.fb15k237_graph(feat_dim=128, seed=0, recipe="survey")
    d = _task(g, classes=2).to(DEV)
    counts = torch.bincount(g.edge_type, minlength=g.num_relations)
    mp = [int(v) for v in torch.argsort(counts, descending=True, stable=True)[:3]]
    runs = [lambda: main.mpgnn_parallel_multiple(d, 128, 128, g.num_relations, 128, 2, [mp], epochs=6),
            lambda: main_rgcn.mpgnn_parallel_multiple(d, 128, 128, g.num_relations, 128, 2, 3, epochs=6,
                                                      verbose=False)]
    for run in runs:
        torch.manual_seed(30)
        run()  # plan built + cached, default-stream scratch sized
        torch.cuda.synchronize()
        base, base_ws = torch.cuda.memory_allocated(), workspace_bytes_cached()
        for _ in range(3):
            run()
            torch.cuda.synchronize()
            assert torch.cuda.memory_allocated() == base, (torch.cuda.memory_allocated(), base)
            assert workspace_bytes_cached() == base_ws, (workspace_bytes_cached(), base_ws)


@pytest.mark.gpu
def test_interleaved_loops_keep_the_outer_graph_valid():
    """two _epochs loops interleaved on one device. The inner loop must not
    release the shared side stream's scratch buffers under the outer loop's captured graph — it
    runs eagerly instead — and the outer loop's replayed epochs still equal the eager ones."""
    g = data.config_graph("C1")
    d = _task(g).to(DEV)
    big = data.synthetic_graph(20000, 5, 12, feat_dim=128, seed=8)
    xb, eib, etb = big.x.to(DEV), big.edge_index.to(DEV), big.edge_type.to(DEV)

    def make(seed):
        torch.manual_seed(seed)
        net = mpgnn_amd.Net(d.x.shape[1], 64, g.num_relations, 64, 3, 3).to(DEV)
        return net, main._adam_graphable(net)

    def epoch_fn(net, opt):
        def fn():
            loss, _ = main._train_step(net, opt, d)
            return loss
        return fn
    net_a, opt_a = make(30)
    ref_a, ref_opt = make(30)
    losses_ref = [float(epoch_fn(ref_a, ref_opt)()) for _ in range(8)]
    gen_a = main._epochs(epoch_fn(net_a, opt_a), 8, True)
    losses = [float(next(gen_a)[1]) for _ in range(5)]  # 3 eager + capture + 1 replay
    conv = mpgnn_amd.RGCNConv(128, 128, 5, flow="target_to_source").to(DEV)

    def inner():
        (conv(xb, eib, etb) ** 2).mean().backward()
        return torch.zeros(())
    for _ in main._epochs(inner, 6, True):  # a larger graph on the same device, mid-loop
        pass
    losses += [float(v) for _, v in gen_a]
    assert losses == losses_ref, (losses, losses_ref)


def _lean_case(device, capturable=False):
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(16, 8), torch.nn.ReLU(), torch.nn.Linear(8, 3)).to(device)
    return m


@pytest.mark.parametrize("capturable", [False, pytest.param(True, marks=pytest.mark.gpu)])
def test_lean_adam_bit_identical_to_torch_fused_adam(capturable):
    """main.LeanAdam (the loops' optimizer: torch's fused Adam calls issued directly once the
    state exists) = torch.optim.Adam(fused=True) bit for bit — parameters and state — over
    several steps, through a missing-gradient step (torch's own path), zero_grad(set_to_none=
    False), a state_dict reload, and with a step pre-hook that must run once per step."""
    if capturable and not torch.cuda.is_available():
        pytest.skip("capturable fused Adam needs the GPU")
    dev = torch.device("cuda", 0) if capturable else torch.device("cpu")
    a, b = _lean_case(dev), _lean_case(dev)
    kw = dict(lr=0.01, weight_decay=5e-4, fused=True, capturable=capturable)
    oa = torch.optim.Adam(a.parameters(), **kw)
    ob = main.LeanAdam(b.parameters(), **kw)
    calls = []
    ob.register_step_pre_hook(lambda o, ar, k: calls.append(1))
    x = torch.randn(32, 16, generator=torch.Generator().manual_seed(1)).to(dev)
    for it in range(7):
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad(set_to_none=(it != 3))
            m(x).square().mean().backward()
            if it == 4:
                m[0].bias.grad = None  # a parameter without a gradient this step
            o.step()
        if it == 5:  # reload (a copy: load_state_dict keeps same-device tensors as they are)
            import copy
            ob.load_state_dict(copy.deepcopy(oa.state_dict()))
    assert len(calls) == 7
    for p, q in zip(a.parameters(), b.parameters()):
        assert torch.equal(p, q)
        for k in ("exp_avg", "exp_avg_sq", "step"):
            assert torch.equal(oa.state[p][k], ob.state[q][k]), k


def test_loops_use_lean_adam_on_gpu_params_only():
    net = torch.nn.Linear(4, 2)
    assert type(main._adam(net)) is torch.optim.Adam  # CPU parameters: torch's (unfused) Adam


def test_net_activations_internal_only_without_module_hooks():
    """Net fuses its ReLU backwards into the consumers' input-gradient kernels only while its
    activations are internal: a forward hook (sees them) or a module backward hook (sees their
    gradients) on a conv or the head, or a global one, turns the fusion off (model._hooked)."""
    from mpgnn_amd import model as mdl
    net = mpgnn_amd.Net(8, 8, 3, 8, 2, 3)
    mods = (net.conv1, net.conv2, net.LinearLayer)
    assert not mdl._hooked(*mods)
    for reg in (lambda m: m.register_forward_hook(lambda *_: None),
                lambda m: m.register_full_backward_hook(lambda *_: None),
                lambda m: m.register_full_backward_pre_hook(lambda *_: None)):
        for m in mods:
            h = reg(m)
            assert mdl._hooked(*mods)
            h.remove()
            assert not mdl._hooked(*mods)
    h = torch.nn.modules.module.register_module_full_backward_hook(lambda *_: None)
    try:
        assert mdl._hooked(*mods)
    finally:
        h.remove()
    assert not mdl._hooked(*mods)
