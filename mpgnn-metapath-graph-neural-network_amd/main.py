"""Drop-in for the MPGNN training loop of the reference ``main.py``:
the graph loaders it feeds the layers with and ``mpgnn_train`` / ``mpgnn_validation`` /
``mpgnn_test`` / ``mpgnn_parallel_multiple(_x)`` (main.py:1055-1160), driving
``MPNetm`` (model.py:179-228) whose CustomRGCNConv layers run on the gfx950 kernels.

Same names, arguments, return values and printed lines as the reference. What changes is
where things live: the model and the ``data`` tensors stay on the GPU, losses are reduced on
the device, and the macro-F1 scores are finished from per-class counts (``metrics``) instead
of Python lists — one host sync per scoring call. The metapath search driver around these
functions (main.py:1163-1460) is outside the hot path (SURVEY §2, §7 of DESIGN.md).
"""
from __future__ import annotations

import numpy as np
import torch

from . import data as _data
from .metrics import class_weight_balanced, confusion_counts_rows, f1_from_counts, nll_loss_rows
from .model import MPNetm
# score function helpers of main.py:387-917 (both branches, GPU kernels): same names, plus the
# batched first-round scoring of every relation (score_relations_batched)
from .score import (clean_bags_for_relation_type, create_bags, create_edge_dictionary,  # noqa: F401
                    get_loss, get_loss_per_node, get_model, get_optimizer, initialize_weights,
                    reinitialize_weights, retrieve_destinations_low_loss, score_relation_bags_parallel,
                    score_relation_parallel, score_relations_batched, train)

__all__ = ["Data", "load_files", "get_node_features", "get_edge_index_and_type_no_reverse",
           "load_graph", "mpgnn_train", "mpgnn_validation", "mpgnn_test",
           "mpgnn_parallel_multiple", "mpgnn_parallel_multiple_x", "EPOCHS", "create_edge_dictionary",
           "initialize_weights", "get_model", "get_optimizer", "get_loss", "get_loss_per_node", "train",
           "score_relation_parallel", "create_bags", "clean_bags_for_relation_type", "reinitialize_weights",
           "retrieve_destinations_low_loss", "score_relation_bags_parallel", "score_relations_batched"]

EPOCHS = 999  # ``for epoch in range(1, 1000)`` (main.py:1121, 1144)


class Data:
    """Attribute bag standing in for ``torch_geometric.data.Data`` as the loops use it
    (main.py:1470-1480: x, edge_index, edge_type, train_idx/_y, val_idx/_y, test_idx/_y)."""

    def __init__(self, **kw):
        self.__dict__.update(kw)

    def to(self, device) -> "Data":
        return Data(**{k: (v.to(device) if torch.is_tensor(v) else v) for k, v in self.__dict__.items()})

    def __repr__(self) -> str:
        parts = [f"{k}={list(v.shape) if torch.is_tensor(v) else v}" for k, v in self.__dict__.items()]
        return f"Data({', '.join(parts)})"


# ---------------------------------------------------------------------------------------
# loaders (A1)
# ---------------------------------------------------------------------------------------
def load_files(node_file_path, link_file_path, label_file_path):
    """main.py:174-191: (labels tensor, features DataFrame, links DataFrame, [labels],
    number of relation types). pandas frames as in the reference, for code that keeps using
    them; ``load_graph`` is the fast path to the tensors."""
    import pandas as pd
    features = pd.read_csv(node_file_path, sep="\t", header=None)
    features = features.dropna(axis=1, how="all")
    features.rename(columns={0: "node", 1: "features"}, inplace=True)
    labels_df = pd.read_csv(label_file_path, sep="\t", header=None)
    labels_df.rename(columns={0: "node", 1: "label"}, inplace=True)
    labels = torch.tensor(labels_df["label"].values)
    links = pd.read_csv(link_file_path, sep="\t", header=None)
    links.rename(columns={0: "node_1", 1: "relation_type", 2: "node_2"}, inplace=True)
    tot_relation_types = len(set(links["relation_type"].to_list()))
    return labels, features, links, [labels], tot_relation_types


def _one_hot_colours(colors) -> np.ndarray:
    """``pd.get_dummies`` of the colour frame with the 'node' column dropped, float32
    (main.py:348-352 ≡ main_rgcn.py:346-350)."""
    import pandas as pd
    node_features = pd.get_dummies(colors)
    node_features.drop(["node"], axis=1, inplace=True)
    return node_features.to_numpy().astype(np.float32)


def get_node_features(colors):
    """main.py:347-355: one-hot columns of the colour frame, float32, in ``get_dummies``
    column order. The column flip is commented out in this file (main.py:353); only the
    RGCN driver flips (``main_rgcn.get_node_features``, main_rgcn.py:351)."""
    return torch.from_numpy(np.ascontiguousarray(_one_hot_colours(colors)))


def get_edge_index_and_type_no_reverse(links):
    """main.py:366-372: links frame → (edge_index int64 [2, E] = (node_1, node_2),
    edge_type int64 [E]), file order kept."""
    n1 = np.ascontiguousarray(links["node_1"].to_numpy(dtype=np.int64))
    n2 = np.ascontiguousarray(links["node_2"].to_numpy(dtype=np.int64))
    edge_index = torch.from_numpy(np.stack([n1, n2]))
    edge_type = torch.from_numpy(np.ascontiguousarray(links["relation_type"].to_numpy(dtype=np.int64)))
    return edge_index, edge_type


def load_graph(link_file_path):
    """link.dat straight to ``get_edge_index_and_type_no_reverse``'s output through the
    library's native reader (csrc/io.cpp) — no DataFrame, no Python lists."""
    return _data.load_links(link_file_path)


# ---------------------------------------------------------------------------------------
# loop (A11)
# ---------------------------------------------------------------------------------------
# MPGNN_HIP_ADAM=0: LeanAdam issues torch's _foreach_add_ + _fused_adam_ pair (A/B switch; same values)
_HIP_ADAM = __import__("os").environ.get("MPGNN_HIP_ADAM", "1") != "0"


class LeanAdam(torch.optim.Adam):
    """``torch.optim.Adam(fused=True)`` with a short host path for the loops' steady state.

    The fused optimizer's ``step`` costs ~80-110 µs of host time per call (group bookkeeping,
    checks, per-call regrouping of the tensors by device) and ``zero_grad`` ~30 µs — at C3 mode
    SINGLE, where the eager epoch is host-bound, that is a tenth of the epoch. Once the state
    exists, this class issues the step torch's fused path computes for one device and dtype —
    on the GPU as ONE launch of the library's ``mpgnn_adam_step`` (step counters + ATen's fused
    update arithmetic over a chip-filling grid; torch's pair of launches: ``_foreach_add_`` of
    the step counters, ``_fused_adam_`` on ~120 blocks), else torch's two calls with the same
    arguments — so parameters and state are bit-identical to ``torch.optim.Adam`` (tests/
    test_loop.py, tests/test_gpu_parity.py). Anything else (several groups or devices, amsgrad, maximize, a missing
    gradient, a closure) goes through torch's own ``step``. Step hooks run as for any optimizer
    (torch wraps every optimizer class's ``step``)."""

    def _lean_lists(self):
        if len(self.param_groups) != 1:
            return None
        g = self.param_groups[0]
        if not g.get("fused") or g.get("amsgrad") or g.get("maximize") or g.get("differentiable") or \
                g.get("decoupled_weight_decay", False):
            return None
        params = g["params"]
        cache = getattr(self, "_lean_cache", None)
        # valid while the parameter list and the state objects are the ones it was made from
        # (load_state_dict replaces the state; clearing it empties the dict)
        if cache is not None and cache[0] == [id(p) for p in params] and cache[2] is self.state and \
                len(self.state) == len(params) and self.state.get(params[0]) is cache[3]:
            return cache[1]
        st = [self.state.get(p) for p in params]
        if not params or any(s is None or "exp_avg" not in s for s in st):
            return None
        dev, dt = params[0].device, params[0].dtype
        if any(p.device != dev or p.dtype != dt or p.is_complex() for p in params):
            return None
        lists = (list(params), [s["exp_avg"] for s in st], [s["exp_avg_sq"] for s in st], [s["step"] for s in st])
        self._lean_cache = ([id(p) for p in params], lists, self.state, st[0])
        return lists

    def load_state_dict(self, state_dict):
        self._lean_cache = None
        return super().load_state_dict(state_dict)

    def _torch_step(self, closure):
        # Adam.step without torch's hook wrapper (this class's own step already ran inside one)
        return getattr(torch.optim.Adam.step, "__wrapped__", torch.optim.Adam.step)(self, closure)

    @torch.no_grad()
    def step(self, closure=None):
        lists = None if closure is not None else self._lean_lists()
        # AMP: GradScaler sets grad_scale / found_inf on the optimizer; torch's step reads them
        if lists is None or getattr(self, "grad_scale", None) is not None or getattr(self, "found_inf", None) is not None:
            return self._torch_step(closure)
        params, exp_avgs, exp_avg_sqs, steps = lists
        grads = [p.grad for p in params]
        if any(gr is None or gr.is_sparse for gr in grads):
            return self._torch_step(closure)
        g = self.param_groups[0]
        beta1, beta2 = g["betas"]
        lr = g["lr"]
        if torch.is_tensor(lr) and lr.device != params[0].device:
            return self._torch_step(closure)
        if _HIP_ADAM and not torch.is_tensor(lr) and self._hip_step(lists, grads, g, float(lr), beta1, beta2):
            return None
        torch._foreach_add_(steps, 1)
        torch._fused_adam_(params, grads, exp_avgs, exp_avg_sqs, [], steps, amsgrad=False, lr=lr,
                           beta1=float(beta1), beta2=float(beta2), weight_decay=g["weight_decay"], eps=g["eps"],
                           maximize=False, grad_scale=None, found_inf=None)
        return None

    def _hip_step(self, lists, grads, g, lr, beta1, beta2) -> bool:
        """The same step as mpgnn_adam_step: ONE launch (step counters + update) instead of torch's
        two, over a grid that fills the chip (csrc/optim_kernels.hip). False (nothing launched):
        not fp32 CUDA tensors, more than 24 tensors, or a pointer not 16-byte aligned."""
        params, exp_avgs, exp_avg_sqs, steps = lists
        p0 = params[0]
        if not p0.is_cuda or p0.dtype != torch.float32 or len(params) > 24:
            return False
        from . import _lib
        from .functional import _stream
        hc = getattr(self, "_hip_cache", None)
        if hc is None or hc[0] is not lists:
            if any(not t.is_contiguous() or t.dtype != torch.float32 for t in (*params, *exp_avgs, *exp_avg_sqs)) or \
                    any(s.dtype != torch.float32 or not s.is_cuda for s in steps):
                return False
            arr = (_lib.AdamTensor * len(params))()
            for k, (p, m, v, s) in enumerate(zip(params, exp_avgs, exp_avg_sqs, steps)):
                arr[k].param, arr[k].exp_avg, arr[k].exp_avg_sq = p.data_ptr(), m.data_ptr(), v.data_ptr()
                arr[k].step, arr[k].numel = s.data_ptr(), p.numel()
            arrive = torch.zeros(1, dtype=torch.int32, device=p0.device)
            hc = self._hip_cache = (lists, arr, arrive)
        _, arr, arrive = hc
        for k, gr in enumerate(grads):
            if gr.dtype != torch.float32 or not gr.is_contiguous() or gr.device != p0.device:
                return False
            arr[k].grad = gr.data_ptr()
        st = _lib.lib.mpgnn_adam_step(arr, len(params), lr, float(beta1), float(beta2), float(g["weight_decay"]),
                                      float(g["eps"]), arrive.data_ptr(), _stream(p0))
        if st == _lib.MPGNN_ERR_UNSUPPORTED:
            return False
        _lib.check(st, "mpgnn_adam_step")
        return True

    def zero_grad(self, set_to_none: bool = True):
        if not set_to_none or self._lean_lists() is None:
            return super().zero_grad(set_to_none)
        for p in self.param_groups[0]["params"]:
            p.grad = None


def _adam(model):
    """Adam(lr=0.01, weight_decay=0.0005) of main.py:1119 / main_rgcn.py:454. On the GPU the
    fused implementation (one multi-tensor kernel per step instead of one per Adam sub-step;
    same update rule, rounding-level differences) — scripts/epoch_ab.py: 1.23 → 1.12 ms per
    FB15K epoch — behind ``LeanAdam``'s short host path."""
    params = list(model.parameters())
    fused = bool(params) and all(p.is_cuda for p in params)
    return (LeanAdam if fused else torch.optim.Adam)(params, lr=0.01, weight_decay=0.0005, fused=fused)


def _adam_graphable(model):
    """``_adam`` for a captured epoch: fused and capturable (the step counter on the device);
    the same update rule."""
    params = list(model.parameters())
    return LeanAdam(params, lr=0.01, weight_decay=0.0005, fused=True, capturable=True)


def _graphs_enabled(data) -> bool:
    import os
    return (os.environ.get("MPGNN_LOOP_GRAPH", "1") != "0" and torch.cuda.is_available() and data.x.is_cuda
            and not getattr(data, "shard_kw", None))


_LOOP_STREAMS: dict = {}
LAST_CAPTURE_ERROR = None  # why _epochs' last failed capture fell back to eager epochs
_LOOP_ACTIVE: set = set()  # devices whose loop stream a running _epochs generator owns


def _loop_stream() -> torch.cuda.Stream:
    """The side stream the loops warm up and capture on: ONE per device for the process. torch
    keeps a BLAS workspace per (handle, stream) for the process lifetime (~76 MiB each for the
    Linear heads' GEMMs on this image), so a fresh stream per loop call would leave one behind
    per call."""
    dev = torch.cuda.current_device()
    st = _LOOP_STREAMS.get(dev)
    if st is None:
        st = _LOOP_STREAMS[dev] = torch.cuda.Stream()
    return st


def _epochs(epoch_fn, epochs: int, use_graph: bool, warmup: int = 3):
    """Run ``epoch_fn`` ``epochs`` times, yielding (epoch, outputs). With ``use_graph`` the first
    ``warmup`` epochs run eagerly on a side stream, then ONE epoch is captured as a HIP graph
    (nothing executes during the capture) and replayed for the remaining epochs: every epoch
    still runs every kernel of the reference's epoch, the host only issues one launch per
    epoch. Falls back to eager epochs if the capture fails."""
    dev = torch.cuda.current_device() if use_graph else None
    if not use_graph or epochs <= warmup or dev in _LOOP_ACTIVE:
        # (a loop nested in or interleaved with another on this device runs eagerly: the shared
        # side stream's scratch buffers belong to the outer loop's captured graph, and releasing
        # them at this loop's end would free memory that graph still replays into — ADVICE r4)
        for e in range(1, epochs + 1):
            yield e, epoch_fn()
        return
    from .functional import release_workspaces
    side = _loop_stream()
    side.wait_stream(torch.cuda.current_stream())
    graph = None
    _LOOP_ACTIVE.add(dev)
    try:
        with torch.cuda.stream(side):
            for e in range(1, warmup + 1):
                out = epoch_fn()
                yield e, out
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(graph, stream=side):
                static = epoch_fn()
        except Exception as exc:  # capture unsupported here: the remaining epochs run eagerly
            global LAST_CAPTURE_ERROR
            LAST_CAPTURE_ERROR = f"{type(exc).__name__}: {exc}"
            graph = None
            torch.cuda.synchronize()
        for e in range(warmup + 1, epochs + 1):
            if graph is None:
                yield e, epoch_fn()
            else:
                graph.replay()
                yield e, static
    finally:
        # the loop owns its side stream's scratch buffers: once its graph is gone they are
        # released (the next loop's work on the stream is ordered after the last replay)
        graph = None
        side.wait_stream(torch.cuda.current_stream())
        release_workspaces(side)
        _LOOP_ACTIVE.discard(dev)


def take_rows(out: torch.Tensor, idx):
    """``out[idx]`` (main.py:1062, main_rgcn.py:380). For a 1-D integer index tensor (the loaders'
    train_idx: unique rows) this is ``index_select``: the same rows, and its backward is one
    index_add instead of advanced indexing's sort-based accumulate (~8 launches per epoch)."""
    if torch.is_tensor(idx) and idx.dim() == 1 and idx.dtype in (torch.int64, torch.int32):
        return out.index_select(0, idx.to(out.device))
    return out[idx]


def _train_step(model, optimizer, data):
    """mpgnn_train's body with the loss left on the device (no host sync)."""
    model.train()
    optimizer.zero_grad()
    out = model(data.x, data.edge_index, data.edge_type)
    weights = class_weight_balanced(data.train_y)
    loss = nll_loss_rows(out, data.train_idx, data.train_y)
    loss.backward()
    optimizer.step()
    return loss.detach(), weights


def mpgnn_train(model, optimizer, data):
    """main.py:1055-1082: full-batch forward, unweighted NLL on train_idx, backward, step.
    Returns (float loss, balanced class weights) like the reference (the weights are
    computed there but not applied, main.py:1065)."""
    loss, weights = _train_step(model, optimizer, data)
    return float(loss), weights


@torch.no_grad()
def _val_counts(model, data):
    """mpgnn_validation's work on the device: (val loss, [2, 3, C] train / val confusion counts)."""
    model.eval()
    pred = model(data.x, data.edge_index, data.edge_type)
    loss_val = nll_loss_rows(pred, data.val_idx, data.val_y)
    return loss_val, confusion_counts_rows(pred, [(data.train_idx, data.train_y), (data.val_idx, data.val_y)])


@torch.no_grad()
def mpgnn_validation(model, data, class_weight):
    """main.py:1084-1099 → (f1 train, f1 val, f1 val, val loss tensor); both val scores are
    the same macro F1, as in the reference."""
    model.eval()
    pred = model(data.x, data.edge_index, data.edge_type)
    loss_val = nll_loss_rows(pred, data.val_idx, data.val_y)
    f1_train, f1_val = f1_from_counts(confusion_counts_rows(pred, [(data.train_idx, data.train_y),
                                                                     (data.val_idx, data.val_y)]))
    return f1_train, f1_val, f1_val, loss_val


@torch.no_grad()
def mpgnn_test(model, data, class_weight):
    """main.py:1101-1115 → (test loss tensor, test macro F1)."""
    model.eval()
    pred = model(data.x, data.edge_index, data.edge_type)
    loss_test = nll_loss_rows(pred, data.test_idx, data.test_y)
    (f1_test,) = f1_from_counts(confusion_counts_rows(pred, [(data.test_idx, data.test_y)]))
    return loss_test, f1_test


def _fit(data_mpgnn, input_dim, hidden_dim, num_rel, output_dim, ll_output_dim, metapaths, epochs):
    model = MPNetm(input_dim, hidden_dim, num_rel, output_dim, ll_output_dim, len(metapaths), metapaths)
    model = model.to(data_mpgnn.x.device)
    optimizer = None if _graphs_enabled(data_mpgnn) else _adam(model)
    best_model = model  # the reference keeps a reference, not a copy (main.py:1125)
    use_graph = _graphs_enabled(data_mpgnn)
    if use_graph:
        optimizer = _adam_graphable(model)
    class_weight = class_weight_balanced(data_mpgnn.train_y)
    vcounts = None

    # every epoch trains and scores the validation split on the device; only the last epoch's
    # score is read by the host (its best-score test only re-assigns the same model object)
    def epoch():
        loss, _ = _train_step(model, optimizer, data_mpgnn)
        return (loss,) + _val_counts(model, data_mpgnn)

    for _epoch, (_loss, _loss_val, vcounts) in _epochs(epoch, epochs, use_graph):
        pass
    f1_valt_macro = f1_from_counts(vcounts)[1] if vcounts is not None else 0.
    return model, best_model, class_weight, f1_valt_macro


def mpgnn_parallel_multiple(data_mpgnn, input_dim, hidden_dim, num_rel, output_dim, ll_output_dim, metapaths,
                            epochs: int = EPOCHS):
    """main.py:1117-1136: train an MPNetm over ``metapaths`` for 999 epochs with Adam
    (lr 0.01, wd 5e-4); returns the last epoch's validation macro F1."""
    _, best_model, class_weight, f1_valt_macro = _fit(data_mpgnn, input_dim, hidden_dim, num_rel, output_dim,
                                                      ll_output_dim, metapaths, epochs)
    mpgnn_test(best_model, data_mpgnn, class_weight)
    return f1_valt_macro


def mpgnn_parallel_multiple_x(data_mpgnn, input_dim, hidden_dim, num_rel, output_dim, ll_output_dim, metapaths,
                              testing, epochs: int = EPOCHS):
    """main.py:1138-1160: as ``mpgnn_parallel_multiple`` (a single metapath may be given as a
    flat list); prints the test line; returns the test macro F1 when ``testing`` else the last
    validation macro F1."""
    if isinstance(metapaths[0], int):
        metapaths = [metapaths]
    _, best_model, class_weight, f1_valt_macro = _fit(data_mpgnn, input_dim, hidden_dim, num_rel, output_dim,
                                                      ll_output_dim, metapaths, epochs)
    test_loss, f1_macro_test = mpgnn_test(best_model, data_mpgnn, class_weight)
    print("test loss %0.3f" % test_loss, "test macro %0.3f" % f1_macro_test)
    if testing == False:  # noqa: E712  (reference: 0 and False both select validation)
        return f1_valt_macro
    return f1_macro_test
