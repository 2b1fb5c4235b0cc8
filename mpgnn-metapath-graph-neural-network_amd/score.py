"""The metapath score function on the GPU — drop-in for the reference's
``Score`` / ``InputLayer`` / ``OutputLayer`` (model.py:26-125) and the score-training helpers of
main.py (create_edge_dictionary :387-424, initialize_weights :479-497, train :641-673,
score_relation_parallel :727-760).

The reference represents the relation's edges as a Python dict {source: [destinations]} and its
forward (model.py:82-87) loops over the sources with a few tensor ops each — O(E_r) interpreter
work per epoch, 100 epochs per candidate relation: "where main.py actually spends its time".
Here the dictionary is built once as a CSR on the GPU (``EdgeDictionary``, a read-only Mapping
with the same keys / values / order as the reference dict), the forward is ONE kernel
(``mpgnn_score_argmax``: per-source first argmax of the destination weights, torch.argmax
semantics, bit-identical selection) and the backward ONE kernel (``mpgnn_score_argmax_bwd``:
per destination, the gradients of the sources that picked it, added in the order autograd
unwinds the reference's ``max_weights[source] = weights[max_node]`` chain). The per-epoch
``{source: max_node}`` results are returned as lazy Mappings (no host sync until read).

Scope: the non-bag branch (model.py:74-89) that ``score_relation_parallel`` trains. The bag
branch (model.py:45-72, score_relation_bags_*) is not on this path and raises.
"""
from __future__ import annotations

import os
import random
from collections.abc import Mapping

import numpy as np
import torch
import torch.nn as nn

from ._lib import check, lib

__all__ = ["EdgeDictionary", "DestinationDictionary", "ArgmaxDict", "build_edge_dictionary", "score_argmax",
           "InputLayer", "OutputLayer", "Score", "create_edge_dictionary", "initialize_weights", "get_model",
           "get_optimizer", "get_loss", "get_loss_per_node", "train", "score_relation_parallel", "EPOCHS",
           "FIRST_MASK_DATASETS"]

EPOCHS = 100  # main.py:755
FIRST_MASK_DATASETS = ("IMDB", "ACM", "DBLP", "fb15k-237")  # main.py:653: data.labels is per mask position
COMPLEX = "fb15k-237"  # main.py:1484 (stored by Score, unused by the non-bag forward)


def _stream(device) -> int:
    from .functional import _stream_of
    return _stream_of(torch.device(device))


def _ptr(t):
    return t.data_ptr() if t is not None and t.numel() else None


class EdgeDictionary(Mapping):
    """``{source: [destinations]}`` of one relation (create_edge_dictionary, main.py:387-406) as a
    device CSR. Keys are the sources of ``source_nodes_mask`` (first occurrence order) that have
    an edge of the relation; each value lists its destinations in edge-file order. Reads like the
    reference dict (host lists materialised on first access); ``copy()`` returns a plain dict."""

    def __init__(self, keys, key_ptr, dst, in_ptr, in_pos, in_key, num_nodes, mask_index, mask_list):
        self.keys_t, self.key_ptr_t, self.dst_t = keys, key_ptr, dst          # int32, device
        self.in_ptr_t, self.in_pos_t, self.in_key_t = in_ptr, in_pos, in_key  # int32, device
        self.num_nodes = int(num_nodes)
        self.mask_index = mask_index  # int64 [M] device: the mask as given (predictions[mask])
        self.mask_list = mask_list    # the list object it was built from (train() reuses mask_index)
        self._host = None
        self._pos = None

    @property
    def device(self):
        return self.keys_t.device

    def _load(self):
        if self._host is None:
            keys = self.keys_t.cpu().numpy().astype(np.int64)
            ptr = self.key_ptr_t.cpu().numpy().astype(np.int64)
            dst = self.dst_t.cpu().numpy().astype(np.int64)
            self._host = (keys, ptr, dst)
            self._pos = {int(k): i for i, k in enumerate(keys)}
        return self._host

    def __getitem__(self, source):
        keys, ptr, dst = self._load()
        i = self._pos[int(source)]
        return dst[ptr[i]:ptr[i + 1]].tolist()

    def __iter__(self):
        return iter(self._load()[0].tolist())

    def __len__(self):
        return int(self.keys_t.numel())

    def __contains__(self, source):
        self._load()
        try:
            return int(source) in self._pos
        except (TypeError, ValueError):
            return False

    def copy(self) -> dict:
        keys, ptr, dst = self._load()
        return {int(k): dst[ptr[i]:ptr[i + 1]].tolist() for i, k in enumerate(keys)}

    @property
    def num_entries(self) -> int:
        return int(self.dst_t.numel())


class DestinationDictionary(Mapping):
    """``{destination: [labels of its sources]}`` (main.py:412-423), keys in first-appearance
    order over the relation's edges (file order), values in edge order. Host numpy arrays;
    ``min_labels()`` gives initialize_weights its per-key minimum without building the lists."""

    def __init__(self, dst_edge_order: np.ndarray, labels_edge_order: np.ndarray, label_is_int: bool):
        self._d = dst_edge_order
        self._l = labels_edge_order
        self._int = label_is_int
        uniq, first = np.unique(self._d, return_index=True)
        order = np.argsort(first, kind="stable")
        self.keys_arr = uniq[order]
        srt = np.argsort(self._d, kind="stable")
        ds, ls = self._d[srt], self._l[srt]
        starts = np.flatnonzero(np.r_[True, ds[1:] != ds[:-1]]) if ds.size else np.zeros(0, dtype=np.int64)
        mins = np.minimum.reduceat(ls, starts) if ds.size else np.zeros(0)
        self._min = mins[order]
        self._runs = (srt, starts, order)
        self._pos = None

    def min_labels(self) -> np.ndarray:
        return self._min

    def _val(self, i):
        srt, starts, order = self._runs
        j = order[i]
        b = starts[j]
        e = starts[j + 1] if j + 1 < len(starts) else len(srt)
        v = self._l[srt[b:e]]
        return [int(a) for a in v] if self._int else v.tolist()

    def __getitem__(self, dst):
        if self._pos is None:
            self._pos = {int(k): i for i, k in enumerate(self.keys_arr)}
        return self._val(self._pos[int(dst)])

    def __iter__(self):
        return iter(self.keys_arr.tolist())

    def __len__(self):
        return int(self.keys_arr.size)


def build_edge_dictionary(edge_index, edge_type, relation, source_nodes_mask, labels=None, dataset="synthetic",
                          num_nodes=None, device=None):
    """create_edge_dictionary (main.py:387-424, non-bag) for one relation: (EdgeDictionary,
    DestinationDictionary or None when ``labels`` is None). Integer work only — bit-exact."""
    if device is None:
        device = edge_index.device if edge_index.is_cuda else torch.device("cuda", torch.cuda.current_device())
    device = torch.device(device)
    if device.type != "cuda":
        raise RuntimeError("mpgnn_amd: the score function runs only as HIP kernels on a ROCm GPU "
                           "(there is no CPU fallback)")
    n = int(num_nodes) if num_nodes is not None else (int(edge_index.max()) + 1 if edge_index.numel() else 0)
    ei = edge_index.to(device)
    et = edge_type.to(device)
    rel = int(relation)
    sel = et == rel
    src, dst = ei[0][sel], ei[1][sel]
    if src.numel() and (int(src.min()) < 0 or int(src.max()) >= n or int(dst.min()) < 0 or int(dst.max()) >= n):
        raise IndexError(f"index out of range: relation {rel} has a node outside [0, {n})")
    mask_list = source_nodes_mask
    mask = torch.as_tensor(list(source_nodes_mask), dtype=torch.int64)
    m0 = int(mask.numel())
    mask_d = mask.to(device)
    rank = torch.full((n,), m0, dtype=torch.int64, device=device)
    ok = (mask_d >= 0) & (mask_d < n)
    if m0:
        rank.scatter_reduce_(0, mask_d[ok], torch.arange(m0, device=device)[ok], reduce="amin")  # list.index
    r_src = rank[src] if src.numel() else src
    keep = r_src < m0
    src, dst, r_src = src[keep], dst[keep], r_src[keep]
    order = torch.argsort(r_src, stable=True)
    dst_s, r_s = dst[order], r_src[order]
    uniq, counts = torch.unique_consecutive(r_s, return_counts=True)
    K = int(uniq.numel())
    keys = mask_d[uniq]
    key_ptr = torch.zeros(K + 1, dtype=torch.int64, device=device)
    torch.cumsum(counts, 0, out=key_ptr[1:])
    k_of_p = torch.repeat_interleave(torch.arange(K, device=device), counts)
    # backward list: every (edge position, key) by destination, keys descending
    comp = dst_s * max(K, 1) + (K - 1 - k_of_p)
    order2 = torch.argsort(comp, stable=True)
    in_ptr = torch.zeros(n + 1, dtype=torch.int64, device=device)
    torch.cumsum(torch.bincount(dst_s, minlength=n), 0, out=in_ptr[1:])
    i32 = torch.int32
    ed = EdgeDictionary(keys.to(i32), key_ptr.to(i32), dst_s.to(i32), in_ptr.to(i32), order2.to(i32),
                        k_of_p[order2].to(i32), n, mask_d, mask_list)
    dd = None
    if labels is not None:
        lab = labels.reshape(-1) if torch.is_tensor(labels) else torch.as_tensor(labels).reshape(-1)
        lab_d = lab.to(device)
        per_edge = lab_d[src] if dataset == "synthetic" else lab_d[r_src]
        is_int = not torch.is_floating_point(lab)
        dd = DestinationDictionary(dst.cpu().numpy(), per_edge.cpu().numpy().astype(np.float64), is_int)
    return ed, dd


class ArgmaxDict(Mapping):
    """``{source: max_node}`` (model.py:86) of one forward, read lazily from the device."""

    def __init__(self, ed: EdgeDictionary, max_node: torch.Tensor):
        self._ed = ed
        self._mn = max_node
        self._host = None

    def _load(self):
        if self._host is None:
            keys = self._ed._load()[0]
            self._host = dict(zip(keys.tolist(), self._mn.cpu().numpy().astype(np.int64).tolist()))
        return self._host

    def __getitem__(self, k):
        return self._load()[k]

    def __iter__(self):
        return iter(self._load())

    def __len__(self):
        return len(self._ed)

    def values_tensor(self) -> torch.Tensor:
        """max_node of every key, in key order (int32, device) — no host copy."""
        return self._mn


class _ScoreArgmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, weights, ed: EdgeDictionary):
        n = ed.num_nodes
        w = weights.contiguous()
        dev = w.device
        K = len(ed)
        max_w = torch.empty(n, 1, dtype=torch.float32, device=dev)
        arg_pos = torch.empty(K, dtype=torch.int32, device=dev)
        max_node = torch.empty(K, dtype=torch.int32, device=dev)
        check(lib.mpgnn_score_argmax(w.data_ptr(), n, _ptr(ed.keys_t), _ptr(ed.key_ptr_t), _ptr(ed.dst_t), K,
                                     max_w.data_ptr(), _ptr(arg_pos), _ptr(max_node), _stream(dev)),
              "mpgnn_score_argmax")
        ctx.ed = ed
        ctx.save_for_backward(arg_pos)
        ctx.mark_non_differentiable(max_node)
        return max_w, max_node

    @staticmethod
    def backward(ctx, g_max, _g_node):
        (arg_pos,) = ctx.saved_tensors
        ed = ctx.ed
        g = g_max.contiguous().float()
        gw = torch.empty(ed.num_nodes, 1, dtype=torch.float32, device=g.device)
        check(lib.mpgnn_score_argmax_bwd(g.data_ptr(), ed.num_nodes, _ptr(ed.keys_t), _ptr(arg_pos), _ptr(ed.in_ptr_t),
                                         _ptr(ed.in_pos_t), _ptr(ed.in_key_t), gw.data_ptr(), _stream(g.device)),
              "mpgnn_score_argmax_bwd")
        return gw, None


def score_argmax(weights: torch.Tensor, ed: EdgeDictionary):
    """(max_weights [N, 1], max_node [K] int32): model.py:82-87 for every source at once,
    differentiable w.r.t. ``weights`` [N, 1] (float32, on the GPU)."""
    if not weights.is_cuda:
        raise RuntimeError("mpgnn_amd: the score function runs only as HIP kernels on a ROCm GPU "
                           "(there is no CPU fallback); move the weights to 'cuda'")
    if weights.dtype != torch.float32 or weights.numel() != ed.num_nodes:
        raise ValueError(f"weights must be float32 with {ed.num_nodes} entries, got {weights.dtype} {tuple(weights.shape)}")
    return _ScoreArgmaxFn.apply(weights, ed)


# ---------------------------------------------------------------------------------------------
# model.py:26-125
# ---------------------------------------------------------------------------------------------
class InputLayer(nn.Module):
    """model.py:26-34: the trainable destination weights [N, 1]."""

    def __init__(self, weights):
        super().__init__()
        self.weights = nn.Parameter(weights.unsqueeze(-1))

    def forward(self):
        return self.weights


def _edge_dictionary_of(node_dict, num_nodes, device):
    if isinstance(node_dict, EdgeDictionary):
        return node_dict
    # a plain {source: [destinations]} dict (the reference's own): converted per call
    keys = list(node_dict.keys())
    lens = [len(node_dict[k]) for k in keys]
    dst = [d for k in keys for d in node_dict[k]]
    ei = torch.tensor([[k for k, c in zip(keys, lens) for _ in range(c)], dst], dtype=torch.int64).reshape(2, -1)
    et = torch.zeros(ei.size(1), dtype=torch.int64)
    ed, _ = build_edge_dictionary(ei, et, 0, keys, None, num_nodes=num_nodes, device=device)
    return ed


class OutputLayer(nn.Module):
    """model.py:36-89: ``LinearLayerAttri`` (used by the bag branch and clean_dictionaries,
    main.py:460) and the forward: per source the argmax destination (non-bag branch, :74-89)."""

    def __init__(self, features_dim):
        super().__init__()
        self.LinearLayerAttri = nn.Linear(features_dim, 1, bias=False)

    def forward(self, weights, data, node_dict, BAGS, COMPLEX, feat):
        if BAGS:
            raise NotImplementedError("the bag branch of OutputLayer.forward (model.py:45-72) is not on the "
                                      "GPU score path; score_relation_parallel uses the non-bag branch")
        num_nodes = int(data.num_nodes)
        ed = _edge_dictionary_of(node_dict, num_nodes, weights.device)
        max_weights, max_node = score_argmax(weights, ed)
        best = ArgmaxDict(ed, max_node)
        return max_weights, best, best


class Score(nn.Module):
    """model.py:91-125: ``input`` (InputLayer) and ``output`` (OutputLayer) in the reference's
    order, so parameters, state_dict keys and the seeded Linear init are the same."""

    def __init__(self, weights, COMPLEX, features_dim):
        super().__init__()
        self.COMPLEX = COMPLEX
        self.features_dim = features_dim
        self.input = InputLayer(weights)
        self.output = OutputLayer(self.features_dim)

    def frz_weights(self, indices):
        """model.py:104-111 (as written there: flags on a view, no effect on training)."""
        for i in indices:
            self.input.weights[i].requires_grad = False

    def forward(self, data, node_dict, BAGS):
        x = self.input()
        # the reference converts data.x to a CPU FloatTensor (model.py:116) for the bag branch only
        return self.output(x, data, node_dict, BAGS, self.COMPLEX, None)


# ---------------------------------------------------------------------------------------------
# main.py helpers
# ---------------------------------------------------------------------------------------------
def create_edge_dictionary(data, relation, source_nodes_mask, BAGS, dataset="synthetic"):
    """main.py:387-424 (BAGS=False): (EdgeDictionary, DestinationDictionary) built on the GPU."""
    if BAGS:
        raise NotImplementedError("create_edge_dictionary(BAGS=True) (main.py:426-438) is not on the GPU score path")
    return build_edge_dictionary(data.edge_index, data.edge_type, relation, source_nodes_mask, data.labels, dataset,
                                 num_nodes=int(data.num_nodes))


def initialize_weights(data, destination_dictionary, BAGS, rng=None):
    """main.py:479-497: weight[dst] = |min(labels of its sources) + random.uniform(-0.2, 0.2)|,
    drawn from Python's ``random`` (or ``rng``) in destination-dictionary order — the same
    stream as the reference. Entries of nodes that are no destination are 0 (the reference
    leaves them uninitialised; the argmax never reads them)."""
    rng = rng or random
    weights = torch.zeros(int(data.num_nodes))
    if isinstance(destination_dictionary, DestinationDictionary):
        keys, mins = destination_dictionary.keys_arr, destination_dictionary.min_labels()
    else:
        keys = np.array(list(destination_dictionary.keys()), dtype=np.int64)
        mins = [min(v) for v in destination_dictionary.values()]
    vals = [abs(float(m) + rng.uniform(-0.2, 0.2)) for m in mins]
    if len(vals):
        weights[torch.from_numpy(np.asarray(keys, dtype=np.int64))] = torch.tensor(vals, dtype=torch.float64).float()
    return weights


def get_model(weights, features_dim):
    """main.py:518-519."""
    return Score(weights, COMPLEX, features_dim)


def get_optimizer(model):
    """main.py:521-522: Adam(lr 0.1); on the GPU the fused single-kernel implementation."""
    params = list(model.parameters())
    fused = bool(params) and all(p.is_cuda for p in params)
    return torch.optim.Adam(params, lr=0.1, fused=fused)


def get_loss():
    return nn.MSELoss(reduction="mean")       # main.py:524-525


def get_loss_per_node():
    return nn.MSELoss(reduction="none")       # main.py:527-528


def _mask_index(edge_dictionary, source_nodes_mask, device):
    if isinstance(edge_dictionary, EdgeDictionary) and edge_dictionary.mask_list is source_nodes_mask:
        return edge_dictionary.mask_index
    return torch.as_tensor(list(source_nodes_mask), dtype=torch.int64).to(device)


def train(data, edge_dictionary, model, optimizer, criterion, source_nodes_mask, criterion_per_node,
          destination_nodes_with_freezed_weights, previous_weights, grad_mask, BAGS, bags_to_predict=None,
          bags_to_predict_labels=None, dataset="synthetic"):
    """main.py:641-673, non-bag: one epoch → (loss, {source: max_node}, loss_per_node,
    {source: max_node}, predictions). No host sync (the dicts are lazy, the loss a device
    tensor). ``data.labels`` may live on the CPU: it is moved once and cached on ``data``."""
    if BAGS:
        raise NotImplementedError("train(BAGS=True) (main.py:644-649) is not on the GPU score path")
    model.train()
    optimizer.zero_grad()
    predictions, max_destination_node_for_bag, max_destination_node_for_source = model(data, edge_dictionary, BAGS)
    dev = predictions.device
    labels = getattr(data, "_labels_dev", None)
    if labels is None or labels[0] is not data.labels:
        labels = (data.labels, data.labels.to(dev))
        try:
            data._labels_dev = labels
        except AttributeError:
            pass
    labels = labels[1]
    if dataset in FIRST_MASK_DATASETS:
        idx = _mask_index(edge_dictionary, source_nodes_mask, dev)
        predictions, labels = predictions.index_select(0, idx).to(torch.float32), labels.to(torch.float32)
    elif dataset == "synthetic":
        idx = _mask_index(edge_dictionary, source_nodes_mask, dev)
        predictions, labels = predictions.index_select(0, idx).to(torch.float32), \
            labels.index_select(0, idx).to(torch.float32)
    loss = criterion(predictions, labels)
    loss_per_node = criterion_per_node(predictions.detach(), labels)
    loss.backward()
    if destination_nodes_with_freezed_weights:  # main.py:663-664
        model.input.weights.grad = model.input.weights.grad * grad_mask.to(dev)
    optimizer.step()
    with torch.no_grad():  # main.py:667-672
        model.input.weights.clamp_(min=0.0, max=1.0)
        model.output.LinearLayerAttri.weight.clamp_(min=0.0, max=1.0)
        if destination_nodes_with_freezed_weights:
            idx = torch.as_tensor(list(destination_nodes_with_freezed_weights), dtype=torch.int64, device=dev)
            model.input.weights[idx] = previous_weights.reshape(-1, 1).to(dev)[idx].to(torch.float32)
    return loss, max_destination_node_for_source, loss_per_node, max_destination_node_for_bag, predictions


def score_relation_parallel(data, relation, source_nodes, features_dim, dataset, epochs: int = EPOCHS):
    """main.py:727-760: score one candidate relation — edge dictionary, weights, 100 epochs of
    ``train`` — on the GPU. Returns (relation, final loss, edge_dictionary,
    destination_dictionary) like the reference (one host sync: the final loss)."""
    if not source_nodes:
        et = data.edge_type
        src = data.edge_index[0][et == relation]
        source_nodes = torch.unique(src).tolist()
    edge_dictionary, destination_dictionary = create_edge_dictionary(data, relation, source_nodes, BAGS=False,
                                                                     dataset=dataset)
    weights = initialize_weights(data, destination_dictionary, BAGS=False)
    model = get_model(weights, features_dim).to(edge_dictionary.device)
    criterion, criterion_per_node = get_loss(), get_loss_per_node()
    # the 100 epochs replay one captured HIP graph after three eager ones (main._epochs: every
    # kernel of every epoch still runs; the host issues one launch per epoch instead of ~25)
    from .main import _epochs
    use_graph = os.environ.get("MPGNN_LOOP_GRAPH", "1") != "0" and edge_dictionary.device.type == "cuda"
    if use_graph:  # Adam(lr 0.1) of main.py:521-522, fused and capturable: the same update
        optimizer = torch.optim.Adam(list(model.parameters()), lr=0.1, fused=True, capturable=True)
    else:
        optimizer = get_optimizer(model)
    grad_mask = torch.tensor(0)

    def epoch():
        return train(data, edge_dictionary, model, optimizer, criterion, source_nodes, criterion_per_node,
                     [], weights, grad_mask, BAGS=False, dataset=dataset)[0]

    loss = None
    for _, loss in _epochs(epoch, epochs, use_graph):
        pass
    return relation, loss.item(), edge_dictionary, destination_dictionary
