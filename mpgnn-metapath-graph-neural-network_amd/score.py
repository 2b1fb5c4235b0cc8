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

The bag branch (model.py:45-72) that ``score_relation_bags_parallel`` (main.py:853-917) trains
in the metapath-extension rounds is the same on the GPU: the bags (lists of source nodes) are a
device CSR (``BagSet``), the forward ONE kernel (``mpgnn_score_bag_argmax``: one wave per bag
walks its members in bag order, each member's first argmax of ``weights[dst] · lin(feat[src])``
wave-parallel, the strict ``>`` pick of the reference), the backward ONE pair of kernels
(``mpgnn_score_bag_argmax_bwd``: d weights per destination and d LinearLayerAttri per feature,
added in the order autograd unwinds the reference's chain — bags descending).
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
           "FIRST_MASK_DATASETS", "BagSet", "BagDestinationDictionary", "score_bag_argmax", "create_bags",
           "clean_bags_for_relation_type", "reinitialize_weights", "retrieve_destinations_low_loss",
           "score_relation_bags_parallel", "BAG_EPOCHS", "RelationDictionaries", "score_relations_batched"]

EPOCHS = 100  # main.py:755
BAG_EPOCHS = 50  # main.py:888
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
        if BAGS:  # model.py:45-72: per bag the best member pick (HIP kernels, see score_bag_argmax)
            num_nodes = int(data.num_nodes)
            ed = _edge_dictionary_of(node_dict, num_nodes, weights.device)
            bs = _bag_set_of(data.bags, ed)
            if feat is None:
                feat = _features_of(data, weights.device)
            max_weights, bag_mem, mem_v, mem_max = score_bag_argmax(weights, self.LinearLayerAttri.weight, feat, bs)
            return max_weights, BagPickDict(bs, bag_mem, mem_max), SourceValueDict(bs, mem_v)
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
        # data.x as float32 (model.py:116), read by the bag branch only: kept on the GPU
        feat = _features_of(data, x.device) if BAGS else None
        return self.output(x, data, node_dict, BAGS, self.COMPLEX, feat)


# ---------------------------------------------------------------------------------------------
# main.py helpers
# ---------------------------------------------------------------------------------------------
def create_edge_dictionary(data, relation, source_nodes_mask, BAGS, dataset="synthetic"):
    """main.py:387-438: (EdgeDictionary, DestinationDictionary) built on the GPU; with BAGS the
    second dictionary is {destination: [labels of the bags of its sources]} (:426-438)."""
    if BAGS:
        ed, _ = build_edge_dictionary(data.edge_index, data.edge_type, relation, source_nodes_mask, None, dataset,
                                      num_nodes=int(data.num_nodes))
        return ed, BagDestinationDictionary(data, relation)
    return build_edge_dictionary(data.edge_index, data.edge_type, relation, source_nodes_mask, data.labels, dataset,
                                 num_nodes=int(data.num_nodes))


def initialize_weights(data, destination_dictionary, BAGS, rng=None):
    """main.py:479-497: weight[dst] = |min(labels of its sources) + random.uniform(-0.2, 0.2)|,
    drawn from Python's ``random`` (or ``rng``) in destination-dictionary order — the same
    stream as the reference. Entries of nodes that are no destination are 0 (the reference
    leaves them uninitialised; the argmax never reads them)."""
    rng = rng or random
    weights = torch.zeros(int(data.num_nodes))
    if isinstance(destination_dictionary, (DestinationDictionary, BagDestinationDictionary)):
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
        return _train_bags(data, edge_dictionary, model, optimizer, criterion, criterion_per_node,
                           destination_nodes_with_freezed_weights, previous_weights, grad_mask, bags_to_predict,
                           bags_to_predict_labels)
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
    _clamp_and_restore(model, destination_nodes_with_freezed_weights, previous_weights)
    return loss, max_destination_node_for_source, loss_per_node, max_destination_node_for_bag, predictions


def _clamp_and_restore(model, frozen, previous_weights):
    """main.py:667-672: both parameters clamped to [0, 1], frozen destinations reset to
    ``previous_weights`` (a no-op when previous_weights IS the parameter's storage, as in
    score_relation_bags_parallel: InputLayer wraps the weights tensor it is given)."""
    with torch.no_grad():
        model.input.weights.clamp_(min=0.0, max=1.0)
        model.output.LinearLayerAttri.weight.clamp_(min=0.0, max=1.0)
        if frozen:
            dev = model.input.weights.device
            idx = _device_cached(("frozen_idx", tuple(int(v) for v in frozen)), dev,
                                 lambda: torch.as_tensor([int(v) for v in frozen], dtype=torch.int64))
            prev = previous_weights.reshape(-1, 1)
            if prev.device != dev:
                prev = _device_cached(("prev", id(previous_weights), previous_weights._version), dev,
                                      lambda: previous_weights.reshape(-1, 1).to(torch.float32), keep=previous_weights)
            model.input.weights[idx] = prev[idx].to(torch.float32)


_DEV_CACHE: dict = {}


def _device_cached(key, dev, make, keep=None):
    """A host-built tensor copied to ``dev`` once per key (the loops call train() under HIP-graph
    capture, where a fresh host-to-device copy must not be recorded); ``keep`` pins the object
    whose id is part of the key."""
    k = (key, str(dev))
    hit = _DEV_CACHE.get(k)
    if hit is None:
        if len(_DEV_CACHE) > 256:
            _DEV_CACHE.clear()
        hit = _DEV_CACHE[k] = (make().to(dev), keep)
    return hit[0]


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


# ---------------------------------------------------------------------------------------------
# bag branch: model.py:45-72; main.py:426-438, 498-512, 530-592, 641-673, 853-917
# ---------------------------------------------------------------------------------------------
class BagDestinationDictionary(Mapping):
    """``{destination: [labels of the bags holding one of its sources]}`` (main.py:426-438):
    over the relation's edges in file order whose source lies in some bag of ``data.bags``, the
    labels of that source's bags (bag order) are appended to the destination's list; keys in
    first-appearance order. Built with numpy; ``min_labels()`` feeds initialize_weights."""

    def __init__(self, data, relation):
        ei = data.edge_index.cpu().numpy() if torch.is_tensor(data.edge_index) else np.asarray(data.edge_index)
        et = data.edge_type.cpu().numpy() if torch.is_tensor(data.edge_type) else np.asarray(data.edge_type)
        sel = et == int(relation)
        src, dst = ei[0][sel].astype(np.int64), ei[1][sel].astype(np.int64)
        labels = data.bag_labels.reshape(-1).cpu().numpy().astype(np.float64) if len(data.bags) else np.zeros(0)
        per_node = {}  # node -> labels of its bags, bag order (main.py:428-432)
        for i, bag in enumerate(data.bags):
            for node in bag:
                per_node.setdefault(int(node), []).append(float(labels[i]))
        keep = np.fromiter((int(v) in per_node for v in src), dtype=bool, count=src.size)
        self._src, self._dst = src[keep], dst[keep]
        self._per_node = per_node
        uniq, first = np.unique(self._dst, return_index=True)
        order = np.argsort(first, kind="stable")
        self.keys_arr = uniq[order]
        node_min = {n: min(v) for n, v in per_node.items()}
        mins = {}
        for s_, d_ in zip(self._src.tolist(), self._dst.tolist()):
            m = node_min[s_]
            if d_ not in mins or m < mins[d_]:
                mins[d_] = m
        self._min = np.array([mins[int(k)] for k in self.keys_arr], dtype=np.float64)
        self._pos = None

    def min_labels(self) -> np.ndarray:
        return self._min

    def __getitem__(self, dst):
        d = int(dst)
        if d not in self:
            raise KeyError(dst)
        out = []
        for s_ in self._src[self._dst == d].tolist():
            out.extend(self._per_node[s_])
        return out

    def __contains__(self, dst):
        if self._pos is None:
            self._pos = {int(k): i for i, k in enumerate(self.keys_arr)}
        try:
            return int(dst) in self._pos
        except (TypeError, ValueError):
            return False

    def __iter__(self):
        return iter(self.keys_arr.tolist())

    def __len__(self):
        return int(self.keys_arr.size)


class BagSet:
    """Bags (lists of source nodes, data.bags) against one EdgeDictionary, on the device:
    ``bag_ptr`` [B+1] / ``mem_node`` [M] the CSR of members in bag order, ``mem_key`` [M] each
    member's dictionary key index (-1: not a key, skipped as model.py:59 does), and the backward's
    candidate lists — per destination node n every (bag, member, edge position) that can pick n,
    bags descending (``in_ptr`` [N+1], ``in_bag``, ``in_mem``, ``in_pos``). Integer work, once per
    (bags, dictionary)."""

    def __init__(self, bags, ed: EdgeDictionary):
        self.bags = bags
        self.ed = ed
        dev = ed.device
        N = ed.num_nodes
        lens = np.fromiter((len(b) for b in bags), dtype=np.int64, count=len(bags))
        B = int(lens.size)
        self.num_bags = B
        nodes = np.fromiter((int(n) for b in bags for n in b), dtype=np.int64, count=int(lens.sum()))
        ptr = np.zeros(B + 1, dtype=np.int64)
        np.cumsum(lens, out=ptr[1:])
        i32 = torch.int32
        self.bag_ptr = torch.from_numpy(ptr).to(dev, i32)
        nodes_d = torch.from_numpy(nodes).to(dev)
        self.mem_node = nodes_d.clamp(0, max(N - 1, 0)).to(i32)
        K = len(ed)
        key_of = torch.full((max(N, 1),), -1, dtype=torch.int64, device=dev)
        if K:
            key_of[ed.keys_t.long()] = torch.arange(K, device=dev)
        valid = (nodes_d >= 0) & (nodes_d < N)
        mk = torch.where(valid, key_of[nodes_d.clamp(0, max(N - 1, 0))], torch.full_like(nodes_d, -1))
        self.mem_key = mk.to(i32)
        m_idx = torch.nonzero(mk >= 0).reshape(-1)
        k = mk[m_idx]
        kp = ed.key_ptr_t.long()
        deg = (kp[k + 1] - kp[k]) if k.numel() else k
        total = int(deg.sum()) if k.numel() else 0
        if total:
            m_rep = torch.repeat_interleave(m_idx, deg)
            starts = torch.repeat_interleave(kp[k], deg)
            offs = torch.arange(total, device=dev) - torch.repeat_interleave(torch.cumsum(deg, 0) - deg, deg)
            pos = starts + offs
            node = ed.dst_t.long()[pos]
            bag_of_mem = torch.repeat_interleave(torch.arange(B, device=dev), torch.from_numpy(lens).to(dev))
            bag = bag_of_mem[m_rep]
            order = torch.argsort(node * max(B, 1) + (B - 1 - bag), stable=True)
            in_ptr = torch.zeros(N + 1, dtype=torch.int64, device=dev)
            torch.cumsum(torch.bincount(node, minlength=N), 0, out=in_ptr[1:])
            self.in_ptr, self.in_bag = in_ptr.to(i32), bag[order].to(i32)
            self.in_mem, self.in_pos = m_rep[order].to(i32), pos[order].to(i32)
        else:
            self.in_ptr = torch.zeros(N + 1, dtype=i32, device=dev)
            self.in_bag = self.in_mem = self.in_pos = torch.zeros(0, dtype=i32, device=dev)
        self._strs = None

    @property
    def num_members(self) -> int:
        return int(self.mem_node.numel())

    def bag_strs(self):
        """str(bag) of every bag, the reference's dictionary keys (model.py:69)."""
        if self._strs is None:
            self._strs = [str(b) for b in self.bags]
        return self._strs


def _bag_set_of(bags, ed: EdgeDictionary) -> BagSet:
    cache = ed.__dict__.setdefault("_bag_sets", {})
    hit = cache.get(id(bags))
    if hit is None or hit.bags is not bags or hit.num_bags != len(bags):
        if len(cache) > 8:
            cache.clear()
        hit = cache[id(bags)] = BagSet(bags, ed)
    return hit


def _features_of(data, dev):
    """data.x as float32 on ``dev`` (model.py:116 ``data.x.type(torch.FloatTensor)``), cached
    on ``data`` per source tensor."""
    owner = data.__dict__.get("_data", data)  # a _BagsView caches on the data it wraps
    x = owner.x
    hit = getattr(owner, "_x_f32_dev", None)
    if hit is None or hit[0] is not x or hit[1].device != torch.device(dev):
        hit = (x, x.to(dev, torch.float32).contiguous())
        try:
            owner._x_f32_dev = hit
        except AttributeError:
            pass
    return hit[1]


class _ScoreBagArgmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, weights, lin_weight, feat, bs: BagSet):
        dev = weights.device
        B, M = bs.num_bags, bs.num_members
        w = weights.contiguous()
        lw = lin_weight.detach().reshape(-1).contiguous()
        f = feat.contiguous()
        F = int(f.shape[1]) if f.dim() == 2 else 0
        max_w = torch.zeros(B, 1, dtype=torch.float32, device=dev)
        bag_mem = torch.empty(B, dtype=torch.int32, device=dev)
        bag_w = torch.empty(B, dtype=torch.float32, device=dev)
        mem_s = torch.empty(M, dtype=torch.float32, device=dev)
        mem_v = torch.empty(M, dtype=torch.float32, device=dev)
        mem_pos = torch.empty(M, dtype=torch.int32, device=dev)
        mem_max = torch.empty(M, dtype=torch.int32, device=dev)
        ed = bs.ed
        check(lib.mpgnn_score_bag_argmax(w.data_ptr(), _ptr(f), F, _ptr(lw), bs.bag_ptr.data_ptr(), _ptr(bs.mem_node),
                                         _ptr(bs.mem_key), B, _ptr(ed.key_ptr_t), _ptr(ed.dst_t), _ptr(max_w),
                                         _ptr(bag_mem), _ptr(bag_w), _ptr(mem_s), _ptr(mem_v), _ptr(mem_pos),
                                         _ptr(mem_max), _stream(dev)), "mpgnn_score_bag_argmax")
        ctx.bs, ctx.F, ctx.lin_shape = bs, F, lin_weight.shape
        ctx.save_for_backward(bag_mem, bag_w, mem_s, mem_pos, f)
        ctx.mark_non_differentiable(bag_mem, mem_v, mem_max)
        return max_w, bag_mem, mem_v, mem_max

    @staticmethod
    def backward(ctx, g_max, _g1, _g2, _g3):
        bag_mem, bag_w, mem_s, mem_pos, f = ctx.saved_tensors
        bs = ctx.bs
        g = g_max.contiguous().float().reshape(-1)
        dev = g.device
        want_w, want_l = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        gw = torch.empty(bs.ed.num_nodes, 1, dtype=torch.float32, device=dev) if want_w else None
        gl = torch.empty(ctx.lin_shape, dtype=torch.float32, device=dev) if want_l else None
        check(lib.mpgnn_score_bag_argmax_bwd(_ptr(g), bs.num_bags, _ptr(bag_mem), _ptr(bag_w), _ptr(bs.mem_node),
                                             _ptr(mem_s), _ptr(mem_pos), _ptr(f), ctx.F if want_l else 0,
                                             bs.ed.num_nodes if want_w else 0, _ptr(bs.in_ptr), _ptr(bs.in_bag),
                                             _ptr(bs.in_mem), _ptr(bs.in_pos), _ptr(gw), _ptr(gl), _stream(dev)),
              "mpgnn_score_bag_argmax_bwd")
        return gw, gl, None, None


def score_bag_argmax(weights: torch.Tensor, lin_weight: torch.Tensor, feat: torch.Tensor, bs: BagSet):
    """model.py:45-72 for every bag at once: (max_weights [B, 1], bag_mem [B] (the picked member,
    -1: none), mem_v [M] (weights[max] · lin(feat[source]) per member), mem_max [M] (its argmax
    destination)); differentiable w.r.t. ``weights`` [N, 1] and ``lin_weight`` [1, F]."""
    if not weights.is_cuda:
        raise RuntimeError("mpgnn_amd: the score function runs only as HIP kernels on a ROCm GPU "
                           "(there is no CPU fallback); move the weights to 'cuda'")
    if weights.dtype != torch.float32 or weights.numel() != bs.ed.num_nodes:
        raise ValueError(f"weights must be float32 with {bs.ed.num_nodes} entries, got {weights.dtype} "
                         f"{tuple(weights.shape)}")
    if feat.dim() != 2 or feat.shape[0] != bs.ed.num_nodes or lin_weight.numel() != feat.shape[1]:
        raise RuntimeError(f"mat1 and mat2 shapes cannot be multiplied (features {tuple(feat.shape)}, "
                           f"LinearLayerAttri {tuple(lin_weight.shape)})")
    return _ScoreBagArgmaxFn.apply(weights, lin_weight, feat.to(torch.float32), bs)


class BagPickDict(Mapping):
    """``{str(bag): max_node}`` of one forward (model.py:69), read lazily from the device: bags in
    order, a bag without a pick has no entry, a bag whose string repeats an earlier one
    overwrites its value in place — the reference dict's contents and order."""

    def __init__(self, bs: BagSet, bag_mem: torch.Tensor, mem_max: torch.Tensor):
        self._bs, self._bm, self._mm = bs, bag_mem, mem_max
        self._host = None

    def _load(self):
        if self._host is None:
            bm = self._bm.cpu().numpy()
            mm = self._mm.cpu().numpy()
            d = {}
            for s_, m in zip(self._bs.bag_strs(), bm.tolist()):
                if m >= 0:
                    d[s_] = int(mm[m])
            self._host = d
        return self._host

    def __getitem__(self, k):
        return self._load()[k]

    def __iter__(self):
        return iter(self._load())

    def __len__(self):
        return len(self._load())


class SourceValueDict(Mapping):
    """``{source: weights[max_node] · lin(feat[source])}`` (model.py:64) of one forward: keys in
    first-visit order over the bags' members that are dictionary keys, values 1-element tensors
    like the reference's (``.item()`` reads them)."""

    def __init__(self, bs: BagSet, mem_v: torch.Tensor):
        self._bs, self._v = bs, mem_v
        self._host = None

    def _load(self):
        if self._host is None:
            v = self._v.cpu().numpy()
            keys = self._bs.mem_key.cpu().numpy()
            nodes = [int(n) for b in self._bs.bags for n in b]
            d = {}
            for m, (n, k) in enumerate(zip(nodes, keys.tolist())):
                if k >= 0:
                    d[n] = float(v[m])
            self._host = d
        return self._host

    def __getitem__(self, k):
        return torch.tensor([self._load()[k]], dtype=torch.float32)

    def __iter__(self):
        return iter(self._load())

    def __len__(self):
        return len(self._load())

    def floats(self) -> dict:
        """The values as Python floats (no tensor per entry)."""
        return dict(self._load())


class _BagsView:
    """``data.clone()`` with ``bags`` replaced (main.py:645-646) without copying the graph."""

    def __init__(self, data, bags):
        self.__dict__["_data"] = data
        self.__dict__["bags"] = bags

    def __getattr__(self, name):
        return getattr(self.__dict__["_data"], name)


def _train_bags(data, edge_dictionary, model, optimizer, criterion, criterion_per_node, frozen, previous_weights,
                grad_mask, bags, bag_labels):
    """main.py:641-673 with BAGS=True: MSE of the bag picks against the bag labels, backward,
    gradient mask when destinations are frozen, Adam step, clamps, frozen restore."""
    model.train()
    optimizer.zero_grad()
    predictions, by_bag, by_source = model(_BagsView(data, bags), edge_dictionary, True)
    dev = predictions.device
    labels = _device_cached(("bag_labels", id(bag_labels), bag_labels._version), dev,
                            lambda: bag_labels.to(torch.float32), keep=bag_labels)
    loss = criterion(predictions, labels)
    loss_per_node = criterion_per_node(predictions.detach(), labels)
    loss.backward()
    if frozen:  # main.py:663-664
        gm = _device_cached(("grad_mask", id(grad_mask), grad_mask._version), dev,
                            lambda: grad_mask.to(torch.float32), keep=grad_mask)
        model.input.weights.grad = model.input.weights.grad * gm
    optimizer.step()
    _clamp_and_restore(model, frozen, previous_weights)
    return loss, by_source, loss_per_node, by_bag, predictions


def create_bags(edg_dictionary, dest_dictionary, data):
    """main.py:545-575: for every source, its destinations whose labels are all > 0.9 make one
    bag (label 1); every other destination is a singleton bag (label 0, once); repeated bags
    dropped (first kept). Sets ``data.bags`` / ``data.bag_labels`` [B, 1]."""
    bag, labels = [], []
    singles = set()
    for key in edg_dictionary.keys():
        group = []
        for value in edg_dictionary[key]:
            if min(dest_dictionary[value]) > 0.9:
                group.append(value)
            elif value not in singles:
                singles.add(value)
                bag.append([value])
                labels.append(0)
        if group:
            bag.append(group)
            labels.append(1)
    seen = set()
    new_bag, new_labels = [], []
    for b, lab in zip(bag, labels):
        t = tuple(b)
        if t not in seen:
            seen.add(t)
            new_bag.append(b)
            new_labels.append(lab)
    data.bags = list(new_bag)
    data.bag_labels = torch.Tensor(new_labels).unsqueeze(-1)


def clean_bags_for_relation_type(data, edge_dictionary):
    """main.py:577-592: every bag reduced to its members that are dictionary keys; emptied bags
    dropped with their labels. Returns (bags, labels [B, 1])."""
    keys = set(edge_dictionary.keys())
    keep, keep_labels = [], []
    for c, b in enumerate(data.bags):
        tmp = [node for node in b if node in keys]
        if tmp:
            keep.append(tmp)
            keep_labels.append(data.bag_labels[c])
    return keep, torch.Tensor(keep_labels).unsqueeze(-1)


def reinitialize_weights(data, destination_dictionary, previous_weights, destination_nodes_with_freezed_weights,
                         BAGS, rng=None):
    """main.py:498-512: frozen destinations keep ``previous_weights``, every other destination key
    gets U(0, 1) from Python's ``random`` (dictionary order); other entries 0 (uninitialised in
    the reference, never read)."""
    rng = rng or random
    weights = torch.zeros(int(data.num_nodes))
    keys = (destination_dictionary.keys_arr.tolist() if isinstance(destination_dictionary, BagDestinationDictionary)
            else list(destination_dictionary.keys()))
    frozen = set(int(v) for v in destination_nodes_with_freezed_weights)
    prev = previous_weights.detach().reshape(-1).cpu() if frozen else None
    for key in keys:
        weights[key] = prev[key] if key in frozen else rng.uniform(0., 1.)
    return weights


def retrieve_destinations_low_loss(max_destination_node_dict, loss_per_node, source_nodes_mask=None):
    """main.py:530-543: the destinations of the dictionary entries (i-th entry ↔ loss_per_node[i])
    with loss < 1e-4, first occurrence order."""
    losses = loss_per_node.detach().reshape(-1).cpu().tolist() if torch.is_tensor(loss_per_node) else \
        list(loss_per_node)
    out = []
    for index, value in enumerate(max_destination_node_dict.values()):
        if losses[index] < 0.0001 and value not in out:
            out.append(value)
    return out


def score_relation_bags_parallel(data_object, relation, features_dim, dataset, epochs: int = BAG_EPOCHS,
                                 trace=None):
    """main.py:853-917: score one candidate relation against the bags of ``data_object`` —
    restarts of 50 epochs of train(BAGS=True) until two restarts in a row fail to lower the
    loss; after an improving restart the destinations of the bags with loss < 1e-4 are frozen
    (gradient mask 0) for the later restarts, whose weights are re-drawn. Returns (relation,
    current_loss, model, predictions_for_each_restart, v) like the reference. Each restart's
    epochs replay one captured HIP graph after three eager ones (main._epochs).
    ``trace`` (a list) receives (loss, [pick per bag]) of every epoch (one host sync each)."""
    mask, seen = [], set()
    for bag in data_object.bags:
        for elm in bag:
            if elm not in seen:
                seen.add(elm)
                mask.append(elm)
    edge_dictionary, destination_dictionary = create_edge_dictionary(data_object, relation, mask, BAGS=True,
                                                                     dataset=dataset)
    bags, bag_labels = clean_bags_for_relation_type(data_object, edge_dictionary)
    weights = initialize_weights(data_object, destination_dictionary, BAGS=True)
    N = int(data_object.num_nodes)
    grad_mask = torch.ones(len(weights), 1)
    criterion, criterion_per_node = get_loss(), get_loss_per_node()
    preds = {}
    frozen = []
    v = len(bags) == 1 or (len(bags) > 1 and bag_labels.squeeze().tolist().count(1) == 0)
    dev = edge_dictionary.device
    from .main import _epochs
    use_graph = os.environ.get("MPGNN_LOOP_GRAPH", "1") != "0" and trace is None
    rest, current_loss, model = 0, 100, None
    while rest < 2:
        w_dev = weights.to(dev)
        model = get_model(w_dev, features_dim).to(dev)  # InputLayer wraps w_dev: the restore reads the live weights
        optimizer = torch.optim.Adam(list(model.parameters()), lr=0.1, fused=True, capturable=use_graph)
        frozen_now = list(frozen)

        def epoch():
            return train(data_object, edge_dictionary, model, optimizer, criterion, mask, criterion_per_node,
                         frozen_now, w_dev, grad_mask, True, bags_to_predict=bags, bags_to_predict_labels=bag_labels,
                         dataset=dataset)

        out = None
        for _, out in _epochs(epoch, epochs, use_graph):
            if trace is not None:
                picks = out[3]
                trace.append((float(out[0].item()), [picks.get(s_, -1) for s_ in [str(b) for b in bags]]))
        loss, by_source, loss_per_bag, by_bag, _ = out
        for key, val in by_source.floats().items():
            preds.setdefault(key, []).append(val)
        lv = float(loss.item())
        if lv < current_loss:
            frozen = retrieve_destinations_low_loss(by_bag, loss_per_bag, mask)
            current_loss = lv
            rest = 0
        else:
            rest += 1
        for node in frozen:
            grad_mask[node] = 0
        weights = reinitialize_weights(data_object, destination_dictionary, model.input.weights.detach(), frozen,
                                       BAGS=False)
    return relation, current_loss, model, preds, v


# ---------------------------------------------------------------------------------------------
# every candidate relation of one scoring round at once (main.py:1309-1330)
# ---------------------------------------------------------------------------------------------
class RelationDictionaries:
    """The edge dictionaries of SEVERAL relations (each: every source of the relation, sorted —
    the first-iteration mask of main.py:734-735 — with its destinations in edge order) as one
    relation-major CSR on the device: key k = (relation index key_rel[k], source keys[k]); the
    graph plan's segment order. Plus the backward's candidate lists per (relation, destination)
    pair, keys descending (score_scatter_kernel's order), and per-relation key ranges."""

    def __init__(self, edge_index, edge_type, relations, num_nodes, device):
        dev = torch.device(device)
        ei, et = edge_index.to(dev), edge_type.to(dev)
        N = int(num_nodes)
        rels = torch.as_tensor([int(r) for r in relations], dtype=torch.int64, device=dev)
        R = int(rels.numel())
        self.relations = [int(r) for r in relations]
        self.num_nodes, self.num_relations = N, R
        # dense index of each edge's relation among `relations` (-1: not scored)
        srt, order = torch.sort(rels)
        pos = torch.searchsorted(srt, et)
        hit = (pos < R) & (srt[pos.clamp(max=max(R - 1, 0))] == et) if R else torch.zeros_like(et, dtype=torch.bool)
        dense = torch.where(hit, order[pos.clamp(max=max(R - 1, 0))], torch.full_like(et, -1)) if R else \
            torch.full_like(et, -1)
        sel = dense >= 0
        src, dst, d = ei[0][sel], ei[1][sel], dense[sel]
        if src.numel() and (int(src.min()) < 0 or int(src.max()) >= N or int(dst.min()) < 0 or int(dst.max()) >= N):
            raise IndexError(f"index out of range: an edge of a scored relation has a node outside [0, {N})")
        key = d * N + src
        o = torch.argsort(key, stable=True)  # (relation, source, edge order)
        key_s, dst_s = key[o], dst[o]
        uk, counts = torch.unique_consecutive(key_s, return_counts=True)
        K = int(uk.numel())
        i32 = torch.int32
        self.keys_t = (uk % N).to(i32)
        self.key_rel_t = (uk // N).to(i32)
        kp = torch.zeros(K + 1, dtype=torch.int64, device=dev)
        torch.cumsum(counts, 0, out=kp[1:])
        self.key_ptr_t = kp.to(i32)
        self.dst_t = dst_s.to(i32)
        rk = torch.zeros(R + 1, dtype=torch.int64, device=dev)
        torch.cumsum(torch.bincount(self.key_rel_t.long(), minlength=R), 0, out=rk[1:])
        self.rel_key_ptr_t = rk.to(i32)
        self.rel_key_ptr = rk.cpu().numpy()
        # backward candidates: every (edge position p, key k) by (relation, destination), k descending
        k_of_p = torch.repeat_interleave(torch.arange(K, device=dev), counts)
        rel_p = (uk // N)[k_of_p]
        target = rel_p * N + dst_s
        comp_order = torch.argsort(target * max(K, 1) + (K - 1 - k_of_p), stable=True)
        tgt_s = target[comp_order]
        ut, tcnt = torch.unique_consecutive(tgt_s, return_counts=True)
        pp = torch.zeros(int(ut.numel()) + 1, dtype=torch.int64, device=dev)
        torch.cumsum(tcnt, 0, out=pp[1:])
        self.pair_ptr_t, self.pair_target_t = pp.to(i32), ut.contiguous()
        self.in_pos_t, self.in_key_t = comp_order.to(i32), k_of_p[comp_order].to(i32)
        self._src_host = None

    @property
    def num_keys(self) -> int:
        return int(self.keys_t.numel())

    def edge_dictionary(self, r: int) -> EdgeDictionary:
        """Relation index r's dictionary as the per-relation path builds it (EdgeDictionary)."""
        b, e = int(self.rel_key_ptr[r]), int(self.rel_key_ptr[r + 1])
        kp = self.key_ptr_t[b:e + 1].long()
        keys = self.keys_t[b:e]
        dst = self.dst_t[int(kp[0]):int(kp[-1])] if e > b else self.dst_t[:0]
        ed, _ = build_edge_dictionary(torch.stack([torch.repeat_interleave(keys.long(), kp[1:] - kp[:-1]),
                                                   dst.long()]),
                                      torch.zeros(dst.numel(), dtype=torch.int64, device=dst.device), 0,
                                      keys.cpu().tolist(), None, num_nodes=self.num_nodes, device=dst.device)
        return ed


def score_relations_batched(data, relations=None, features_dim=2, dataset="synthetic", epochs: int = EPOCHS,
                            trace=None):
    """Every candidate relation of the first metapath-search round (main.py:1309-1330: each
    relation scored by score_relation_parallel, 100 epochs, the relations split over MPI ranks)
    as ONE problem on the GPU: per epoch one argmax launch over all relations' dictionaries (the
    relation-major CSR of ``RelationDictionaries``), the MSE gradient fused into it, one scatter
    launch for the weights' gradients, ONE fused Adam step over the stacked [R, N] weights and
    one clamp — the same elementwise arithmetic per relation as R separate trainings (Adam and
    the clamp are elementwise, the argmax / scatter orders are the per-relation kernels').
    Sources are all nodes with an edge of the relation (the first-iteration mask); labels are per
    node (dataset 'synthetic', main.py:654-656). Weights drawn relation by relation from Python's
    ``random`` and the LinearLayerAttri inits from torch's RNG, in the order a sequential loop of
    score_relation_parallel calls draws them. Returns [(relation, final loss, EdgeDictionary,
    DestinationDictionary)] in ``relations`` order, like the per-relation function; ``trace``
    (a list) receives per epoch (losses [R], argmax node per key) with a host sync each."""
    if dataset != "synthetic":
        raise NotImplementedError("score_relations_batched: labels per mask position (datasets other than "
                                  "'synthetic') differ per relation; score those with score_relation_parallel")
    dev = data.edge_index.device if data.edge_index.is_cuda else torch.device("cuda", torch.cuda.current_device())
    if relations is None:
        relations = torch.unique(data.edge_type).tolist()
    relations = [int(r) for r in relations]
    N = int(data.num_nodes)
    rd = RelationDictionaries(data.edge_index, data.edge_type, relations, N, dev)
    R = rd.num_relations
    # initial weights of every relation at once (initialize_weights, main.py:479-497): per
    # relation, its destinations in first-appearance order over its edges (every source is in the
    # first-iteration mask), weight = |min(labels of its sources) + U(-0.2, 0.2)| with the draws
    # taken from Python's ``random`` relation after relation — the stream of a sequential loop
    ei = data.edge_index.cpu().numpy()
    et = data.edge_type.cpu().numpy()
    lab_h = data.labels.reshape(-1).cpu().numpy().astype(np.float64)
    dense = {r: i for i, r in enumerate(relations)}
    d_of_e = np.array([dense.get(int(v), -1) for v in np.unique(et)], dtype=np.int64)
    d_e = d_of_e[np.searchsorted(np.unique(et), et)] if et.size else np.zeros(0, dtype=np.int64)
    keep = d_e >= 0
    e_idx = np.flatnonzero(keep)
    e_idx = e_idx[np.argsort(d_e[e_idx], kind="stable")]  # relation-major, file order inside
    comp = d_e[e_idx] * N + ei[1][e_idx]
    uniq, first = np.unique(comp, return_index=True)
    order = np.argsort(first, kind="stable")
    pair = uniq[order]                                     # (relation, destination), dictionary order
    srt = np.argsort(comp, kind="stable")
    starts = np.flatnonzero(np.r_[True, comp[srt][1:] != comp[srt][:-1]]) if comp.size else np.zeros(0, np.int64)
    mins = (np.minimum.reduceat(lab_h[ei[0][e_idx][srt]], starts) if comp.size else np.zeros(0))[order]
    draws = np.array([random.uniform(-0.2, 0.2) for _ in range(pair.size)], dtype=np.float64)
    W0 = torch.zeros(R * N)
    if pair.size:
        W0[torch.from_numpy(pair)] = torch.from_numpy(np.abs(mins + draws)).float()
    for _ in range(R):  # get_model's LinearLayerAttri init per relation (main.py:518-519): torch's RNG stream
        nn.Linear(features_dim, 1, bias=False)
    weights = nn.Parameter(W0.to(dev))
    counts = torch.from_numpy(np.diff(rd.rel_key_ptr)).to(torch.float64)
    alpha = (2.0 / counts.clamp(min=1)).to(torch.float32).to(dev)  # torch's mse norm, 2 / numel, as fp32
    labels = data.labels.reshape(-1).to(dev).to(torch.float32)
    K = rd.num_keys
    i32 = torch.int32
    arg_pos = torch.empty(K, dtype=i32, device=dev)
    max_node = torch.empty(K, dtype=i32, device=dev)
    val = torch.empty(K, dtype=torch.float32, device=dev)
    dval = torch.empty(K, dtype=torch.float32, device=dev)
    sq = torch.empty(K, dtype=torch.float32, device=dev)
    loss = torch.empty(R, dtype=torch.float32, device=dev)
    grad = torch.zeros(R * N, dtype=torch.float32, device=dev)
    use_graph = os.environ.get("MPGNN_LOOP_GRAPH", "1") != "0" and trace is None
    # capturable in both modes: the step count on the device, the bias corrections formed there —
    # the arithmetic of score_relation_parallel's graph-replayed Adam
    opt = torch.optim.Adam([weights], lr=0.1, fused=True, capturable=True)

    def epoch():
        check(lib.mpgnn_score_argmax_multi(weights.data_ptr(), N, _ptr(rd.keys_t), _ptr(rd.key_ptr_t), _ptr(rd.dst_t),
                                           _ptr(rd.key_rel_t), K, labels.data_ptr(), alpha.data_ptr(), _ptr(arg_pos),
                                           _ptr(max_node), _ptr(val), _ptr(dval), _ptr(sq), _stream(dev)),
              "mpgnn_score_argmax_multi")
        check(lib.mpgnn_score_loss_multi(_ptr(sq), rd.rel_key_ptr_t.data_ptr(), R, loss.data_ptr(), _stream(dev)),
              "mpgnn_score_loss_multi")
        check(lib.mpgnn_score_argmax_multi_bwd(_ptr(dval), _ptr(arg_pos), _ptr(rd.pair_ptr_t), _ptr(rd.pair_target_t),
                                               _ptr(rd.in_pos_t), _ptr(rd.in_key_t), int(rd.pair_target_t.numel()),
                                               R * N, grad.data_ptr(), _stream(dev)), "mpgnn_score_argmax_multi_bwd")
        weights.grad = grad
        opt.step()
        with torch.no_grad():
            weights.clamp_(min=0.0, max=1.0)   # main.py:667-669 (LinearLayerAttri: clamp of its init)
        return loss

    from .main import _epochs
    out = None
    for _, out in _epochs(epoch, epochs, use_graph):
        if trace is not None:
            trace.append((out.cpu().numpy().copy(), max_node.cpu().numpy().copy()))
    final = out.cpu().tolist() if out is not None else [float("nan")] * R

    def dest_dict(rel, ri):
        b, e = int(rd.rel_key_ptr[ri]), int(rd.rel_key_ptr[ri + 1])
        return build_edge_dictionary(data.edge_index, data.edge_type, rel, rd.keys_t[b:e].cpu().tolist(), data.labels,
                                     dataset, num_nodes=N, device=dev)[1]
    return [(rel, final[ri], _LazyMapping(lambda ri=ri: rd.edge_dictionary(ri)),
             _LazyMapping(lambda rel=rel, ri=ri: dest_dict(rel, ri))) for ri, rel in enumerate(relations)]


class _LazyMapping(Mapping):
    """A dictionary built on first use (the round's per-relation dictionaries are read only for
    the relations the search keeps)."""

    def __init__(self, factory):
        self._factory, self._obj = factory, None

    def get_object(self):
        if self._obj is None:
            self._obj = self._factory()
        return self._obj

    def __getitem__(self, k):
        return self.get_object()[k]

    def __iter__(self):
        return iter(self.get_object())

    def __len__(self):
        return len(self.get_object())

    def __getattr__(self, name):  # EdgeDictionary attributes (dst_t, keys_t, ...)
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self.get_object(), name)
