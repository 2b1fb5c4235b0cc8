"""CPU ORACLE for the relation-typed aggregation path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / the timed CPU baseline. The product path
(``mpgnn_amd``) never imports it and has no CPU fallback.

What it restates (pure PyTorch fp32 on the CPU, the same ATen ops the reference reaches):

* ``masked_edge_index``           — mp_rgcn_layer.py:29-35
* ``propagate_mean``              — PyG 2.3.1 ``MessagePassing.propagate`` as invoked at
  mp_rgcn_layer.py:236 with ``flow='target_to_source'`` (model.py:137,190), ``aggr='mean'``
  (mp_rgcn_layer.py:98), ``node_dim=0`` (:104), ``message`` = identity (:274-275):
  ``x_j = x.index_select(0, edge_index[j])``; ``scatter(x_j, edge_index[i], dim_size=size[i],
  reduce='mean')`` = ``zeros.scatter_add_`` / ``count.clamp(min=1)`` (torch_geometric/utils/
  scatter.py of PyG 2.3.1). PyG itself is a third-party dependency (requirements.txt:7,
  torch-geometric==2.3.1) that is absent from /root/reference and from this image.
* ``custom_rgcn_forward``         — CustomRGCNConv.forward, used branch mp_rgcn_layer.py:176-199,
  225-246, 260-271 ("mode SINGLE").
* ``rgcn_forward``                — PyG 2.3.1 RGCNConv.forward loop path (used at
  model.py:137-138), textually ≙ mp_rgcn_layer.py:249-258 with a 3-D weight ("mode ALL").
* ``net_forward`` / ``mpnetm_forward`` — model.py:141-149 and model.py:203-228.
* ``glorot`` / ``zeros``          — PyG inits as called at mp_rgcn_layer.py:151-155.

Pinning: the forward of ``custom_rgcn_forward`` is checked against golden vectors produced by
running the reference's own ``mp_rgcn_layer.py`` / ``model.py`` (tests/golden/make_golden.py),
and the edge-direction / masking / empty-row semantics against the planted ground truth the
reference ships (embedding.dat / label.dat KAT). Gradients come from torch
autograd over this restatement.
"""
from __future__ import annotations

import math

import torch
from torch import Tensor

__all__ = [
    "glorot", "zeros", "masked_edge_index", "propagate_mean", "custom_rgcn_forward",
    "rgcn_forward", "net_forward", "mpnetm_forward", "segment_means",
]


def glorot(value):
    """PyG ``torch_geometric.nn.inits.glorot`` (called at mp_rgcn_layer.py:152-154)."""
    if value is None:
        return
    stdv = math.sqrt(6.0 / (value.size(-2) + value.size(-1)))
    value.data.uniform_(-stdv, stdv)


def zeros(value):
    """PyG ``zeros`` (mp_rgcn_layer.py:155)."""
    if value is not None:
        value.data.fill_(0.0)


def masked_edge_index(edge_index: Tensor, edge_mask: Tensor) -> Tensor:
    """mp_rgcn_layer.py:29-35 (dense Tensor branch)."""
    return edge_index[:, edge_mask]


def propagate_mean(edge_index: Tensor, x: Tensor, size, flow: str = "target_to_source") -> Tensor:
    """PyG 2.3.1 propagate(..., aggr='mean') with the identity message (mp_rgcn_layer.py:236,274)."""
    i, j = (0, 1) if flow == "target_to_source" else (1, 0)
    x_j = x.index_select(0, edge_index[j])
    index = edge_index[i]
    dim_size = size[i]
    count = x_j.new_zeros(dim_size)
    count.scatter_add_(0, index, x_j.new_ones(x_j.size(0)))
    count = count.clamp(min=1)
    out = x_j.new_zeros((dim_size,) + tuple(x_j.shape[1:]))
    out.scatter_add_(0, index.view(-1, 1).expand_as(x_j), x_j)
    return out / count.view(-1, 1)


def custom_rgcn_forward(x: Tensor, edge_index: Tensor, edge_type: Tensor, relation: int,
                        weight: Tensor, root: Tensor | None, bias: Tensor | None,
                        flow: str = "target_to_source") -> Tensor:
    """CustomRGCNConv.forward (mp_rgcn_layer.py:158-271), float features, no bases/blocks."""
    size = (x.size(0), x.size(0))                                   # :191
    out = torch.zeros(x.size(0), weight.size(-1), dtype=x.dtype)    # :198
    tmp = masked_edge_index(edge_index, edge_type == relation)      # :231
    h = propagate_mean(tmp, x, size, flow)                          # :236
    out = out + (h @ weight)                                        # :245
    out = out.squeeze()                                             # :246
    if root is not None:
        out += x @ root                                             # :265
    if bias is not None:
        out += bias                                                 # :268
    return out


def rgcn_forward(x: Tensor, edge_index: Tensor, edge_type: Tensor, weight: Tensor,
                 root: Tensor | None, bias: Tensor | None, flow: str = "target_to_source") -> Tensor:
    """PyG 2.3.1 RGCNConv.forward loop path (≙ mp_rgcn_layer.py:249-258, weight [R, F_in, F_out])."""
    size = (x.size(0), x.size(0))
    out = torch.zeros(x.size(0), weight.size(-1), dtype=x.dtype)
    for i in range(weight.size(0)):
        tmp = masked_edge_index(edge_index, edge_type == i)
        h = propagate_mean(tmp, x, size, flow)
        out = out + (h @ weight[i])
    if root is not None:
        out = out + x @ root
    if bias is not None:
        out = out + bias
    return out


def fast_rgcn_forward(x: Tensor, edge_index: Tensor, edge_type: Tensor, weight: Tensor,
                      root: Tensor | None, bias: Tensor | None, flow: str = "target_to_source") -> Tensor:
    """CustomFastRGCNConv (mp_rgcn_layer.py:287-357) with the 3-D weight of PyG FastRGCNConv:
    per-edge transform x_j @ W[edge_type] (:344), scaled by 1 / deg_(i, rel) (:350-355),
    scatter-summed into row i (:357), then + x @ root (:313) + bias (:316). Transform-then-
    aggregate: the same function as rgcn_forward up to summation order."""
    n, r = x.size(0), weight.size(0)
    i, j = (0, 1) if flow == "target_to_source" else (1, 0)
    index = edge_index[i]
    x_j = x.index_select(0, edge_index[j])
    msg = torch.bmm(x_j.unsqueeze(-2), weight[edge_type]).squeeze(-2)
    norm = torch.nn.functional.one_hot(edge_type, r).to(x.dtype)
    norm = torch.zeros(n, r, dtype=x.dtype).index_add_(0, index, norm)[index]
    norm = torch.gather(norm, 1, edge_type.view(-1, 1))
    norm = 1.0 / norm.clamp_(1.0)
    out = torch.zeros(n, weight.size(-1), dtype=x.dtype).index_add_(0, index, norm * msg)
    if root is not None:
        out = out + x @ root
    if bias is not None:
        out = out + bias
    return out


def segment_means(x: Tensor, edge_index: Tensor, edge_type: Tensor, relation: int,
                  flow: str = "target_to_source") -> Tensor:
    """h = propagate_mean over the edges of one relation (the bit-exact part of the path)."""
    tmp = masked_edge_index(edge_index, edge_type == relation)
    return propagate_mean(tmp, x, (x.size(0), x.size(0)), flow)


def net_forward(params: dict, x: Tensor, edge_index: Tensor, edge_type: Tensor,
                metapath_length: int, act=None) -> Tensor:
    """model.py:141-149 — conv1 at layer 0, the SAME conv2 for layers >= 1, Linear, log_softmax.
    ``act(k, pre)`` replaces the k-th ``F.relu`` (default torch.relu); tests use it to take the
    GPU's side at ReLU kinks (pre-activations within rounding of 0)."""
    act = act or (lambda k, v: torch.relu(v))
    for layer in range(metapath_length):
        p = "conv1." if layer == 0 else "conv2."
        x = act(layer, rgcn_forward(x, edge_index, edge_type, params[p + "weight"],
                                    params.get(p + "root"), params.get(p + "bias")))
    x = x @ params["LinearLayer.weight"].t() + params["LinearLayer.bias"]
    return torch.log_softmax(x, dim=1)


def mpnetm_forward(params: dict, x: Tensor, edge_index: Tensor, edge_type: Tensor,
                   metapaths, act=None) -> Tensor:
    """model.py:203-228 in eval mode (Dropout(0.6) is the identity). ``act(k, pre)`` replaces
    the k-th ReLU in call order (default torch.relu; see net_forward)."""
    act = act or (lambda k, v: torch.relu(v))
    k = 0
    embeddings = []
    for i, mp in enumerate(metapaths):
        h = x
        for layer, rel in enumerate(mp):
            p = f"layers_list.{i}.{layer}."
            h = act(k, custom_rgcn_forward(h, edge_index, edge_type, rel, params[p + "weight"],
                                           params.get(p + "root"), params.get(p + "bias")))
            k += 1
        embeddings.append(h)
    h = torch.cat(embeddings, dim=1)
    h = act(k, h @ params["fc1.weight"].t() + params["fc1.bias"])
    h = h @ params["fc2.weight"].t() + params["fc2.bias"]
    return torch.log_softmax(h, dim=1)
