"""Drop-in for the reference module ``mp_rgcn_layer.py`` (``from mp_rgcn_layer import *``).

``CustomRGCNConv`` keeps the reference constructor, forward signature, parameter names/shapes
and init order (mp_rgcn_layer.py:91-155,158-159) so that ``MPNetm`` (model.py:179-228),
its ``state_dict`` and a seed-30 initialisation (main.py:31) are unchanged; the forward runs
the gfx950 kernels through ``functional.rgcn_conv`` (mode SINGLE).
"""
from __future__ import annotations

import math
from typing import Optional, Tuple, Union

import torch
from torch import Tensor
from torch.nn import Parameter

from .functional import MODE_SINGLE, rgcn_conv
from .plan import FLOWS, get_plan

__all__ = ["CustomRGCNConv", "masked_edge_index", "glorot", "zeros"]


def glorot(value):
    """PyG ``inits.glorot`` (mp_rgcn_layer.py:14,152-154): U(±sqrt(6/(fan_in+fan_out)))."""
    if value is None:
        return
    stdv = math.sqrt(6.0 / (value.size(-2) + value.size(-1)))
    with torch.no_grad():
        value.uniform_(-stdv, stdv)


def zeros(value):
    """PyG ``inits.zeros`` (mp_rgcn_layer.py:155)."""
    if value is not None:
        with torch.no_grad():
            value.fill_(0.0)


def masked_edge_index(edge_index: Tensor, edge_mask: Tensor) -> Tensor:
    """mp_rgcn_layer.py:29-35 (dense branch). Kept for API parity; the layers never call it:
    the graph plan replaces the per-call compaction."""
    if not isinstance(edge_index, Tensor):
        raise NotImplementedError("SparseTensor adjacency (torch_sparse) is not supported")
    return edge_index[:, edge_mask]


def _squeeze_like_reference(out: Tensor, has_root: bool) -> Tensor:
    """mp_rgcn_layer.py:246 squeezes ``zeros + h @ W`` BEFORE the in-place root add (:265).
    When that changes the shape (N == 1 or F_out == 1) the reference's ``out += x @ root``
    raises; without a root weight the squeezed tensor is returned."""
    if out.dim() == 2 and (out.size(0) == 1 or out.size(1) == 1):
        if has_root:
            squeezed = list(out.squeeze().shape)
            raise RuntimeError(f"output with shape {squeezed} doesn't match the broadcast shape "
                               f"{list(out.shape)}")
        return out.squeeze()
    return out


class CustomRGCNConv(torch.nn.Module):
    r"""MPGNN layer: mean aggregation over ONE relation per call, then
    ``out = h_r @ weight + x @ root + bias`` (mp_rgcn_layer.py:40-283, used branch :225-246).

    Args mirror the reference (mp_rgcn_layer.py:91-104). ``flow`` (MessagePassing kwarg) selects
    which row of ``edge_index`` receives the aggregation; callers use 'target_to_source'
    (model.py:190,192). Only ``aggr='mean'`` without bases/blocks is the reference's live path.
    """

    def __init__(self, in_channels: Union[int, Tuple[int, int]], out_channels: int, num_relations: int,
                 num_bases: Optional[int] = None, num_blocks: Optional[int] = None, aggr: str = "mean",
                 root_weight: bool = True, bias: bool = True, flow: str = "source_to_target",
                 node_dim: int = 0, **kwargs):
        super().__init__()
        if num_bases is not None and num_blocks is not None:
            raise ValueError("Can not apply both basis-decomposition and "
                             "block-diagonal-decomposition at the same time.")
        if flow not in FLOWS:
            raise ValueError(f"Expected 'flow' to be either {FLOWS} (got '{flow}')")
        self.aggr = kwargs.pop("aggr", aggr)
        self.flow = flow
        self.node_dim = node_dim
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.num_relations = num_relations
        self.num_bases = num_bases
        self.num_blocks = num_blocks
        if isinstance(in_channels, int):
            in_channels = (in_channels, in_channels)
        self.in_channels_l = in_channels[0]
        if num_bases is not None:
            self.weight = Parameter(torch.empty(num_bases, in_channels[0], out_channels))
            self.comp = Parameter(torch.empty(num_relations, num_bases))
        elif num_blocks is not None:
            assert in_channels[0] % num_blocks == 0 and out_channels % num_blocks == 0
            self.weight = Parameter(torch.empty(num_relations, num_blocks, in_channels[0] // num_blocks,
                                                out_channels // num_blocks))
            self.register_parameter("comp", None)
        else:
            self.weight = Parameter(torch.empty(in_channels[0], out_channels))
            self.register_parameter("comp", None)
        if root_weight:
            self.root = Parameter(torch.empty(in_channels[1], out_channels))
        else:
            self.register_parameter("root", None)
        if bias:
            self.bias = Parameter(torch.empty(out_channels))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        # same RNG consumption order as mp_rgcn_layer.py:151-155
        glorot(self.weight)
        glorot(self.comp)
        glorot(self.root)
        zeros(self.bias)

    def forward(self, layer_num, relation, x, edge_index, edge_type=None, *, activation=None):
        """mp_rgcn_layer.py:158 — ``layer_num`` is accepted and unused, as in the reference.
        ``activation='relu'`` returns ``F.relu(layer(...))`` (MPNetm, model.py:211,214) with the
        ReLU fused into the layer's output kernel."""
        if isinstance(x, tuple):
            raise NotImplementedError("bipartite (x_l, x_r) input is not supported")
        if x is None or x.dtype == torch.long:
            raise NotImplementedError("featureless / index input (x=None or long) is not supported")
        if not isinstance(edge_index, Tensor):
            raise NotImplementedError("SparseTensor adjacency (torch_sparse) is not supported")
        assert edge_type is not None
        if self.aggr != "mean":
            raise NotImplementedError(f"aggr='{self.aggr}' (the reference path uses 'mean')")
        if self.num_bases is not None or self.num_blocks is not None:
            raise NotImplementedError("basis / block-diagonal decomposition is not on the MPGNN path")
        if isinstance(relation, Tensor):
            relation = int(relation.item())
        plan = get_plan(edge_index, edge_type, x.size(0), flow=self.flow, device=x.device)
        out = rgcn_conv(x, self.weight, self.root, self.bias, plan, MODE_SINGLE, relation=int(relation),
                        activation=activation)
        return _squeeze_like_reference(out, self.root is not None)

    def __repr__(self) -> str:
        return (f"{self.__class__.__name__}({self.in_channels}, "
                f"{self.out_channels}, num_relations={self.num_relations})")
