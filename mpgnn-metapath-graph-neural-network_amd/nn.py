"""Drop-in for ``torch_geometric.nn.RGCNConv`` as the reference uses it (model.py:5,137-138).

PyG 2.3.1 (requirements.txt:7) RGCNConv, no bases/blocks, float features, loop path:
    out = Σ_{r=0}^{R-1} mean_r(x) @ weight[r] + x @ root + bias
(textually ≙ mp_rgcn_layer.py:249-258 with a 3-D weight). Parameter names/shapes and init
order match PyG (weight [R, in, out], root [in, out], bias [out]; glorot, glorot, zeros).
The aggregation + contraction run as gfx950 kernels (functional.rgcn_conv, mode ALL).
"""
from __future__ import annotations

from typing import Optional, Tuple, Union

import torch
from torch import Tensor
from torch.nn import Parameter

from .functional import MODE_ALL, rgcn_conv
from .mp_rgcn_layer import glorot, zeros
from .plan import FLOWS, get_plan

__all__ = ["RGCNConv", "FastRGCNConv", "CustomFastRGCNConv"]


class RGCNConv(torch.nn.Module):
    def __init__(self, in_channels: Union[int, Tuple[int, int]], out_channels: int, num_relations: int,
                 num_bases: Optional[int] = None, num_blocks: Optional[int] = None, aggr: str = "mean",
                 root_weight: bool = True, is_sorted: bool = False, bias: bool = True,
                 flow: str = "source_to_target", node_dim: int = 0, **kwargs):
        super().__init__()
        if num_bases is not None and num_blocks is not None:
            raise ValueError("Can not apply both basis-decomposition and "
                             "block-diagonal-decomposition at the same time.")
        if flow not in FLOWS:
            raise ValueError(f"Expected 'flow' to be either {FLOWS} (got '{flow}')")
        self.aggr = aggr
        self.flow = flow
        self.node_dim = node_dim
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.num_relations = num_relations
        self.num_bases = num_bases
        self.num_blocks = num_blocks
        self.is_sorted = is_sorted
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
            self.weight = Parameter(torch.empty(num_relations, in_channels[0], out_channels))
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
        glorot(self.weight)
        glorot(self.comp)
        glorot(self.root)
        zeros(self.bias)

    def forward(self, x, edge_index, edge_type=None, *, shard=None, group=None, activation=None,
                shard_side="gathered", _grad_stash=None):
        """``shard=(lo, hi)`` + ``group``: this rank owns the edges whose gathered node lies in
        [lo, hi) (dst-range sharding; ``shard_side="rows"``: whose aggregating
        node lies in it, the rank's output rows then being complete); outputs are all-reduced.
        ``activation='relu'`` returns ``F.relu(conv(...))`` (model.py:144,146) with the ReLU
        fused into the layer's last kernel when unsharded."""
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
            raise NotImplementedError("basis / block-diagonal decomposition is not on the RGCN path")
        plan = get_plan(edge_index, edge_type, x.size(0), flow=self.flow, shard=shard, device=x.device,
                        shard_side=shard_side)
        row_range = shard if shard is not None else None
        reduced = False
        weight, root, bias = self.weight, self.root, self.bias
        if group is not None and torch.is_grad_enabled() and \
                any(p is not None and p.requires_grad for p in (weight, root, bias)):
            # partial dW / droot / dbias of this use go to the layer's reducer (not to .grad):
            # one bucketed async all-reduce once every use of the step has been deposited
            # (Net shares conv2 across layers 1..L-1), then added to .grad
            red = self.__dict__.get("_grad_reducer")
            if red is None or red.group is not group:
                from .distributed import ShardGradReducer
                red = ShardGradReducer((weight, root, bias), group)
                self.__dict__["_grad_reducer"] = red
            weight, root, bias = red.tap(weight, root, bias)
            reduced = True
        return rgcn_conv(x, weight, root, bias, plan, MODE_ALL,
                         num_relations=self.num_relations, row_range=row_range, group=group,
                         activation=activation, params_reduced=reduced,
                         grad_stash=_grad_stash if shard is None else None)

    def __repr__(self) -> str:
        return (f"{self.__class__.__name__}({self.in_channels}, "
                f"{self.out_channels}, num_relations={self.num_relations})")


class FastRGCNConv(RGCNConv):
    """``CustomFastRGCNConv`` (mp_rgcn_layer.py:287-357) / PyG ``FastRGCNConv``: the
    transform-then-aggregate formulation of the same layer — per edge ``x_j @ W[edge_type]``
    (:344), scaled by ``1 / deg_(i, rel)`` (:350-355), scatter-summed (:357), ``+ x @ root +
    bias`` (:313-317). Mathematically equal to ``RGCNConv`` (summation order aside), so it runs
    the same aggregate-then-transform kernels, which do 2·S·F_in·F_out instead of
    2·E·F_in·F_out MFMA work (S = distinct (row, relation) segments ≤ E) and never materialise
    the [E, F_in, F_out] weight gather.

    The reference class inherits CustomRGCNConv's 2-D ``weight [F_in, F_out]``
    (mp_rgcn_layer.py:135-136), with which ``torch.bmm`` at :344 raises; this class takes the
    3-D ``weight [R, F_in, F_out]`` of PyG FastRGCNConv (the class it was adapted from), the
    only shape its forward can run with. ``oracle.rgcn_oracle.fast_rgcn_forward`` restates the
    per-edge arithmetic; tests/test_gpu_parity.py checks this layer against it."""


CustomFastRGCNConv = FastRGCNConv
