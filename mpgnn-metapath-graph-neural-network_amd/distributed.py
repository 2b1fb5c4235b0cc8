"""Multi-GPU sharding of the relational layers by gathered-node (node_2) range — SURVEY §8e.

The aggregation is linear in x, so rank k owns the edges whose node_2 (= edge_index[1], the
gathered side under flow='target_to_source') falls in its contiguous range [lo_k, hi_k);
ranges are balanced by edge count. Every rank produces a partial output for ALL node_1 rows
(normalised by the GLOBAL per-(node_1, relation) counts, kept in the plan), adds x @ root +
bias only for rows in its own range, and one all-reduce (RCCL over xGMI with the "nccl"
backend) per layer sums the partials. Backward: grad_x rows are local to the owner of the
range, dW / droot / dbias are partial sums — all reduced by all-reduce.

This replaces the reference's mpi4py object fan-out (main.py:1193-1459), which replicated the
whole graph on every rank and parallelised only over candidate relations/metapaths.
"""
from __future__ import annotations

import numpy as np
import torch

__all__ = ["shard_ranges", "edge_balanced_ranges"]


def edge_balanced_ranges(gathered: np.ndarray | torch.Tensor, num_nodes: int, world: int) -> list[tuple[int, int]]:
    """Contiguous node ranges [lo, hi) of the gathered side with ~equal edge counts."""
    g = gathered.cpu().numpy() if isinstance(gathered, torch.Tensor) else np.asarray(gathered)
    g = g[(g >= 0) & (g < num_nodes)]
    cnt = np.bincount(g, minlength=num_nodes).astype(np.int64)
    cum = np.concatenate([[0], np.cumsum(cnt)])
    total = int(cum[-1])
    bounds = [0]
    for k in range(1, world):
        target = total * k // world
        b = int(np.searchsorted(cum, target, side="left"))
        bounds.append(min(max(b, bounds[-1]), num_nodes))
    bounds.append(num_nodes)
    return [(bounds[k], bounds[k + 1]) for k in range(world)]


def shard_ranges(edge_index: torch.Tensor, num_nodes: int, world: int,
                 flow: str = "target_to_source") -> list[tuple[int, int]]:
    """Per-rank gathered-node ranges for ``edge_index`` (row 1 under target_to_source)."""
    gathered = edge_index[1] if flow == "target_to_source" else edge_index[0]
    return edge_balanced_ranges(gathered, num_nodes, world)
