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

__all__ = ["shard_ranges", "edge_balanced_ranges", "rank_slice", "metapath_fanout", "best_metapaths",
           "sharded_stack_forward"]


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
                 flow: str = "target_to_source", side: str = "gathered") -> list[tuple[int, int]]:
    """Per-rank node ranges balanced by edge count: of the gathered node (row 1 under
    target_to_source) for ``side="gathered"``, of the aggregating node for ``side="rows"``."""
    gathered = edge_index[1] if flow == "target_to_source" else edge_index[0]
    aggregating = edge_index[0] if flow == "target_to_source" else edge_index[1]
    return edge_balanced_ranges(aggregating if side == "rows" else gathered, num_nodes, world)


# ---------------------------------------------------------------------------------------
# metapath-candidate fan-out: replicas only
# ---------------------------------------------------------------------------------------
def rank_slice(items: list, world: int, rank: int) -> list:
    """The contiguous share of ``items`` rank ``rank`` trains (main.py:1432-1438: the first
    ``len % world`` ranks take one extra item; ≡ np.array_split(items, world)[rank],
    main.py:1319)."""
    n = len(items)
    size, rem = n // world, n % world
    start = rank * size + min(rank, rem)
    return items[start:start + size + (1 if rank < rem else 0)]


def metapath_fanout(data_mpgnn, input_dim, hidden_dim, num_rel, output_dim, ll_output_dim, metapaths,
                    group=None, train_fn=None, **train_kw) -> dict:
    """Score every candidate metapath with ``mpgnn_parallel_multiple`` (main.py:1117) across
    the ranks of ``group`` — main.py:1430-1449: each rank trains its contiguous share of
    ``metapaths`` (one MPNetm per metapath, on its own GPU) and the {str(metapath): validation
    macro F1} dicts are gathered. The reference gathers to rank 0 over mpi4py; here every rank
    gets the merged dict (all_gather_object over torch.distributed). Candidates are
    independent trainings: no data-path collective, one object gather at the end.
    ``train_fn`` defaults to ``main.mpgnn_parallel_multiple`` (extra keywords go to it)."""
    import torch.distributed as dist
    if train_fn is None:
        from .main import mpgnn_parallel_multiple as train_fn
    if group is not None or (dist.is_available() and dist.is_initialized()):
        world, rank = dist.get_world_size(group), dist.get_rank(group)
    else:
        world, rank = 1, 0
    partial = {}
    for meta in rank_slice(list(metapaths), world, rank):
        partial[str(meta)] = train_fn(data_mpgnn, input_dim, hidden_dim, num_rel, output_dim, ll_output_dim,
                                      [meta], **train_kw)
    if world == 1:
        return partial
    gathered = [None] * world
    dist.all_gather_object(gathered, partial, group=group)
    final = {}
    for d in gathered:  # rank order, as the reference's final_dict.update loop (main.py:1447-1449)
        final.update(d)
    return final


def best_metapaths(scores: dict, k: int = 3) -> dict:
    """main.py:1451-1452: the ``k`` best candidates by score, descending (stable for ties)."""
    ordered = dict(sorted(scores.items(), key=lambda item: item[1], reverse=True))
    return dict(list(ordered.items())[:k])


# ---------------------------------------------------------------------------------------
# inference stack with reduce-scatter between layers
# ---------------------------------------------------------------------------------------
def _padded_index(ranges: list[tuple[int, int]], device) -> tuple[torch.Tensor, int]:
    """Row i of range k goes to padded slot k·m + (i - lo_k), m = the largest range."""
    m = max(hi - lo for lo, hi in ranges)
    idx = torch.cat([torch.arange(lo, hi, dtype=torch.int64) - lo + k * m for k, (lo, hi) in enumerate(ranges)])
    return idx.to(device), m


def sharded_stack_forward(convs, x: torch.Tensor, edge_index: torch.Tensor, edge_type: torch.Tensor,
                          ranges: list[tuple[int, int]], group=None, activation: str | None = "relu",
                          shard_side: str = "gathered") -> torch.Tensor:
    """Forward of a relational layer stack (``relu(conv(h))`` per layer, model.py:141-146) over
    dst-range shards with ONE reduction per layer that moves half the bytes of an all-reduce.

    Rank k owns the gathered-node range ranges[k]: its layer output is a partial sum for every
    row, but the next layer only gathers rows of its own range (its edges' node_2, its root
    rows), so a reduce-scatter of the partials (RCCL over xGMI with the "nccl" backend) gives
    each rank exactly the summed rows it needs; rows outside the range are never read. One
    all-gather after the last layer assembles the full output. Inference path (no autograd
    across ranks): the training path is the per-layer all-reduce of ``RGCNConv(shard=, group=)``.

    ``shard_side="rows"``: rank k owns the edges whose AGGREGATING node lies in ranges[k]
    (ranges then balanced by node_1 edge counts, ``shard_ranges(..., side="rows")``); its layer
    output is complete for its rows and zero elsewhere, every rank gathers from all rows, so each
    layer ends with an all-gather of the rows (same bytes as the reduce-scatter) and every
    per-rank pass — means, transform, combine — shrinks with the shard instead of only the edges."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lo, hi = ranges[rank]
    idx, m = _padded_index(ranges, x.device)
    n = x.shape[0]
    h = x
    if shard_side == "rows":
        for conv in convs:
            part = conv(h, edge_index, edge_type, shard=(lo, hi), group=None, shard_side="rows")
            slab = part.new_zeros(m, part.shape[1])
            slab[:hi - lo] = torch.relu(part[lo:hi]) if activation == "relu" else part[lo:hi]
            full = part.new_empty(world * m, part.shape[1])
            dist.all_gather_into_tensor(full, slab, group=group)
            h = full.index_select(0, idx)
        return h
    for conv in convs:
        part = conv(h, edge_index, edge_type, shard=(lo, hi), group=None)  # partial sums, all rows
        f = part.shape[1]
        pad = part.new_empty(world * m, f)
        pad.index_copy_(0, idx, part)
        mine = part.new_empty(m, f)
        dist.reduce_scatter_tensor(mine, pad, group=group)
        h = part.new_empty(n, f)  # only [lo, hi) is written: the only rows the next layer reads
        h[lo:hi] = torch.relu(mine[:hi - lo]) if activation == "relu" else mine[:hi - lo]
    slab = h.new_zeros(m, h.shape[1])
    slab[:hi - lo] = h[lo:hi]
    full = h.new_empty(world * m, h.shape[1])
    dist.all_gather_into_tensor(full, slab, group=group)
    return full.index_select(0, idx)
