"""Multi-GPU sharding of the relational layers by gathered-node (node_2) range — SURVEY §8e.

The aggregation is linear in x, so rank k owns the edges whose node_2 (= edge_index[1], the
gathered side under flow='target_to_source') falls in its contiguous range [lo_k, hi_k);
ranges are balanced by edge count. Every rank produces a partial output for ALL node_1 rows
(normalised by the GLOBAL per-(node_1, relation) counts, kept in the plan), adds x @ root +
bias only for rows in its own range, and one all-reduce (RCCL over xGMI with the "nccl"
backend) per layer sums the partials. Backward: grad_x rows are local to the owner of the
range — one all-gather of the owned rows (``gather_owned_rows``); dW / droot / dbias are
partial sums — each use's partials are deposited in one flat bucket per layer and reduced by
one asynchronous all-reduce once every use of the step has been deposited
(``ShardGradReducer``), overlapped with the earlier layers' backward.

This replaces the reference's mpi4py object fan-out (main.py:1193-1459), which replicated the
whole graph on every rank and parallelised only over candidate relations/metapaths.
"""
from __future__ import annotations

import numpy as np
import torch

__all__ = ["shard_ranges", "edge_balanced_ranges", "rank_slice", "metapath_fanout", "best_metapaths",
           "sharded_stack_forward", "sharded_stack_forwards", "ShardGradReducer", "gather_owned_rows",
           "group_ranges"]


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
_PAD_CACHE: dict = {}


def _padded_index(ranges: list[tuple[int, int]], device) -> tuple[torch.Tensor, int]:
    """Row i of range k goes to padded slot k·m + (i - lo_k), m = the largest range (cached per
    (ranges, device): the index is rebuilt and uploaded once, not per layer call)."""
    key = (tuple(tuple(r) for r in ranges), str(device))
    hit = _PAD_CACHE.get(key)
    if hit is not None:
        return hit
    m = max(hi - lo for lo, hi in ranges)
    idx = torch.cat([torch.arange(lo, hi, dtype=torch.int64) - lo + k * m for k, (lo, hi) in enumerate(ranges)])
    _PAD_CACHE[key] = (idx.to(device), m)
    return _PAD_CACHE[key]


_RANGES_CACHE: dict = {}


def group_ranges(shard: tuple[int, int], group=None) -> list[tuple[int, int]]:
    """Every rank's shard range, gathered once per (group, own range) — a collective on first
    use (all ranks reach it at the same layer call), cached afterwards."""
    import torch.distributed as dist
    key = (id(group), tuple(shard))
    hit = _RANGES_CACHE.get(key)
    if hit is not None:
        return hit
    world = dist.get_world_size(group)
    got = [None] * world
    dist.all_gather_object(got, (int(shard[0]), int(shard[1])), group=group)
    _RANGES_CACHE[key] = [tuple(r) for r in got]
    return _RANGES_CACHE[key]


def gather_owned_rows(g: torch.Tensor, shard: tuple[int, int], group=None) -> torch.Tensor:
    """Assemble a [N, F] tensor of which each rank holds only its own rows [lo_k, hi_k) — the
    grad_x of a node_2-range shard (a rank's edges gather only node_2 rows of its range and its
    root term only touches its own rows, so every other row of its partial grad_x is zero). One
    all-gather of the padded row slabs moves N·F·4·(W-1)/W bytes per rank: half of the all-reduce
    of the full partials it replaces."""
    import torch.distributed as dist
    ranges = group_ranges(shard, group)
    world = len(ranges)
    idx, m = _padded_index(ranges, g.device)
    lo, hi = shard
    f = g.shape[1]
    slab = g.new_empty(m, f)
    slab[:hi - lo] = g[lo:hi]  # the padding rows are never read back
    full = g.new_empty(world * m, f)
    dist.all_gather_into_tensor(full, slab, group=group)
    return full.index_select(0, idx)


class _GradTap(torch.autograd.Function):
    """Identity on a sharded layer's parameters whose backward hands the rank-local partial
    gradients of this use to the layer's ShardGradReducer instead of to autograd's leaf
    accumulation (it returns no gradient for the parameters themselves)."""

    @staticmethod
    def forward(ctx, reducer, *params):
        ctx.reducer = reducer
        return tuple(p.view_as(p) for p in params)

    @staticmethod
    def backward(ctx, *grads):
        ctx.reducer._deposit(grads)
        return (None,) + (None,) * len(grads)


class ShardGradReducer:
    """Bucketed, overlapped all-reduce of one sharded layer's parameter gradients (SURVEY §8e:
    "partial dW_r, droot and dbias go through an all-reduce once per step, bucketed").

    Every grad-enabled forward of the layer passes its parameters through ``tap`` (an identity
    autograd node). The tap's backward receives this use's RANK-LOCAL partial dW / droot / dbias
    and adds them into ONE flat buffer owned by the reducer (the first use of a backward
    overwrites it) — autograd never accumulates partials into ``param.grad``. A layer applied
    several times per forward (``Net.conv2``, model.py:146, shared by layers 1..L-1) has one tap
    per use: once every tap of the step has deposited, ONE asynchronous all-reduce of the flat
    buffer is issued, so it runs behind the backward of the earlier layers. The end-of-backward
    callback launches what is still pending (a tap whose forward was never backpropagated),
    makes the stream wait for the reductions (NCCL: no host block) and ADDS the reduced sums to
    ``param.grad`` (or sets it when None): with no ``zero_grad`` between two backward passes the
    gradients accumulate as G1 + G2, as autograd's own accumulation does.

    Not supported (raises rather than returning partial sums): ``torch.autograd.grad`` with the
    sharded layer's parameters as inputs — the tap hands autograd no parameter gradient, so
    autograd reports them unused."""

    _pending: list = []  # reducers touched by the running backward (one end-of-backward callback)

    def __init__(self, params, group):
        self.params = [p for p in params if p is not None]
        self.group = group
        self.flat = None
        self.outstanding = 0  # grad-enabled forwards (taps) whose backward has not deposited yet
        self.deposits = 0     # deposits in the buffer since it was last reduced
        self.work = None

    def tap(self, *params):
        """The layer's parameters for one grad-enabled forward (None entries pass through)."""
        live = [p for p in params if p is not None and p.requires_grad]
        if not live:
            return params
        self.outstanding += 1
        out = iter(_GradTap.apply(self, *live))
        return tuple(next(out) if (p is not None and p.requires_grad) else p for p in params)

    def _layout(self):
        ps = [p for p in self.params if p.requires_grad]
        total = sum(p.numel() for p in ps)
        if self.flat is None or self.flat.numel() != total or self.flat.device != ps[0].device:
            self.flat = torch.zeros(total, dtype=torch.float32, device=ps[0].device)
        views, off = [], 0
        for p in ps:
            views.append((p, self.flat[off:off + p.numel()].view_as(p)))
            off += p.numel()
        return views

    def _deposit(self, grads):
        if not ShardGradReducer._pending:
            torch.autograd.Variable._execution_engine.queue_callback(ShardGradReducer._finish_all)
        if self not in ShardGradReducer._pending:
            ShardGradReducer._pending.append(self)
        if self.work is not None:
            # a reduction of earlier deposits is still reading and writing the buffer (a use that
            # was not counted: retain_graph=True backward again, or forwards interleaved with
            # backwards): fold its sums into .grad first, then the buffer starts over
            self._drain()
        views = self._layout()
        first = self.deposits == 0
        for (p, v), g in zip(views, grads):
            if g is None:
                if first:
                    v.zero_()
            elif first:
                v.copy_(g)
            else:
                v.add_(g)
        self.deposits += 1
        if self.outstanding > 0:
            self.outstanding -= 1
            if self.outstanding == 0:
                self._launch()  # every counted use deposited: reduce now, behind the earlier layers' backward

    def _launch(self):
        import torch.distributed as dist
        self.work = dist.all_reduce(self.flat, group=self.group, async_op=True)

    def _drain(self):
        """Wait for the in-flight reduction (the stream waits; NCCL: no host block) and add its
        sums into param.grad (assigned when None); the buffer is free afterwards."""
        self.work.wait()
        self.work = None
        for p, v in self._layout():
            if p.grad is None:
                p.grad = v.clone()
            else:
                p.grad.add_(v)
        self.deposits = 0

    @staticmethod
    def _finish_all():
        """End of the backward: reduce what has not been, make the stream wait for every
        reduction, then add the sums into param.grad. Same order on every rank. Uses counted by
        forwards whose backward did not run in this pass are forgotten: the next backward
        launches its reduction here, at its end (correct, without the overlap)."""
        pending, ShardGradReducer._pending = ShardGradReducer._pending, []
        for r in pending:
            if r.work is None and r.deposits > 0:
                r._launch()
        for r in pending:
            if r.work is not None:
                r._drain()
            r.outstanding = 0

    def remove(self):
        """Kept for callers of the hook-based reducer: nothing is registered on the params."""


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
    return sharded_stack_forwards(convs, x, edge_index, edge_type, ranges, group, steps=1, inflight=1,
                                  activation=activation, shard_side=shard_side)[0]


def _stack_pass(convs, x, edge_index, edge_type, ranges, group, activation, shard_side, outs, k):
    """One pass of sharded_stack_forward as a generator: it yields right after issuing each
    layer's collective asynchronously and waits for that collective only when resumed, so the
    scheduler in sharded_stack_forwards can run another pass's layer meanwhile. Every tensor a
    pending collective reads or writes stays referenced here until its wait."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lo, hi = ranges[rank]
    idx, m = _padded_index(ranges, x.device)
    n = x.shape[0]
    act = (lambda t: torch.relu(t)) if activation == "relu" else (lambda t: t)
    h = x
    if shard_side == "rows":
        for conv in convs:
            part = conv(h, edge_index, edge_type, shard=(lo, hi), group=None, shard_side="rows")
            slab = part.new_zeros(m, part.shape[1])
            slab[:hi - lo] = act(part[lo:hi])
            full = part.new_empty(world * m, part.shape[1])
            work = dist.all_gather_into_tensor(full, slab, group=group, async_op=True)
            yield
            work.wait()
            h = full.index_select(0, idx)
        outs[k] = h
        return
    for conv in convs:
        part = conv(h, edge_index, edge_type, shard=(lo, hi), group=None)  # partial sums, all rows
        f = part.shape[1]
        pad = part.new_empty(world * m, f)
        pad.index_copy_(0, idx, part)
        mine = part.new_empty(m, f)
        work = dist.reduce_scatter_tensor(mine, pad, group=group, async_op=True)
        yield
        work.wait()
        h = part.new_empty(n, f)  # only [lo, hi) is written: the only rows the next layer reads
        h[lo:hi] = act(mine[:hi - lo])
    slab = h.new_zeros(m, h.shape[1])
    slab[:hi - lo] = h[lo:hi]
    full = h.new_empty(world * m, h.shape[1])
    work = dist.all_gather_into_tensor(full, slab, group=group, async_op=True)
    yield
    work.wait()
    outs[k] = full.index_select(0, idx)


def sharded_stack_forwards(convs, x: torch.Tensor, edge_index: torch.Tensor, edge_type: torch.Tensor,
                           ranges: list[tuple[int, int]], group=None, steps: int = 1, inflight: int = 2,
                           activation: str | None = "relu", shard_side: str = "gathered") -> list:
    """``steps`` independent passes of ``sharded_stack_forward`` over the same input with up to
    ``inflight`` of them in flight: a pass issues its layer's collective asynchronously and the
    next pass computes its own layer while that collective runs (RCCL on its own HIP stream; the
    compute stream waits for a collective only where the pass that needs its rows continues) —
    the inference-serving overlap of communication with computation. Each pass performs exactly
    the single-pass operations in the single-pass order: outputs bit-identical to
    ``sharded_stack_forward`` (tests/test_distributed_gloo.py). Passes run round robin in the same
    order on every rank, so the collectives match."""
    from collections import deque
    outs = [None] * steps
    live = deque()
    started = 0
    while started < steps or live:
        while len(live) < max(1, inflight) and started < steps:
            live.append(_stack_pass(convs, x, edge_index, edge_type, ranges, group, activation, shard_side, outs,
                                    started))
            started += 1
        gen = live.popleft()
        try:
            next(gen)
            live.append(gen)
        except StopIteration:
            pass
    return outs
