"""CPU, world_size 2 (gloo): the dst-range sharding of SURVEY §8e.

Each rank builds its shard plan with the C++ builder (node_2 in its edge-balanced range,
GLOBAL per-(node_1, relation) counts), computes its partial output with the shard oracle,
and one all_reduce(SUM) — the collective the GPU path issues over RCCL — must reproduce the
unsharded reference forward; the all-reduced per-rank gradients must equal the unsharded
gradients. Rendezvous on 127.0.0.1."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, name, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.set_num_threads(1)
        import mpgnn_amd
        from mpgnn_amd import data
        from oracle import rgcn_oracle as orc
        from oracle.shard_oracle import shard_partial_forward
        g = data.config_graph(name) if name != "small" else data.synthetic_graph(400, 5, 9, feat_dim=24, seed=3)
        R = g.num_relations
        F = g.x.shape[1]
        gen = torch.Generator().manual_seed(7)
        W = (torch.rand(R, F, 16, generator=gen) - 0.5).requires_grad_(True)
        root = (torch.rand(F, 16, generator=gen) - 0.5).requires_grad_(True)
        bias = (torch.rand(16, generator=gen) - 0.5).requires_grad_(True)
        x = g.x.clone().requires_grad_(True)
        lo, hi = mpgnn_amd.distributed.shard_ranges(g.edge_index, g.num_nodes, world)[rank]
        plan = mpgnn_amd.GraphPlan(g.edge_index, g.edge_type, g.num_nodes, shard=(lo, hi))
        tables = {k: plan.table(k) for k in ("e_col", "s_ptr", "s_row", "s_rel", "s_cnt")}
        part = shard_partial_forward(tables, x, W, root, bias, (lo, hi))
        out = part.detach().clone()
        dist.all_reduce(out)
        gout = torch.randn(out.shape, generator=torch.Generator().manual_seed(11))
        part.backward(gout)
        grads = [x.grad.clone(), W.grad.clone(), root.grad.clone(), bias.grad.clone()]
        for gr in grads:
            dist.all_reduce(gr)
        # unsharded reference (every rank computes it; rank 0 checks)
        xs = g.x.clone().requires_grad_(True)
        Ws, rs, bs = (t.detach().clone().requires_grad_(True) for t in (W, root, bias))
        ref = orc.rgcn_forward(xs, g.edge_index, g.edge_type, Ws, rs, bs)
        ref.backward(gout)
        # float64 truth (decides elements where the two fp32 summation orders differ)
        x64 = g.x.double().requires_grad_(True)
        W64, r64, b64 = (t.detach().double().requires_grad_(True) for t in (W, root, bias))
        ref64 = orc.rgcn_forward(x64, g.edge_index, g.edge_type, W64, r64, b64)
        ref64.backward(gout.double())
        ok = True
        msgs = []
        from tests._bars import passes

        def close(a, b, t, what):
            nonlocal ok
            good, msg = passes(a, b, t)
            if not good:
                ok = False
                msgs.append(f"{what}: {msg}")

        close(out, ref.detach(), ref64.detach(), "out")
        for a, b, t, w in zip(grads, [xs.grad, Ws.grad, rs.grad, bs.grad], [x64.grad, W64.grad, r64.grad, b64.grad],
                              ["dx", "dW", "droot", "dbias"]):
            close(a, b, t, w)
        # the local edge sets partition the graph
        n_local = torch.tensor([plan.num_edges])
        dist.all_reduce(n_local)
        if int(n_local) != g.num_edges:
            ok = False
            msgs.append(f"edges {int(n_local)} != {g.num_edges}")
        q.put((rank, ok, msgs))
        dist.destroy_process_group()
    except Exception:  # report instead of hanging the parent
        import traceback
        q.put((rank, False, [traceback.format_exc()]))


@pytest.mark.parametrize("name", ["small", "C1"])
def test_dst_sharded_allreduce_matches_unsharded(name):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, ok, msgs in results:
        assert ok, (rank, msgs)


# ------------------------------------------------------------------------------------------
# training-path communication: bucketed async gradient all-reduce + owned-row all-gather
# ------------------------------------------------------------------------------------------
def _reducer_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.set_num_threads(1)
        from mpgnn_amd.distributed import ShardGradReducer, gather_owned_rows, shard_ranges
        msgs = []
        gen = torch.Generator().manual_seed(5)
        F = 6
        W0, r0, b0 = torch.randn(3, F, F, generator=gen), torch.randn(F, F, generator=gen), torch.randn(F, generator=gen)
        xs = [torch.randn(10, F, generator=gen) for _ in range(world)]  # rank k's partial input

        class Layer(torch.nn.Module):  # a sharded layer: a partial result per rank
            def __init__(self, reduce):
                super().__init__()
                self.weight = torch.nn.Parameter(W0.clone())
                self.root = torch.nn.Parameter(r0.clone())
                self.bias = torch.nn.Parameter(b0.clone())
                self.red = ShardGradReducer((self.weight, self.root, self.bias), dist.group.WORLD) if reduce else None

            def forward(self, h):
                w, r, b = self.weight, self.root, self.bias
                if self.red is not None and torch.is_grad_enabled():
                    w, r, b = self.red.tap(w, r, b)
                return torch.tanh(h @ w.sum(0) + h @ r * (rank + 1) + b)

        def run(layer, iters, stale=False, set_to_none=True, accumulate=False):
            grads = []
            for it in range(iters):
                if not accumulate or it == 0:
                    layer.zero_grad(set_to_none=set_to_none)
                if stale and it == 0:
                    layer(xs[rank])  # grad-enabled forward never backpropagated (stale use count)
                out = layer(layer(xs[rank]))  # two uses per step (Net.conv2 is shared, model.py:146)
                (out * (it + 1)).sum().backward()
                grads.append([p.grad.clone() for p in (layer.weight, layer.root, layer.bias)])
            return grads

        plain = run(Layer(False), 2)
        for gs in plain:  # expected: the sum over ranks of the local gradients
            for g_ in gs:
                dist.all_reduce(g_)
        # gradient accumulation (no zero_grad between the backward passes): G1 + G2, each
        # reduced once — never the already-reduced G1 summed over the ranks again
        plain_acc = [plain[0], [a + b for a, b in zip(plain[0], plain[1])]]
        for name, kw, ref in (("set_to_none", {}, plain), ("zero_in_place", {"set_to_none": False}, plain),
                              ("stale_use", {"stale": True}, plain), ("accumulate", {"accumulate": True}, plain_acc),
                              ("accumulate_in_place", {"accumulate": True, "set_to_none": False}, plain_acc)):
            got = run(Layer(True), 2, **kw)
            for it, (a, b) in enumerate(zip(got, ref)):
                for pa, pb, pn in zip(a, b, ("weight", "root", "bias")):
                    if not torch.allclose(pa, pb, rtol=1e-6, atol=1e-6):
                        msgs.append(f"{name} iter {it} {pn}: {float((pa - pb).abs().max()):.3e}")
        # uses the reducer did not count — retain_graph=True and a second
        # backward of the same graph; two forwards before their backwards. Each deposit must land
        # in a buffer no reduction is reading, and every use be reduced exactly once.
        def twice(layer, retain):
            layer.zero_grad(set_to_none=True)
            if retain:
                out = layer(layer(xs[rank]))
                out.sum().backward(retain_graph=True)
                (out * 2).sum().backward()
            else:
                out_a = layer(layer(xs[rank]))
                out_b = layer(layer(xs[rank]))
                out_a.sum().backward()
                (out_b * 2).sum().backward()
            return [p.grad.clone() for p in (layer.weight, layer.root, layer.bias)]
        for retain in (True, False):
            ref3 = twice(Layer(False), retain)
            for g_ in ref3:
                dist.all_reduce(g_)
            got3 = twice(Layer(True), retain)
            for pa, pb, pn in zip(got3, ref3, ("weight", "root", "bias")):
                if not torch.allclose(pa, pb, rtol=1e-6, atol=1e-6):
                    msgs.append(f"retain={retain} {pn}: {float((pa - pb).abs().max()):.3e}")
        # a later UNSHARDED backward through the same parameters never touches the reducer
        lay = Layer(True)
        run(lay, 1)
        lay.red = None
        lay.zero_grad()
        lay(xs[rank]).sum().backward()
        plain_one = Layer(False)
        plain_one(xs[rank]).sum().backward()
        for pa, pb in zip((lay.weight, lay.root, lay.bias), (plain_one.weight, plain_one.root, plain_one.bias)):
            if not torch.equal(pa.grad, pb.grad):
                msgs.append("unsharded backward after a sharded one differs")
        # torch.autograd.grad over tapped parameters fails loudly (never partial sums)
        lay2 = Layer(True)
        try:
            torch.autograd.grad(lay2(xs[rank]).sum(), [lay2.weight])
            msgs.append("autograd.grad over a sharded layer's parameters did not raise")
        except RuntimeError:
            pass
        # all-gather of owned rows: rank k contributes rows [lo_k, hi_k) only
        ei = torch.randint(0, 37, (2, 300), generator=torch.Generator().manual_seed(2))
        ranges = shard_ranges(ei, 37, world)
        full = torch.randn(37, 4, generator=torch.Generator().manual_seed(3))
        mine = torch.full_like(full, float("nan"))
        lo, hi = ranges[rank]
        mine[lo:hi] = full[lo:hi]
        got = gather_owned_rows(mine, ranges[rank], dist.group.WORLD)
        if not torch.equal(got, full):
            msgs.append("gather_owned_rows differs")
        q.put((rank, not msgs, msgs))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, False, [traceback.format_exc()]))


@pytest.mark.parametrize("world", [2, 3])
def test_grad_reducer_and_owned_row_gather(world):
    """ShardGradReducer: parameter gradients of a layer used twice per step end up as the sum
    over ranks of the local gradients (one async all-reduce per layer), across zero_grad styles
    and after a forward that was never backpropagated; gather_owned_rows assembles the owners'
    rows exactly."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_reducer_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, ok, msgs in res:
        assert ok, (rank, msgs)


# ------------------------------------------------------------------------------------------
# metapath-candidate fan-out (main.py:1430-1452): replicas only
# ------------------------------------------------------------------------------------------
def _fake_train(data, input_dim, hidden_dim, num_rel, output_dim, ll_output_dim, metapaths, **kw):
    meta = metapaths[0]
    return float(sum((i + 1) * r for i, r in enumerate(meta)) % 7) / 7.0 + kw.get("bump", 0.0)


def _fanout_worker(rank, world, port, cands, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from mpgnn_amd import distributed as mdist
        seen = []

        def train(*a, **kw):
            seen.append(a[6][0])
            return _fake_train(*a, **kw)
        scores = mdist.metapath_fanout(None, 2, 64, 4, 64, 2, cands, train_fn=train, bump=0.0)
        q.put((rank, seen, scores))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, None, repr(e)))


def test_rank_slice_matches_reference_partition():
    from mpgnn_amd.distributed import rank_slice
    for n in range(0, 12):
        items = list(range(n))
        for world in (1, 2, 3, 8):
            parts = [rank_slice(items, world, r) for r in range(world)]
            assert sum(parts, []) == items
            ref = [list(a) for a in np.array_split(np.arange(n), world)]
            assert [list(p) for p in parts] == ref


def test_metapath_fanout_world2_gloo():
    cands = [[1, 0], [2], [0, 2, 1], [3, 3], [1], [2, 0]]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fanout_worker, args=(r, 2, port, cands, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    res.sort(key=lambda t: t[0])
    assert all(r[1] is not None for r in res), res
    assert res[0][1] == cands[:3] and res[1][1] == cands[3:]          # contiguous shares
    expected = {str(m): _fake_train(None, 0, 0, 0, 0, 0, [m]) for m in cands}
    assert res[0][2] == expected and res[1][2] == expected            # every rank has the merged dict
    from mpgnn_amd.distributed import best_metapaths
    best = best_metapaths(expected)
    assert list(best.values()) == sorted(expected.values(), reverse=True)[:3]


# ------------------------------------------------------------------------------------------
# inference stack with reduce-scatter between layers (distributed.sharded_stack_forward)
# ------------------------------------------------------------------------------------------
def _stack_worker(rank, world, port, q, side="gathered"):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.set_num_threads(1)
        import mpgnn_amd
        from mpgnn_amd import data
        from oracle import rgcn_oracle as orc
        from oracle.shard_oracle import shard_partial_forward
        g = data.synthetic_graph(500, 4, 8, feat_dim=16, seed=9)
        N, R = g.num_nodes, g.num_relations
        gen = torch.Generator().manual_seed(3)
        layers = [((torch.rand(R, 16, 16, generator=gen) - 0.5), torch.rand(16, 16, generator=gen) - 0.5,
                   torch.rand(16, generator=gen) - 0.5) for _ in range(3)]
        ranges = mpgnn_amd.distributed.shard_ranges(g.edge_index, N, world, side=side)

        def make_conv(W, root, bias):
            def conv(h, ei, et, shard=None, group=None, shard_side="gathered"):
                assert group is None and shard == ranges[rank] and shard_side == side
                lo, hi = shard
                hx = h
                if side == "gathered":
                    hx = torch.zeros_like(h)
                    hx[lo:hi] = h[lo:hi]  # the kernels read only the rank's own rows
                plan = mpgnn_amd.GraphPlan(ei, et, N, shard=shard, shard_side=side)
                tables = {k: plan.table(k) for k in ("e_col", "s_ptr", "s_row", "s_rel", "s_cnt")}
                return shard_partial_forward(tables, hx, W, root, bias, shard)
            return conv

        convs = [make_conv(*p) for p in layers]
        out = mpgnn_amd.distributed.sharded_stack_forward(convs, g.x, g.edge_index, g.edge_type, ranges,
                                                          shard_side=side)
        ref, ref64 = g.x, g.x.double()
        for W, root, bias in layers:
            ref = torch.relu(orc.rgcn_forward(ref, g.edge_index, g.edge_type, W, root, bias))
            ref64 = torch.relu(orc.rgcn_forward(ref64, g.edge_index, g.edge_type, W.double(), root.double(),
                                                bias.double()))
        from tests._bars import passes
        ok, msg = passes(out, ref, ref64)
        # three passes with two in flight (collectives overlapped with the other pass's layer):
        # bit-identical to the single pass
        many = mpgnn_amd.distributed.sharded_stack_forwards(convs, g.x, g.edge_index, g.edge_type, ranges,
                                                            steps=3, inflight=2, shard_side=side)
        if not all(torch.equal(o, out) for o in many):
            ok, msg = False, "pipelined passes differ from the single pass"
        q.put((rank, ok, msg))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.parametrize("world,side", [(2, "gathered"), (3, "gathered"), (2, "rows"), (3, "rows")])
def test_sharded_stack_reduce_scatter_matches_unsharded(world, side):
    """side "gathered": reduce-scatter of partial sums per layer; side "rows": complete rows
    per rank (plan sharded by the aggregating node), all-gather per layer."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stack_worker, args=(r, world, port, q, side)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, ok, msg in res:
        assert ok is not None, msg
        assert ok, (rank, msg)  # the suite's elementwise + normwise bar (tests/_bars.py)
