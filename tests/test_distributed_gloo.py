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
        ok = True
        msgs = []

        def close(a, b, what):
            nonlocal ok
            scale = float(b.abs().max())
            err = float((a - b).abs().max())
            if err > 1e-5 * scale + 1e-6:
                ok = False
                msgs.append(f"{what}: err {err:.3e} scale {scale:.3e}")

        close(out, ref.detach(), "out")
        for a, b, w in zip(grads, [xs.grad, Ws.grad, rs.grad, bs.grad], ["dx", "dW", "droot", "dbias"]):
            close(a, b, w)
        # the local edge sets partition the graph
        n_local = torch.tensor([plan.num_edges])
        dist.all_reduce(n_local)
        if int(n_local) != g.num_edges:
            ok = False
            msgs.append(f"edges {int(n_local)} != {g.num_edges}")
        q.put((rank, ok, msgs))
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, False, [repr(e)]))


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
