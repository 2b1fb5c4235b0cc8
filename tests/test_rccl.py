"""GPU: the sharded path over a REAL RCCL process group (backend "nccl") at world size 1.

The gloo tests (test_distributed_gloo.py, test_multirank_gpu.py) check the partition math and
the multi-rank results, but gloo enforces none of RCCL's rules (device tensors, contiguity,
equal per-rank sizes for reduce_scatter_tensor / all_gather_into_tensor, the device_id binding,
stream semantics of async work). Here one spawned process — before any GPU call — initialises
``init_process_group("nccl", device_id=cuda:0)`` with world size 1 and runs, through that group,
every collective the C4 path issues (replaces main.py:1309-1459's mpi4py fan-out):

* ``sharded_stack_forward`` on the C3 graph with ranges [(0, N)] for both shard sides: the
  per-layer reduce_scatter_tensor / all_gather_into_tensor;
* one training step of ``Net(..., shard=(0, N), group=WORLD)``: the forward's per-layer
  all_reduce, grad_x's all_gather_into_tensor, and the bucketed async all_reduce of the
  parameter gradients (ShardGradReducer);
* ``bench.main()`` with MPGNN_BENCH_FORCE_DIST=1 (the sharded bench path at N = 1).

With one rank every collective is an identity, so results must equal the unsharded stack and
gradients BIT FOR BIT: any difference is a bug of the sharded path, not rounding."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    msgs = []
    try:
        import torch.distributed as dist
        os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": "0", "WORLD_SIZE": "1",
                           "LOCAL_RANK": "0"})
        dev = torch.device("cuda", 0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        assert dist.get_backend() == "nccl"
        group = dist.group.WORLD
        import mpgnn_amd
        from mpgnn_amd import data
        from mpgnn_amd.distributed import sharded_stack_forward
        g = data.fb15k237_graph(feat_dim=128, seed=0, recipe="survey")  # C3
        N = g.num_nodes
        x, ei, et = g.x.to(dev), g.edge_index.to(dev), g.edge_type.to(dev)
        torch.manual_seed(10)
        net = mpgnn_amd.Net(128, 128, g.num_relations, 128, 2, 3).to(dev)
        with torch.no_grad():
            for c in (net.conv1, net.conv2):
                c.bias.uniform_(-0.3, 0.3)
        convs = [net.conv1, net.conv2, net.conv2]
        # (1) inference stack: reduce-scatter (gathered side) / all-gather (rows side) per layer
        with torch.no_grad():
            h = x
            for c in convs:
                h = c(h, ei, et, activation="relu")
            for side in ("gathered", "rows"):
                out = sharded_stack_forward(convs, x, ei, et, [(0, N)], group, shard_side=side)
                torch.cuda.synchronize()
                if not torch.equal(out, h):
                    msgs.append(f"sharded_stack_forward[{side}] differs: {float((out - h).abs().max()):.3e}")
        # (2) one training step: per-layer all_reduce, grad_x all_gather, async bucketed dW all_reduce
        twin = mpgnn_amd.Net(128, 128, g.num_relations, 128, 2, 3).to(dev)
        twin.load_state_dict(net.state_dict())
        y = torch.randint(0, 2, (N,), generator=torch.Generator().manual_seed(0)).to(dev)
        idx = torch.arange(0, N, 3, device=dev)
        res = []
        for k, model in enumerate((net, twin)):
            xg = x.clone().requires_grad_(True)
            kw = dict(shard=(0, N), group=group) if k == 0 else {}
            for step in range(2):  # the second backward WITHOUT zero_grad: gradients accumulate
                out = model(xg, ei, et, **kw)
                loss = torch.nn.functional.nll_loss(out.index_select(0, idx), y[idx])
                loss.backward()
            torch.cuda.synchronize()
            res.append([out.detach(), xg.grad] + [p.grad for p in model.parameters()])
        names = ["out", "dx"] + [n for n, _ in net.named_parameters()]
        for n, a, b in zip(names, res[0], res[1]):
            if b is None or a is None or not torch.equal(a, b):
                err = None if (a is None or b is None) else float((a - b).abs().max())
                msgs.append(f"training step {n} differs ({err})")
        # (3) the bench's sharded path at N = 1 through the same process group
        import contextlib
        import io
        import json
        os.environ["MPGNN_BENCH_FORCE_DIST"] = "1"
        sys.argv = ["bench.py", "--gpus", "1", "--steps", "3", "--warmup", "1", "--epoch-steps", "2",
                    "--loop-epochs", "8", "--no-cpu-baseline"]
        import bench
        bench.setup_dist = (lambda n, _f=bench.setup_dist: (0, 1, 0, group))  # the group is already up
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            bench.main()  # destroys the process group at the end
        lines = [json.loads(ln) for ln in buf.getvalue().splitlines() if ln.startswith("{")]
        if len(lines) != 1:
            msgs.append(f"bench printed {len(lines)} JSON lines")
        else:
            ln = lines[0]
            # the loop leg ran through the group (its ms may be None when t(6 + K) - t(6) is
            # within the run-to-run noise of so short a timing: that is reported, not a failure)
            checks = {"value": ln["value"] > 0, "epoch_ms": ln["epoch_ms"] > 0,
                      "shard_side": ln["config"]["shard_side"] == "gathered",
                      "parallelism": "RCCL" in ln["config"]["parallelism"],
                      "loop_epoch": isinstance(ln["loop_epoch"], dict) and "epochs_timed" in ln["loop_epoch"]}
            bad = [k for k, ok in checks.items() if not ok]
            if bad:
                msgs.append(f"bench line fails {bad}: " + str({k: ln.get(k) for k in ("value", "epoch_ms", "loop_epoch")}))
        q.put((msgs, None))
    except BaseException:
        import traceback
        q.put((msgs, traceback.format_exc()))


def test_rccl_world1_sharded_path_bit_exact():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    try:
        msgs, tb = q.get(timeout=400)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert tb is None, tb
    assert not msgs, msgs
