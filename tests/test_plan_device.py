"""GPU: the plan built on the device (csrc/plan_device.hip, mpgnn_plan_create_device: rocPRIM
radix sorts, device scans, the chunk-start walk of the flat lists) is bit-identical to the host
builder (csrc/plan.cpp) on every table, exported or internal (mpgnn_plan_digest), and to the
numpy restatement (oracle/plan_oracle.py) on the exported ones — the same graphs, shards and
edge cases as tests/test_plan.py, plus graphs large enough for many walk blocks and hub rows
split across workgroups."""
import os
import sys

import numpy as np
import pytest
import torch

import mpgnn_amd
from mpgnn_amd import _lib, data
from oracle import plan_oracle

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_plan import FLAT, TABLES, graphs  # noqa: E402

pytestmark = pytest.mark.gpu


def hub_graph():
    rows = [1, 31, 32, 33, 64, 65, 300, 600, 1100, 2, 5, 40_000, 0, 3]
    n1 = np.concatenate([np.full(k, i) for i, k in enumerate(rows)])
    n2 = np.concatenate([np.arange(k) % 40 for k in rows])
    return "hubs", np.stack([n1, n2]), np.zeros(len(n1), np.int64), 40


def big_graph(seed=0):
    """30k nodes, 6 relations, skewed degrees (hub rows and hub columns), zero-degree nodes."""
    rng = np.random.default_rng(seed)
    E = 400_000
    n1 = np.minimum((rng.pareto(1.2, E) * 20).astype(np.int64), 29_999)
    n2 = rng.integers(0, 30_000, E)
    n2[:50_000] = rng.integers(0, 7, 50_000)  # hub columns: grad_x rows longer than 16 chunks
    et = rng.integers(0, 6, E)
    return "big", np.stack([n1, n2]), et, 30_000


def both(ei, et, N, lo, hi, side="gathered"):
    dev = torch.device("cuda:0")
    eit = torch.from_numpy(np.ascontiguousarray(ei)).to(torch.int64)
    ett = torch.from_numpy(np.asarray(et)).to(torch.int64)
    host = mpgnn_amd.GraphPlan(eit, ett, N, shard=(lo, hi), shard_side=side, build="host")
    devp = mpgnn_amd.GraphPlan(eit.to(dev), ett.to(dev), N, shard=(lo, hi), shard_side=side, build="device")
    return host, devp


CASES = list(graphs()) + [hub_graph(), big_graph()]


@pytest.mark.parametrize("case", CASES, ids=lambda c: c[0])
@pytest.mark.parametrize("shard", [None, (0.0, 0.5), (0.3, 0.7), (0.2, 0.21)])
@pytest.mark.parametrize("side", ["gathered", "rows"])
def test_device_plan_equals_host_plan_and_oracle(case, shard, side):
    name, ei, et, N = case
    lo, hi = (0, N) if shard is None else (int(shard[0] * N), int(shard[1] * N))
    host, devp = both(ei, et, N, lo, hi, side)
    assert devp.digest() == host.digest()
    if side == "gathered":
        ref = plan_oracle.build_plan(ei, et, N, lo, hi)
        for tname in TABLES + FLAT:
            got = devp.table(tname)
            assert got.dtype == ref[tname].dtype, tname
            assert np.array_equal(got, ref[tname]), tname
    for tname in _lib.TABLES:
        assert np.array_equal(devp.table(tname), host.table(tname)), tname


def test_device_plan_64bit_keys_and_sparse_relation_ids():
    """relation count × nodes beyond 2^32 (64-bit sort keys) and relation ids that are far
    apart (negative, 2^40): same tables as the host builder."""
    rng = np.random.default_rng(7)
    N = 3_000_000
    rels = np.array([-5, 0, 1, 2, 3, 7, 11, 2**40] + list(range(100, 1600)), np.int64)
    E = 200_000
    ei = np.stack([rng.integers(0, N, E), rng.integers(0, N, E)])
    et = rels[rng.integers(0, len(rels), E)]
    ei[0, :2000] = rng.integers(0, 50, 2000)  # some multi-edge segments
    host, devp = both(ei, et, N, 0, N)
    assert devp.digest() == host.digest()


def test_device_plan_c2_full_and_layer_parity():
    """At C2 size (100k nodes, 1.65 M edges): digest equal to the host build; an RGCNConv layer on
    the device-built plan gives bitwise the output of the host-built plan."""
    g = data.config_graph("C2")
    host, devp = both(g.edge_index.numpy(), g.edge_type.numpy(), g.num_nodes, 0, g.num_nodes)
    assert devp.digest() == host.digest()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    conv = mpgnn_amd.RGCNConv(128, 128, 16, flow="target_to_source").to(dev)
    x = g.x.to(dev)
    ei, et = g.edge_index.to(dev), g.edge_type.to(dev)
    mpgnn_amd.plan_cache.clear()
    y_dev = conv(x, ei, et)  # CUDA edge tensors: device build ("auto")
    assert mpgnn_amd.get_plan(ei, et, g.num_nodes, device=dev).digest() == host.digest()
    mpgnn_amd.plan_cache.clear()
    os.environ["MPGNN_PLAN_BUILD"] = "host"
    try:
        y_host = conv(x, ei, et)
    finally:
        del os.environ["MPGNN_PLAN_BUILD"]
        mpgnn_amd.plan_cache.clear()
    assert torch.equal(y_dev, y_host)


@pytest.mark.parametrize("seed", range(24))
def test_device_plan_random_graphs(seed):
    """Random shapes: node counts from 1 to 5000, empty / tiny / long rows, duplicate edges,
    sparse and negative relation ids, shards on either side — the device build equals the host
    build on every table (digest)."""
    rng = np.random.default_rng(1000 + seed)
    N = int(rng.choice([1, 2, 7, 64, 333, 5000]))
    E = int(rng.choice([0, 1, 5, 100, 3000, 20000]))
    R = int(rng.integers(1, 12))
    rel_ids = rng.choice(np.array([-9, -1, 0, 1, 2, 3, 5, 8, 13, 1000, 2**35], np.int64), size=R, replace=False)
    hub = int(rng.integers(0, N))
    n1 = np.where(rng.random(E) < 0.2, hub, rng.integers(0, N, E))      # a hub row: long segments
    n2 = np.where(rng.random(E) < 0.2, hub, rng.integers(0, N, E))      # and a hub column: long in-lists
    et = rel_ids[rng.integers(0, R, E)]
    if E and rng.random() < 0.3:
        n1[rng.integers(0, E)] = N + 3                                   # an invalid edge
    side = "rows" if rng.random() < 0.5 else "gathered"
    lo = int(rng.integers(0, N + 1))
    hi = int(rng.integers(lo, N + 1))
    for shard in ((0, N), (lo, hi)):
        host, devp = both(np.stack([n1, n2]), et, N, shard[0], shard[1], side)
        assert devp.digest() == host.digest(), (seed, shard, side)
