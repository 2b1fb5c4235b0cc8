"""CPU: the C++ graph plan (csrc/plan.cpp, via the C ABI) is bit-identical to the numpy
oracle (oracle/plan_oracle.py) and reproduces the reference's masked edge lists
(``edge_index[:, edge_type == r]``, mp_rgcn_layer.py:35) — order within each node_1 kept."""
import numpy as np
import pytest
import torch

import mpgnn_amd
from mpgnn_amd import data
from oracle import plan_oracle

TABLES = ["rel_values", "rel_seg_ptr", "rel_edge_ptr", "e_col", "e_id", "s_ptr", "s_row", "s_rel",
          "s_cnt", "s_pos", "rw_ptr", "rw_seg", "t_ptr", "t_seg", "ta_col", "ta_seg", "rel_invalid",
          "s_src", "m_ptr", "em_col", "m_cnt", "rel_m_ptr"]
FLAT = [f"{l}_f_{n}" for l in ("seg", "t", "rw", "segm")
        for n in ("chunk_ptr", "chunk_info", "row_of", "split_row", "split_ptr", "split_slot", "group_ptr",
                  "group_long")]


def graphs():
    g1 = data.config_graph("C1")
    yield "C1", g1.edge_index.numpy(), g1.edge_type.numpy(), g1.num_nodes
    g2 = data.synthetic_graph(3000, 7, 40, seed=5)
    yield "dense7", g2.edge_index.numpy(), g2.edge_type.numpy(), 3000
    rng = np.random.default_rng(3)
    # duplicates, self loops, relation gaps, negative and huge relation ids
    ei = rng.integers(0, 50, size=(2, 400))
    et = rng.choice([-7, 0, 3, 3, 9, 2**40], size=400)
    yield "weird_ids", ei, et, 50
    # invalid node ids in some relations
    ei2 = rng.integers(0, 60, size=(2, 300))
    et2 = rng.integers(0, 5, size=300)
    ei2[0, 7] = 60      # relation et2[7] flagged
    ei2[1, 11] = -1     # relation et2[11] flagged
    yield "invalid", ei2, et2, 60
    yield "empty", np.zeros((2, 0), np.int64), np.zeros(0, np.int64), 10
    yield "single", np.array([[3], [5]]), np.array([1]), 8
    yield "no_nodes", np.zeros((2, 0), np.int64), np.zeros(0, np.int64), 0


@pytest.mark.parametrize("case", list(graphs()), ids=lambda c: c[0])
@pytest.mark.parametrize("shard", [None, (0.0, 0.5), (0.5, 1.0), (0.2, 0.21)])
def test_plan_tables_bit_exact(case, shard):
    name, ei, et, N = case
    lo, hi = (0, N) if shard is None else (int(shard[0] * N), int(shard[1] * N))
    plan = mpgnn_amd.GraphPlan(torch.from_numpy(np.ascontiguousarray(ei)), torch.from_numpy(et), N,
                               shard=(lo, hi))
    ref = plan_oracle.build_plan(ei, et, N, lo, hi)
    for tname in TABLES:
        got = plan.table(tname)
        assert got.dtype == ref[tname].dtype, tname
        assert np.array_equal(got, ref[tname]), tname


@pytest.mark.parametrize("case", list(graphs())[:3], ids=lambda c: c[0])
def test_masked_edge_lists_match_reference_semantics(case):
    name, ei, et, N = case
    plan = mpgnn_amd.GraphPlan(torch.from_numpy(np.ascontiguousarray(ei)), torch.from_numpy(et), N)
    rel_values = plan.table("rel_values")
    rep = plan.table("rel_edge_ptr")
    e_id = plan.table("e_id")
    for d, r in enumerate(rel_values):
        masked = plan_oracle.masked_edges(ei, et, r)            # reference order
        ids = e_id[rep[d]:rep[d + 1]]
        got = np.asarray(ei)[:, ids]
        # same multiset of edges; our order = stable sort of the reference order by node_1
        order = np.argsort(masked[0], kind="stable")
        assert np.array_equal(got, masked[:, order])


def test_segment_counts_are_global_across_shards():
    g = data.config_graph("C1")
    N = g.num_nodes
    full = mpgnn_amd.GraphPlan(g.edge_index, g.edge_type, N)
    key = lambda p: dict(zip(zip(p.table("s_row").tolist(), p.table("s_rel").tolist()),
                             p.table("s_cnt").tolist()))
    ref = key(full)
    ranges = mpgnn_amd.distributed.shard_ranges(g.edge_index, N, 4)
    total_edges = 0
    for lo, hi in ranges:
        p = mpgnn_amd.GraphPlan(g.edge_index, g.edge_type, N, shard=(lo, hi))
        total_edges += p.num_edges
        for k, c in key(p).items():
            assert ref[k] == c
        assert np.all((p.table("e_col") >= lo) & (p.table("e_col") < hi))
    assert total_edges == full.num_edges


def test_shard_ranges_balanced_and_cover():
    g = data.config_graph("C2")
    for world in (1, 2, 4, 8):
        r = mpgnn_amd.distributed.shard_ranges(g.edge_index, g.num_nodes, world)
        assert r[0][0] == 0 and r[-1][1] == g.num_nodes
        assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
        col = g.edge_index[1].numpy()
        counts = [int(((col >= lo) & (col < hi)).sum()) for lo, hi in r]
        assert max(counts) - min(counts) <= 0.01 * g.num_edges + 64


def test_select_ranges():
    g = data.synthetic_graph(500, 6, 8, seed=1)
    p = mpgnn_amd.GraphPlan(g.edge_index, g.edge_type, 500)
    rsp = p.table("rel_seg_ptr")
    assert p.select(mpgnn_amd.MODE_ALL, -1, 6) == (0, p.num_segments)
    assert p.select(mpgnn_amd.MODE_ALL, -1, 3) == (0, int(rsp[3]))
    assert p.select(mpgnn_amd.MODE_SINGLE, 4, 0) == (int(rsp[4]), int(rsp[5]))
    b, e = p.select(mpgnn_amd.MODE_SINGLE, 99, 0)      # absent relation: empty mask, no error
    assert b == e


def test_invalid_index_raises_index_error_only_for_touched_relation():
    ei = torch.tensor([[0, 1, 5], [1, 2, 0]])
    et = torch.tensor([0, 0, 1])
    p = mpgnn_amd.GraphPlan(ei, et, 3)          # node 5 >= N=3 in relation 1
    p.select(mpgnn_amd.MODE_SINGLE, 0, 0)
    with pytest.raises(IndexError):
        p.select(mpgnn_amd.MODE_SINGLE, 1, 0)
    with pytest.raises(IndexError):
        p.select(mpgnn_amd.MODE_ALL, -1, 2)
    p.select(mpgnn_amd.MODE_ALL, -1, 1)          # only relation 0 touched


def test_source_to_target_flow_swaps_roles():
    g = data.config_graph("C1")
    a = mpgnn_amd.GraphPlan(g.edge_index, g.edge_type, g.num_nodes, flow="source_to_target")
    b = mpgnn_amd.GraphPlan(g.edge_index.flip(0), g.edge_type, g.num_nodes)
    for tname in TABLES:
        assert np.array_equal(a.table(tname), b.table(tname))


def test_plan_cache_reuses_and_invalidates():
    g = data.config_graph("C1")
    mpgnn_amd.plan_cache.clear()
    p1 = mpgnn_amd.get_plan(g.edge_index, g.edge_type, g.num_nodes)
    p2 = mpgnn_amd.get_plan(g.edge_index, g.edge_type, g.num_nodes)
    assert p1 is p2
    g.edge_type[0] = (g.edge_type[0] + 1) % 3       # in-place edit bumps _version
    p3 = mpgnn_amd.get_plan(g.edge_index, g.edge_type, g.num_nodes)
    assert p3 is not p1


@pytest.mark.parametrize("case", list(graphs()) + [("hubs", None, None, None)], ids=lambda c: c[0])
@pytest.mark.parametrize("shard", [None, (0.3, 0.7)])
def test_flat_lists_bit_exact_and_well_formed(case, shard):
    """Flat chunked lists (fast-path row sums) == the numpy restatement, and well formed:
    chunks of 1..32 positions covering every position once, cut at row ends; a row longer
    than a chunk is cut into pieces holding only that row; groups of <= 4 chunks of complete
    rows, or the 2..16 pieces of one row (long group); rows of more pieces have one global carry
    slot per piece."""
    name, ei, et, N = case
    if name == "hubs":  # long segments / in-lists: rows of 1, 31, 32, 33, 64, 65, 300, 600, 1100 entries
        rows = [1, 31, 32, 33, 64, 65, 300, 600, 1100, 2, 5]
        n1 = np.concatenate([np.full(k, i) for i, k in enumerate(rows)])
        n2 = np.concatenate([np.arange(k) % 40 for k in rows])
        ei, et, N = np.stack([n1, n2]), np.zeros(len(n1), np.int64), 40
    lo, hi = (0, N) if shard is None else (int(shard[0] * N), int(shard[1] * N))
    plan = mpgnn_amd.GraphPlan(torch.from_numpy(np.ascontiguousarray(ei)), torch.from_numpy(np.asarray(et)), N,
                               shard=(lo, hi))
    ref = plan_oracle.build_plan(ei, et, N, lo, hi)
    for tname in FLAT:
        got = plan.table(tname)
        assert np.array_equal(got, ref[tname]), tname
    for l, run_ptr, chunk in (("seg", ref["s_ptr"], 32), ("t", ref["t_ptr"], 32), ("rw", ref["rw_ptr"], 32),
                              ("segm", ref["m_ptr"], 32)):
        cp = plan.table(f"{l}_f_chunk_ptr")
        sizes = np.diff(cp)
        assert (sizes >= 1).all() and (sizes <= chunk).all(), l
        assert cp[0] == 0 and cp[-1] == (run_ptr[-1] if len(run_ptr) else 0), l
        ends = set(run_ptr.tolist())
        row_of = plan.table(f"{l}_f_row_of")
        info = plan.table(f"{l}_f_chunk_info")
        for c in range(len(cp) - 1):
            a0, a1 = cp[c], cp[c + 1]
            rf, rl = row_of[a0], row_of[a1 - 1]
            if a0 not in ends or a1 not in ends:  # a piece: one long row only
                assert rf == rl and run_ptr[rf + 1] - run_ptr[rf] > chunk, (l, c)
                assert (info[c] & 3) == ((a0 != run_ptr[rf]) | ((a1 != run_ptr[rf + 1]) << 1)), (l, c)
            else:
                assert info[c] == 0, (l, c)
        gp, gl = plan.table(f"{l}_f_group_ptr"), plan.table(f"{l}_f_group_long")
        assert gp[0] == 0 and gp[-1] == len(cp) - 1 and len(gl) == len(gp) - 1, l
        for g in range(len(gl)):
            n = gp[g + 1] - gp[g]
            if gl[g]:  # all pieces of one row, in order, piece index in the info
                rows_g = {row_of[cp[c]] for c in range(gp[g], gp[g + 1])}
                assert len(rows_g) == 1 and 2 <= n <= 16, (l, g)
                assert [info[c] >> 2 for c in range(gp[g], gp[g + 1])] == list(range(n)), (l, g)
            else:
                assert 1 <= n <= 4, (l, g)
        sp, ss = plan.table(f"{l}_f_split_ptr"), plan.table(f"{l}_f_split_slot")
        assert len(np.unique(ss)) == len(ss), l
        for k, r in enumerate(plan.table(f"{l}_f_split_row")):
            assert run_ptr[r + 1] - run_ptr[r] > 16 * chunk, (l, r)
            touched = np.unique(np.searchsorted(cp, np.arange(run_ptr[r], run_ptr[r + 1]), side="right"))
            assert sp[k + 1] - sp[k] == len(touched), (l, r)


@pytest.mark.parametrize("shard", [None, (20_000, 70_000)])
def test_parallel_plan_build_independent_of_thread_count(shard):
    """The host builder splits its passes over threads (MPGNN_OPT_PLAN_THREADS); at C2 size
    (1.65 M edges, well above the one-thread threshold) every exported table is identical
    with 1, 3 and the default number of threads."""
    from mpgnn_amd import _lib
    g = data.config_graph("C2")
    plans = []
    try:
        for threads in (1, 3, 0):
            _lib.check(_lib.lib.mpgnn_set_option(11, threads))
            plans.append(mpgnn_amd.GraphPlan(g.edge_index, g.edge_type, g.num_nodes, shard=shard))
    finally:
        _lib.lib.mpgnn_set_option(11, 0)
    for name in _lib.TABLES:
        ref = plans[0].table(name)
        for p in plans[1:]:
            assert np.array_equal(p.table(name), ref), name


@pytest.mark.parametrize("case", list(graphs()), ids=lambda c: c[0])
@pytest.mark.parametrize("shard", [None, (0.3, 0.7)])
def test_multi_edge_segments_cover_exactly_the_non_trivial_means(case, shard):
    """s_src: a segment reads x[node_2] iff it has one local edge and global count 1 (its mean is
    that row bit for bit); every other segment owns one compact row m whose edge list is the
    segment's own edge list in plan order, with the global count."""
    name, ei, et, N = case
    lo, hi = (0, N) if shard is None else (int(shard[0] * N), int(shard[1] * N))
    plan = mpgnn_amd.GraphPlan(torch.from_numpy(np.ascontiguousarray(ei)), torch.from_numpy(et), N, shard=(lo, hi))
    s_ptr, s_cnt, e_col = plan.table("s_ptr"), plan.table("s_cnt"), plan.table("e_col")
    s_src, m_ptr, em_col, m_cnt = plan.table("s_src"), plan.table("m_ptr"), plan.table("em_col"), plan.table("m_cnt")
    m = 0
    for s in range(len(s_src)):
        b, e = s_ptr[s], s_ptr[s + 1]
        if e - b == 1 and s_cnt[s] == 1:
            assert s_src[s] == e_col[b]
        else:
            assert s_src[s] == -(m + 1)
            assert np.array_equal(em_col[m_ptr[m]:m_ptr[m + 1]], e_col[b:e])
            assert m_cnt[m] == s_cnt[s]
            m += 1
    assert m == len(m_cnt) == len(m_ptr) - 1
    rsp, rmp = plan.table("rel_seg_ptr"), plan.table("rel_m_ptr")
    assert len(rmp) == len(rsp)
    for d in range(len(rsp)):  # rel_m_ptr[d] = multi-edge segments before relation d's first segment
        assert rmp[d] == int((s_src[:rsp[d]] < 0).sum())
