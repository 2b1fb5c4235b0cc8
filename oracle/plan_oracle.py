"""numpy ORACLE for the integer graph plan — TEST INFRASTRUCTURE ONLY.

Restates, with ``np.lexsort`` (stable), the index bookkeeping the reference performs on every
call: the order-preserving compaction ``edge_index[:, edge_type == r]`` (mp_rgcn_layer.py:29-35,
called at :231 / per relation in the RGCNConv loop ≙ :250-251) and the (node_1 → rows,
node_2 → gathered) roles of PyG propagate under flow='target_to_source' (model.py:137,190).

``build_plan`` returns the same tables the C++ builder exports (include/mpgnn_rgcn.h
``mpgnn_table``), so tests compare them bit-for-bit. Only tests/ may import this module.
"""
from __future__ import annotations

import numpy as np

TILE_ROWS = 64
FLAT_CHUNK = 32
FLAT_CHUNK_ROW_MAJOR = 32  # the row-major (combine) list (plan_internal.h kFlatChunkRowMajor)
FLAT_GROUP = 4             # chunks per normal workgroup group (kFlatGroup)
FLAT_LONG_PIECES = 16      # pieces of a run one workgroup sums in LDS (kFlatLongPieces)


def build_plan(edge_index: np.ndarray, edge_type: np.ndarray, num_nodes: int,
               shard_lo: int = 0, shard_hi: int | None = None) -> dict:
    n1 = np.asarray(edge_index[0], dtype=np.int64)
    n2 = np.asarray(edge_index[1], dtype=np.int64)
    et = np.asarray(edge_type, dtype=np.int64)
    N = int(num_nodes)
    shard_hi = N if shard_hi is None else min(int(shard_hi), N)
    shard_lo = max(int(shard_lo), 0)
    E = n1.shape[0]
    rel_values = np.unique(et)
    rel_d = np.searchsorted(rel_values, et)
    valid = (n1 >= 0) & (n1 < N) & (n2 >= 0) & (n2 < N)
    rel_invalid = np.zeros(len(rel_values), dtype=np.uint8)
    rel_invalid[np.unique(rel_d[~valid])] = 1

    ids = np.nonzero(valid)[0]
    order = ids[np.lexsort((ids, n1[ids], rel_d[ids]))]          # (rel, node_1, edge)
    key_d, key_r = rel_d[order], n1[order]
    new_run = np.ones(len(order), dtype=bool)
    new_run[1:] = (key_d[1:] != key_d[:-1]) | (key_r[1:] != key_r[:-1])
    run_id = np.cumsum(new_run) - 1
    run_cnt = np.bincount(run_id, minlength=run_id.max() + 1 if len(run_id) else 0)
    local = (n2[order] >= shard_lo) & (n2[order] < shard_hi)
    loc = order[local]
    loc_run = run_id[local]
    # segments = runs with >= 1 local edge, in run order
    seg_new = np.ones(len(loc), dtype=bool)
    seg_new[1:] = loc_run[1:] != loc_run[:-1]
    seg_of_edge = np.cumsum(seg_new) - 1
    seg_first = np.nonzero(seg_new)[0]
    S = len(seg_first)
    s_ptr = np.append(seg_first, len(loc)).astype(np.int32)
    s_row = n1[loc[seg_first]].astype(np.int32)
    s_reld = rel_d[loc[seg_first]]
    s_rel = rel_values[s_reld].astype(np.int64)
    s_rel = np.where((s_rel >= 0) & (s_rel <= np.iinfo(np.int32).max), s_rel, -1).astype(np.int32)
    s_cnt = run_cnt[loc_run[seg_first]].astype(np.int32)
    R = len(rel_values)
    rel_seg_ptr = np.zeros(R + 1, dtype=np.int32)
    np.add.at(rel_seg_ptr, s_reld + 1, 1)
    rel_seg_ptr = np.cumsum(rel_seg_ptr).astype(np.int32)
    rel_edge_ptr = s_ptr[rel_seg_ptr].astype(np.int32)

    seg_ids = np.arange(S)
    rw_seg = seg_ids[np.lexsort((seg_ids, s_row))].astype(np.int32)   # (node_1, rel)
    s_pos = np.empty(S, dtype=np.int32)
    s_pos[rw_seg] = np.arange(S, dtype=np.int32)
    rw_ptr = np.zeros(N + 1, dtype=np.int32)
    np.add.at(rw_ptr, s_row.astype(np.int64) + 1, 1)
    rw_ptr = np.cumsum(rw_ptr).astype(np.int32)

    e_col = n2[loc].astype(np.int32)
    k = np.arange(len(loc))
    by_col = k[np.lexsort((k, e_col))]                  # (node_2, rel, node_1, edge)
    t_seg = seg_of_edge[by_col].astype(np.int32)
    t_ptr = np.zeros(N + 1, dtype=np.int32)
    np.add.at(t_ptr, e_col.astype(np.int64) + 1, 1)
    t_ptr = np.cumsum(t_ptr).astype(np.int32)
    edge_reld = s_reld[seg_of_edge]
    pos = np.arange(len(by_col))
    by_rel_col = by_col[np.lexsort((pos, edge_reld[by_col]))]   # stable by rel over col-major
    ta_col = e_col[by_rel_col].astype(np.int32)
    ta_seg = seg_of_edge[by_rel_col].astype(np.int32)

    out = dict(
        rel_values=rel_values.astype(np.int64), rel_seg_ptr=rel_seg_ptr, rel_edge_ptr=rel_edge_ptr,
        e_col=e_col, e_id=loc.astype(np.int32), s_ptr=s_ptr, s_row=s_row, s_rel=s_rel,
        s_cnt=s_cnt, s_pos=s_pos, rw_ptr=rw_ptr, rw_seg=rw_seg, t_ptr=t_ptr, t_seg=t_seg,
        ta_col=ta_col, ta_seg=ta_seg, rel_invalid=rel_invalid,
    )
    # multi-edge segments: a segment whose mean is one x row (one local edge, global count 1) is
    # read from x (s_src = node_2); the others are rows m of the compact means (s_src = -(m+1))
    loc_cnt = np.diff(s_ptr)
    multi = ~((loc_cnt == 1) & (s_cnt == 1))
    m_of = np.cumsum(multi) - multi                      # exclusive prefix
    s_src = np.where(multi, -(m_of + 1), e_col[np.minimum(s_ptr[:-1], max(len(e_col) - 1, 0))] if S else 0)
    m_seg = np.nonzero(multi)[0]
    m_ptr = np.append(0, np.cumsum(loc_cnt[m_seg])).astype(np.int32)
    em_col = (np.concatenate([e_col[s_ptr[s]:s_ptr[s + 1]] for s in m_seg]) if len(m_seg)
              else np.zeros(0, np.int64)).astype(np.int32)
    rel_m_ptr = np.append(m_of, len(m_seg))[rel_seg_ptr].astype(np.int32)
    out.update(s_src=np.asarray(s_src, dtype=np.int32).reshape(S), m_ptr=m_ptr, em_col=em_col,
               m_cnt=s_cnt[m_seg].astype(np.int32), rel_m_ptr=rel_m_ptr)
    for name, run_ptr, cuts, chunk in (("seg", s_ptr, rel_seg_ptr, FLAT_CHUNK), ("t", t_ptr, np.array([0, N]), FLAT_CHUNK),
                                       ("rw", rw_ptr, np.array([0, N]), FLAT_CHUNK_ROW_MAJOR),
                                       ("segm", m_ptr, rel_m_ptr, FLAT_CHUNK)):
        for k, v in build_flat(run_ptr, cuts, chunk).items():
            out[f"{name}_f_{k}"] = v
    return out


def build_flat(run_ptr: np.ndarray, cuts: np.ndarray, chunk: int = FLAT_CHUNK) -> dict:
    """Flat chunked list over runs (run r = positions [run_ptr[r], run_ptr[r+1]), output row r),
    as the fast-path row sums consume it (plan_internal.h FlatHost): chunks of at most ``chunk``
    positions holding complete runs, cut at run ends (and at the forced run cuts ``cuts``); a run
    longer than a chunk is cut into pieces that hold only that run. Workgroup groups: up to
    FLAT_GROUP chunks of complete runs, or — for a run of 2..FLAT_LONG_PIECES pieces — that run's
    pieces alone (group_long = 1; chunk_info carries the piece index). A run of more pieces is
    split across groups of FLAT_GROUP pieces with one global carry slot per piece (split tables).
    chunk_info: bit0 first run split (starts earlier), bit1 last run split (continues later),
    >> 2 carry slot."""
    run_ptr = np.asarray(run_ptr, dtype=np.int64)
    runs = len(run_ptr) - 1
    row_of = np.repeat(np.arange(max(runs, 0)), np.diff(run_ptr)) if runs > 0 else np.zeros(0, np.int64)
    bounds, info, gptr, glong = [0], [], [0], []
    split_rows, split_ptr, split_slot = [], [0], []
    slot = 0

    def close_group(is_long):
        if len(bounds) - 1 > gptr[-1]:
            gptr.append(len(bounds) - 1)
            glong.append(is_long)

    for a, b in zip(cuts[:-1], cuts[1:]):
        cs = int(run_ptr[a])
        for r in range(int(a), int(b)):
            q, e = int(run_ptr[r]), int(run_ptr[r + 1])
            if e - q <= chunk:
                if e - cs > chunk:         # run r does not fit the open chunk: close it before r
                    bounds.append(q)
                    info.append(0)
                    cs = q
                    if len(bounds) - 1 - gptr[-1] == FLAT_GROUP:
                        close_group(0)
                continue
            if q > cs:                     # long run: close the open chunk and group
                bounds.append(q)
                info.append(0)
            close_group(0)
            k = (e - q + chunk - 1) // chunk
            local = k <= FLAT_LONG_PIECES
            if not local:
                split_rows.append(r)
                split_ptr.append(split_ptr[-1])
            for i in range(k):
                bounds.append(min(q + (i + 1) * chunk, e))
                flags = (1 if i > 0 else 0) | (2 if i + 1 < k else 0)
                if local:
                    info.append(flags | (i << 2))
                else:
                    info.append(flags | (slot << 2))
                    split_slot.append(slot)
                    slot += 1
                    split_ptr[-1] += 1
                    if len(bounds) - 1 - gptr[-1] == FLAT_GROUP:
                        close_group(0)
            close_group(1 if local else 0)
            cs = e
        pe = int(run_ptr[b])
        if pe > cs:
            bounds.append(pe)
            info.append(0)
        close_group(0)
    i32 = lambda v: np.asarray(v, dtype=np.int32)  # noqa: E731
    return dict(chunk_ptr=i32(bounds), chunk_info=i32(info), row_of=i32(row_of), split_row=i32(split_rows),
                split_ptr=i32(split_ptr), split_slot=i32(split_slot), group_ptr=i32(gptr), group_long=i32(glong))


def masked_edges(edge_index: np.ndarray, edge_type: np.ndarray, relation: int) -> np.ndarray:
    """``edge_index[:, edge_type == relation]`` — mp_rgcn_layer.py:35 — as int64 [2, E_r]."""
    return np.asarray(edge_index)[:, np.asarray(edge_type) == relation]
