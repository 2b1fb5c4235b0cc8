"""CPU ORACLE of the dst-range-sharded layer — TEST INFRASTRUCTURE ONLY.

Restates, over one shard's plan tables (csrc/plan.cpp: e_col, s_ptr, s_row, s_rel, s_cnt), the
partial output a rank contributes before the all-reduce:
    P_k[i] = Σ_{segments (i, r) with a local edge} (Σ_{local e} x[node_2(e)]) / cnt_global(i, r) @ W_r
             + [i in own rows] (x[i] @ root + bias)
so that Σ_k P_k equals rgcn_forward (the PyG-2.3.1 loop ≙ mp_rgcn_layer.py:249-258) and,
by autograd, the summed per-rank gradients equal the unsharded ones.
"""
from __future__ import annotations

import numpy as np
import torch


def shard_partial_forward(tables: dict, x: torch.Tensor, weight: torch.Tensor, root, bias,
                          rows: tuple[int, int]) -> torch.Tensor:
    N = x.size(0)
    out = torch.zeros(N, weight.size(-1), dtype=x.dtype)
    s_ptr = tables["s_ptr"].astype(np.int64)
    seg_of_edge = torch.from_numpy(np.repeat(np.arange(len(s_ptr) - 1), np.diff(s_ptr)))
    e_col = torch.from_numpy(tables["e_col"].astype(np.int64))
    s_row = torch.from_numpy(tables["s_row"].astype(np.int64))
    s_rel = tables["s_rel"].astype(np.int64)
    cnt = torch.from_numpy(tables["s_cnt"].astype(np.float32))
    S = len(s_ptr) - 1
    sums = torch.zeros(S, x.size(1), dtype=x.dtype).index_add(0, seg_of_edge, x.index_select(0, e_col))
    h = sums / cnt.view(-1, 1)
    for r in np.unique(s_rel):
        if r < 0 or r >= weight.size(0):
            continue
        m = torch.from_numpy(np.nonzero(s_rel == r)[0])
        out = out.index_add(0, s_row[m], h[m] @ weight[int(r)])
    lo, hi = rows
    own = torch.zeros(N, 1, dtype=x.dtype)
    own[lo:hi] = 1.0
    if root is not None:
        out = out + own * (x @ root)
    if bias is not None:
        out = out + own * bias
    return out
