#!/usr/bin/env python3
"""Per-item timeline of the wave-specialised tile GEMM (debug stamps, MPGNN_OPT_STAMPS):
MFMA-group and memory-group phase lengths and barrier waits, one FB15K layer forward."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402
from mpgnn_amd import _lib, data  # noqa: E402

g = data.config_graph("fb15k237")
x = torch.rand(g.num_nodes, 128, device="cuda")
ei, et = g.edge_index.cuda(), g.edge_type.cuda()
conv = mpgnn_amd.RGCNConv(128, 128, g.num_relations, flow="target_to_source").cuda()
with torch.no_grad():
    for _ in range(5):
        conv(x, ei, et)
torch.cuda.synchronize()
abl = int(sys.argv[1]) if len(sys.argv) > 1 else 0
_lib.lib.mpgnn_set_option(4, 1)            # wave-specialised kernel (carries the stamps)
_lib.lib.mpgnn_set_option(1, abl << 8)     # its ablation bits (1 stores, 2 A loads, 4 weight loads)
buf = torch.zeros((1 << 20) + 65536 * 8, dtype=torch.int64, device="cuda")  # + row_sum stamps region
_lib.lib.mpgnn_set_option(2, buf.data_ptr())
with torch.no_grad():
    conv(x, ei, et)
torch.cuda.synchronize()
_lib.lib.mpgnn_set_option(2, 0)
_lib.lib.mpgnn_set_option(1, 0)
_lib.lib.mpgnn_set_option(4, 0)
st = buf[: 256 * 128].cpu().numpy().reshape(256, 8, 2, 8)  # wg, item, (mfma, mem), stamps
res = {}
ph_m, ph_s, wait_m, wait_s, item_t = [], [], [], [], []
m_pre, m_strip, m_stage, s_commit, s_issue, s_store = [], [], [], [], [], []
for wg in range(256):
    for i in range(8):
        m, s = st[wg, i, 0], st[wg, i, 1]
        if m[0] == 0 or s[0] == 0:
            continue
        ph_m.append(m[1] - m[0]); ph_s.append(s[1] - s[0])
        wait_m.append(m[2] - m[1]); wait_s.append(s[2] - s[1])
        item_t.append(max(m[2], s[2]) - min(m[0], s[0]))
        m_pre.append(m[4] - m[0]); m_strip.append(m[5] - m[4]); m_stage.append(m[1] - m[5])
        s_commit.append(s[4] - s[0]); s_issue.append(s[5] - s[4]); s_store.append(s[1] - s[5])
for name, arr in [("mfma_phase", ph_m), ("mem_phase", ph_s), ("mfma_barrier_wait", wait_m),
                  ("mem_barrier_wait", wait_s), ("item", item_t), ("mfma_pre", m_pre), ("mfma_strip", m_strip),
                  ("mfma_stage", m_stage), ("mem_commit", s_commit), ("mem_issue", s_issue), ("mem_store", s_store)]:
    a = np.array(arr, dtype=np.float64)
    res[name] = {"p50": float(np.median(a)), "p90": float(np.percentile(a, 90)), "max": float(a.max()), "n": len(a)}
# first item vs later items
first = [st[wg, 0, 1, 1] - st[wg, 0, 1, 0] for wg in range(256) if st[wg, 0, 1, 0]]
res["mem_phase_item0_p50"] = float(np.median(first))
wg_span = [st[wg, :, :, 2].max() - st[wg, 0, 0, 0] for wg in range(256) if st[wg, 0, 0, 0]]
res["wg_span_p50"] = float(np.median(wg_span))
res["wg_span_max"] = float(np.max(wg_span))
print(json.dumps(res))
