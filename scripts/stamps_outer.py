"""Phase stamps of the bf16-split weight gradient (outer_bf3v_kernel) in the C3 layer backward —
debug build only (make -C csrc stamps -> libmpgnn_rgcn_stamps.so, loaded via MPGNN_LIB_PATH).
Per wave and 16-row slice (the first 32 slices of each workgroup): 0 slice start | 1 MFMAs
issued | 6 the rows two slices ahead issued | 2 next slice committed | 3 chunk-end epilogue done | 5 chunk end (stamped only then) |
4 barrier passed; row 0: ids, start, realtime start / end. Cycles of s_memtime."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MPGNN_LIB_PATH"] = os.path.join(ROOT, "mpgnn-metapath-graph-neural-network_amd", "libmpgnn_rgcn_stamps.so")
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import mpgnn_amd  # noqa: E402
from mpgnn_amd import _lib, data  # noqa: E402

ITEMS, PH = 32, 8
g = data.fb15k237_graph(feat_dim=128)
dev = torch.device("cuda", 0)
torch.manual_seed(10)
conv = mpgnn_amd.RGCNConv(128, 128, g.num_relations, flow="target_to_source").to(dev)
x, ei, et = g.x.to(dev), g.edge_index.to(dev), g.edge_type.to(dev)
gout = torch.randn(g.num_nodes, 128, device=dev)
xg = x.clone().requires_grad_(True)
for _ in range(3):
    conv(xg, ei, et).backward(gout)
torch.cuda.synchronize()
nwaves = 256 * 4 * 4
buf = torch.zeros(nwaves * (ITEMS + 1) * PH, dtype=torch.int64, device=dev)
fn = _lib.lib.mpgnn_debug_stamps_set
fn.argtypes = [ctypes.c_void_p]
out = conv(xg, ei, et)
torch.cuda.synchronize()
assert fn(buf.data_ptr()) == 0
out.backward(gout)
torch.cuda.synchronize()
assert fn(None) == 0
st = buf.view(nwaves, ITEMS + 1, PH).cpu().numpy()
used = st[:, 0, 2] != 0
st = st[used]
t = st[:, 1:, :].astype(np.int64)
valid = (t[:, :, 0] != 0) & (t[:, :, 4] != 0)
pct = lambda d: {p: int(np.percentile(d, p)) for p in (10, 50, 90, 99)} if np.size(d) else None  # noqa: E731
res = {"waves": int(used.sum())}
res["mfma_issue"] = pct((t[:, :, 1] - t[:, :, 0])[valid])
v6 = valid & (t[:, :, 6] != 0)
res["rows_issue"] = pct((t[:, :, 6] - t[:, :, 0])[v6])  # slice start -> next rows issued (index wait)
res["mfma_only"] = pct((t[:, :, 1] - t[:, :, 6])[v6])
res["commit"] = pct((t[:, :, 2] - t[:, :, 1])[valid])
ce = valid & (t[:, :, 5] != 0)
res["chunk_end_frac"] = float(ce.sum() / valid.sum())
res["epilogue_chunk_end"] = pct((t[:, :, 3] - t[:, :, 2])[ce])
res["epilogue_other"] = pct((t[:, :, 3] - t[:, :, 2])[valid & ~ce])
res["barrier"] = pct((t[:, :, 4] - t[:, :, 3])[valid])
res["slice_total"] = pct((t[:, :, 4] - t[:, :, 0])[valid])
start = st[:, 0, 2].astype(np.int64)
res["prologue"] = pct(t[:, 0, 0] - start)
rs, re_ = st[:, 0, 6].astype(np.int64), st[:, 0, 7].astype(np.int64)
ok = re_ > 0
t0 = rs.min()
res["rt_kernel_us"] = float((re_[ok].max() - t0) / 100.0)
res["rt_end_us_pct"] = {p: float(np.percentile(re_[ok] - t0, p) / 100.0) for p in (10, 50, 90, 100)}
print(json.dumps(res))
