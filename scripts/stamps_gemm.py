"""Phase stamps of the forward transform (rel_gemm_kernel) on the C3 layer — debug build only
(make -C csrc stamps -> libmpgnn_rgcn_stamps.so, loaded through MPGNN_LIB_PATH).
Phases per wave and item: 0 item start (after the barrier) | 1 MFMA chain done (the pipelined
forward loop commits the next tile and stores the previous item inside the chain) | 3 weight
swap done | 4 barrier passed. Prints per-phase cycle percentiles
and the co-resident workgroups' phase offset."""
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
with torch.no_grad():
    for _ in range(3):
        conv(x, ei, et)
torch.cuda.synchronize()
nwaves = 256 * 4 * 4
buf = torch.zeros(nwaves * (ITEMS + 1) * PH, dtype=torch.int64, device=dev)
fn = _lib.lib.mpgnn_debug_stamps_set
fn.argtypes = [ctypes.c_void_p]
assert fn(buf.data_ptr()) == 0
with torch.no_grad():
    conv(x, ei, et)
torch.cuda.synchronize()
assert fn(None) == 0
st = buf.view(nwaves, ITEMS + 1, PH).cpu().numpy()
used = st[:, 0, 2] != 0
st = st[used]
ids = st[:, 0, :2]
t = st[:, 1:, :5].astype(np.int64)
valid = t[:, :, 0] != 0
res = {}
names = ["chain", "commit", "stores", "barrier"]
for k, nm in enumerate(names):
    d = (t[:, :, k + 1] - t[:, :, k])[valid & (t[:, :, k + 1] != 0) & (t[:, :, k] != 0)]
    if d.size:
        res[nm] = {p: int(np.percentile(d, p)) for p in (10, 50, 90)}
d = (t[:, :, 3] - t[:, :, 1])[valid & (t[:, :, 3] != 0) & (t[:, :, 1] != 0)]
res["after_chain"] = {p: int(np.percentile(d, p)) for p in (10, 50, 90)} if d.size else None
tot = (t[:, 1:, 0] - t[:, :-1, 0])[valid[:, 1:]]
res["item_total"] = {p: int(np.percentile(tot, p)) for p in (10, 50, 90)}
start = st[:, 0, 2]
end = np.where(valid, t[:, :, 4], 0).max(axis=1)
first = t[:, 0, 0]
res["prologue"] = {p: int(np.percentile(first - start, p)) for p in (10, 50, 90)}
res["wave_span"] = {p: int(np.percentile(end - start, p)) for p in (10, 50, 90)}
res["kernel_span_cycles"] = int(end.max() - start.min())
res["items_per_wave"] = {p: int(np.percentile(valid.sum(1), p)) for p in (10, 50, 90)}
# co-resident workgroups: waves with the same (XCC, HW_ID minus wave slot bits) = same SIMD
simd_key = ids[:, 1] * (1 << 20) + (ids[:, 0] >> 4)  # drop wave_id[3:0]
offs = []
order = np.argsort(simd_key, kind="stable")
for a, b in zip(order[:-1], order[1:]):
    if simd_key[a] == simd_key[b]:
        n = min(valid[a].sum(), valid[b].sum())
        if n > 2:
            offs.append(np.median(np.abs(t[a, :n, 1] - t[b, :n, 1])))
res["pair_chain_end_offset_median"] = {p: int(np.percentile(offs, p)) for p in (10, 50, 90)} if offs else None
print(json.dumps(res))
