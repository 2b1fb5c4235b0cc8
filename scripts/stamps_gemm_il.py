"""Phase stamps of the bf16-split forward GEMMs (RelGemmBf3::run_il at F = 128, rel_gemm_bf3w_kernel
at F = 256: --workload C5) on one layer —
debug build only (make -C csrc stamps -> libmpgnn_rgcn_stamps.so, loaded via MPGNN_LIB_PATH).
Per wave and item: 0 item start | 1 k-loop done | 2 weight switch (stamped only then) | 3 epilogue
done | 4 barrier passed. Prints phase percentiles, the per-wave span against items and weight
switches, and the spread of wave end times per XCD (cycles of s_memtime: the shader clock)."""
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
import argparse  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="fb15k237")
ap.add_argument("--single", type=int, default=None, help="mode SINGLE over this relation")
ap.add_argument("--opt", action="append", default=[], help="K=V process default before the plan is built "
                "(35=1: rel_gemm_w1_kernel)")
cli = ap.parse_args()
for kv in cli.opt:
    _lib.set_option(int(kv.split("=")[0]), int(kv.split("=")[1]))

ITEMS, PH = 32, 8
g = data.fb15k237_graph(feat_dim=128) if cli.workload == "fb15k237" else data.config_graph(cli.workload)
dev = torch.device("cuda", 0)
torch.manual_seed(10)
F = g.x.shape[1]
if cli.single is None:
    conv = mpgnn_amd.RGCNConv(F, F, g.num_relations, flow="target_to_source").to(dev)
else:
    conv = mpgnn_amd.CustomRGCNConv(F, F, g.num_relations, flow="target_to_source").to(dev)
x, ei, et = g.x.to(dev), g.edge_index.to(dev), g.edge_type.to(dev)


def fwd():
    if cli.single is None:
        return conv(x, ei, et)
    return conv(0, cli.single, x, ei, et)


with torch.no_grad():
    for _ in range(3):
        fwd()
torch.cuda.synchronize()
nwaves = 256 * 4 * 4
buf = torch.zeros(nwaves * (ITEMS + 1) * PH, dtype=torch.int64, device=dev)
fn = _lib.lib.mpgnn_debug_stamps_set
fn.argtypes = [ctypes.c_void_p]
assert fn(buf.data_ptr()) == 0
with torch.no_grad():
    fwd()
torch.cuda.synchronize()
assert fn(None) == 0
st = buf.view(nwaves, ITEMS + 1, PH).cpu().numpy()
used = st[:, 0, 2] != 0
wid = np.nonzero(used)[0]
st = st[used]
xcc = st[:, 0, 1]
t = st[:, 1:, :5].astype(np.int64)
valid = t[:, :, 0] != 0
pct = lambda d: {p: int(np.percentile(d, p)) for p in (10, 50, 90, 99)} if np.size(d) else None  # noqa: E731
res = {}
both = valid & (t[:, :, 1] != 0)
res["chain"] = pct((t[:, :, 1] - t[:, :, 0])[both])
sw = valid & (t[:, :, 2] != 0)
res["switch_items_frac"] = float(sw.sum() / valid.sum())
res["epilogue_no_switch"] = pct((t[:, :, 3] - t[:, :, 1])[valid & ~sw & (t[:, :, 3] != 0)])
res["epilogue_switch"] = pct((t[:, :, 3] - t[:, :, 1])[sw & (t[:, :, 3] != 0)])
res["barrier"] = pct((t[:, :, 4] - t[:, :, 3])[valid & (t[:, :, 4] != 0)])
start = st[:, 0, 2]
last = np.where(valid, t[:, :, 4], 0).max(axis=1)
res["prologue"] = pct(t[:, 0, 0] - start)
pro = st[:, 0, 3:6].astype(np.int64)
res["pro_rows0_issued"] = pct(pro[:, 0] - start)
res["pro_weights_split"] = pct(pro[:, 1] - pro[:, 0])
res["pro_commit"] = pct(pro[:, 2] - pro[:, 1])
res["pro_barrier"] = pct(t[:, 0, 0] - pro[:, 2])
span = last - start
res["wave_span"] = pct(span)
items = valid.sum(1)
res["items_per_wave"] = pct(items)
nsw = sw.sum(1)
res["switches_per_wave"] = pct(nsw)
# span model: span ~ a + b*items + c*switches (least squares)
A = np.stack([np.ones_like(items), items, nsw], 1).astype(np.float64)
coef, *_ = np.linalg.lstsq(A, span.astype(np.float64), rcond=None)
res["span_fit_const_item_switch"] = [round(float(c)) for c in coef]
# end-time spread per XCD (s_memtime is per XCD: compare within one)
spread = {}
for xc in np.unique(xcc):
    m = xcc == xc
    e = last[m]
    s0 = start[m]
    spread[int(xc)] = {"first_start_to_last_end": int(e.max() - s0.min()), "start_spread": int(s0.max() - s0.min()),
                       "end_p10": int(np.percentile(e - s0.min(), 10)), "end_p50": int(np.percentile(e - s0.min(), 50))}
res["per_xcc"] = spread
# realtime (100 MHz, device-global) start / end of every wave: the tail per XCD
rs, re_ = st[:, 0, 6].astype(np.int64), st[:, 0, 7].astype(np.int64)
t0 = rs.min()
res["rt_kernel_us"] = float((re_.max() - t0) / 100.0)
res["rt_start_spread_us"] = float((rs.max() - t0) / 100.0)
res["rt_end_us_pct"] = {p: float(np.percentile(re_ - t0, p) / 100.0) for p in (10, 50, 90, 99, 100)}
res["rt_end_us_by_xcc"] = {int(xc): [float(np.percentile(re_[xcc == xc] - t0, p) / 100.0) for p in (50, 90, 100)]
                           for xc in np.unique(xcc)}
res["clock_ghz_median"] = float(np.median(span / np.maximum(re_ - rs, 1) / 10.0))
# per CU (XCC, HW_ID without the wave / SIMD bits): both workgroups' items and switches against
# the CU's last end time
cu_key = xcc.astype(np.int64) * (1 << 24) + ((st[:, 0, 0].astype(np.int64) >> 8) & 0xFF)
cus = {}
for k in range(len(cu_key)):
    c = cus.setdefault(int(cu_key[k]), {"blocks": set(), "items": 0, "sw": 0, "end": 0})
    blk = int(wid[k]) // 4
    if blk not in c["blocks"]:
        c["blocks"].add(blk)
        c["items"] += int(items[k])
        c["sw"] += int(nsw[k])
    c["end"] = max(c["end"], int(re_[k] - t0))
ci = np.array([c["items"] for c in cus.values()])
cs = np.array([c["sw"] for c in cus.values()])
ce = np.array([c["end"] for c in cus.values()]) / 100.0
nb = np.array([len(c["blocks"]) for c in cus.values()])
res["cu_count"] = int(len(cus))
diffs = [abs(a - b) for c in cus.values() if len(c["blocks"]) == 2 for a, b in [sorted(c["blocks"])]]
res["cu_pair_block_diff_hist"] = {int(v): int(n) for v, n in zip(*np.unique(diffs, return_counts=True))} if diffs else None
res["cu_blocks_hist"] = {int(v): int((nb == v).sum()) for v in np.unique(nb)}
res["cu_items_pct"] = pct(ci)
res["cu_end_us_by_items"] = {int(v): [round(float(np.median(ce[ci == v])), 2), int((ci == v).sum())] for v in np.unique(ci)}
res["cu_end_us_by_switches"] = {int(v): [round(float(np.median(ce[cs == v])), 2), int((cs == v).sum())] for v in np.unique(cs)}
A = np.stack([np.ones_like(ci), ci, cs], 1).astype(np.float64)
coef, *_ = np.linalg.lstsq(A, ce, rcond=None)
res["cu_end_fit_us_const_item_switch"] = [round(float(c), 3) for c in coef]
# the slowest waves: items, switches, prologue
slow = np.argsort(span)[-8:]
res["slowest"] = [{"wave": int(wid[k]), "span": int(span[k]), "items": int(items[k]), "switches": int(nsw[k]),
                   "prologue": int(t[k, 0, 0] - start[k]), "xcc": int(xcc[k]),
                   "rt_end_us": float((re_[k] - t0) / 100.0)} for k in slow]
print(json.dumps(res))
