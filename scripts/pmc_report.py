#!/usr/bin/env python3
"""Per-kernel report from the PMC passes of scripts/pmc.sh (rocprofv3 --pmc, kernel-trace only):
HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, the gfx950 correction of MI355X_MICROARCH.md),
HBM GB/s over the profiled launch duration, L2 hit rate, MFMA utilisation
(SQ_VALU_MFMA_BUSY_CYCLES, summed over the 1024 SIMDs, / (1024 x GRBM_GUI_ACTIVE / 8 XCDs)).
flat_rows_kernel serves several roles; launches are labelled by their order in the layer
(forward: means, combine; backward adds grad_x).

  python scripts/pmc_report.py gpurun_out/pmc [fwd|bwd] > profiles/…json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
mode = sys.argv[2] if len(sys.argv) > 2 else "fwd"


def short(name):
    # "(anonymous namespace)::" would end the name at its "(": plan_device.hip's once-per-graph
    # plan-build kernels (k_fill_edges, k_flat_walk, ...) then all read "mpgnn::" (r05 reports)
    return name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").strip()


def role_labels(rows):
    """Label the mpgnn dispatches of one pass by their position inside a layer call."""
    rows = sorted(rows, key=lambda r: int(r["Dispatch_Id"]))
    labels = {}
    k = 0
    for r in rows:
        n = short(r["Kernel_Name"])
        if not n.startswith("mpgnn::"):
            continue
        if n.startswith("mpgnn::flat_rows_kernel"):
            if mode == "fwd":
                role = ("means", "combine")[k % 2]
            else:  # forward (means, combine) then backward (grad_x)
                role = ("means", "combine", "grad_x")[k % 3]
            k += 1
            n = f"{n} [{role}]"
        labels[r["Dispatch_Id"]] = n
    return labels


acc = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    rows = list(csv.DictReader(open(f)))
    first = {}
    for r in rows:  # one row per (dispatch, counter)
        first.setdefault(r["Dispatch_Id"], r)
    labels = role_labels(list(first.values()))
    for r in rows:
        n = labels.get(r["Dispatch_Id"])
        if n is None:
            continue
        acc[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for d, r in first.items():
        if d in labels:
            dur[labels[d]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
out = {}
for n, cs in acc.items():
    c = {k: sum(v) / len(v) for k, v in cs.items()}
    e = {"profiled_us": round(sum(dur[n]) / len(dur[n]), 2)}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        b = c["FETCH_SIZE"] * 2 * 1024 + c["WRITE_SIZE"] * 1024
        e["hbm_MB_per_launch"] = round(b / 1e6, 2)
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c and c["TCC_HIT_sum"] + c["TCC_MISS_sum"] > 0:
        e["l2_hit"] = round(c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 3)
    if c.get("GRBM_GUI_ACTIVE", 0) > 0 and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
        e["mfma_util"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * c["GRBM_GUI_ACTIVE"] / 8), 3)
    if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"] > 0:
        e["wait_frac"] = round(c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"], 3)
    e["counters"] = {k: round(v, 1) for k, v in c.items()}
    out[n] = e
print(json.dumps(out, indent=1))
