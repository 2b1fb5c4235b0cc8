#!/usr/bin/env python3
"""Summarise FETCH_SIZE / WRITE_SIZE passes (rocprofv3 --pmc, kernel-trace only) into
profiles/pmc_seg_fwd.json: HBM bytes per launch of the forward transform kernel (the bench's
roofline kernel), corrected as MI355X_MICROARCH.md §HBM prescribes for gfx950 (FETCH_SIZE reports
half of the read bytes: doubled; WRITE_SIZE exact).
Usage: pmc_traffic.py <fetch_dir> <write_dir> <out.json> [kernel name prefix]"""
import csv
import glob
import json
import os
import sys

KERNEL = sys.argv[4] if len(sys.argv) > 4 else "mpgnn::rel_gemm_kernel<2, false>"


def avg(root, counter):
    vals = {}
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "").split("(")[0].replace("void ", "")
            if name.startswith(KERNEL) and r["Counter_Name"] == counter:
                vals.setdefault(r.get("Dispatch_Id", len(vals)), 0.0)
                vals[r.get("Dispatch_Id", len(vals))] += float(r["Counter_Value"])
    return sum(vals.values()) / len(vals), len(vals)


fetch_kb, n1 = avg(sys.argv[1], "FETCH_SIZE")
write_kb, n2 = avg(sys.argv[2], "WRITE_SIZE")
out = {
    "workload": "fb15k237", "feat": 128, "kernel": KERNEL,
    "command": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes, kernel-trace only) -- "
               "python3 scripts/prof_layer.py --iters 20 (one RGCN layer forward, mode ALL)",
    "dispatches": [n1, n2],
    "fetch_size_kb_per_launch": round(fetch_kb, 1), "write_size_kb_per_launch": round(write_kb, 1),
    "hbm_bytes_per_launch": int((2 * fetch_kb + write_kb) * 1024),
    "correction": "gfx950: FETCH_SIZE x2 (reports half of wide coalesced read bytes), WRITE_SIZE as is",
}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out))
