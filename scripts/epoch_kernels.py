#!/usr/bin/env python3
"""Kernels of one training epoch from a rocprofv3 kernel trace of `bench.py` (its eager epoch
leg): the window between the last two optimizer launches (the graph replays' steady state; or,
--window middle, two in the middle of the run), per kernel name: launches, total and average µs, share of the epoch's kernel time, plus the
epoch's span and its idle time between kernels.
usage: python scripts/epoch_kernels.py <run_kernel_trace.csv> [--json out.json]"""
import argparse
import csv
import json
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--json", default=None)
ap.add_argument("--window", choices=["last", "middle"], default="last")
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
adam = [i for i, r in enumerate(rows) if "adam" in r["Kernel_Name"].lower()]
if len(adam) < 3:
    raise SystemExit("fewer than 3 Adam launches in the trace")
# the last complete window: bench.py's epoch leg ends with the HIP-graph replays (steady state,
# no host gaps, no one-time setup launches)
k = len(adam) - 1 if a.window == "last" else len(adam) // 2
lo, hi = adam[k - 1] + 1, adam[k] + 1  # kernels after one Adam up to and including the next
win = rows[lo:hi]
by = defaultdict(lambda: [0, 0.0])
busy = 0.0
for r in win:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:90]
    by[n][0] += 1
    by[n][1] += d
    busy += d
span = (int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"])) / 1e3
out = {"span_us": round(span, 1), "kernel_us": round(busy, 1), "idle_us": round(span - busy, 1),
       "launches": len(win),
       "kernels": sorted([{"kernel": n, "launches": c, "total_us": round(t, 2), "avg_us": round(t / c, 2),
                           "share": round(t / busy, 4)} for n, (c, t) in by.items()], key=lambda x: -x["total_us"])}
print(f"epoch span {span:.1f} us, kernels {busy:.1f} us, idle {span - busy:.1f} us, {len(win)} launches")
for x in out["kernels"]:
    print(f"{x['total_us']:9.2f} us {x['launches']:3d}x {x['avg_us']:8.2f}  {x['kernel']}")
if a.json:
    json.dump(out, open(a.json, "w"), indent=1)
