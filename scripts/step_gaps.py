#!/usr/bin/env python3
"""Kernel durations and inter-kernel gaps of the bench's forward steps, from a rocprofv3 kernel
trace of `bench.py --epoch-steps 0 --loop-epochs 0` (every dispatch of the process).

The steps are found as runs of the layer's launch pattern (means, GEMM, combine per layer); the
timed region is the --steps steps right before bench.py's per-kernel HIP-event pass (whose steps
show a gap of several us before every kernel). Prints per-role
average duration, the average gap before each role, and the step time as the trace sees it
(first start to last end over the block / steps).
usage: python scripts/step_gaps.py <run_kernel_trace.csv> [--steps 20] [--json out.json]"""
import argparse
import csv
import json
import statistics as st

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--layers", type=int, default=3)
ap.add_argument("--json", default=None)
ap.add_argument("--event-gap-us", type=float, default=4.0, help="median kernel gap of an event-pass step")
ap.add_argument("--idle-us", type=float, default=40.0, help="GPU idle time that ends a run of steps")
a = ap.parse_args()

rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))


def role(name):
    if "rel_gemm" in name or "layer_" in name:
        return "gemm"
    if "flat_rows_kernel" in name:
        return "flat"
    return "other:" + name.split("(")[0][:60]


seq = [(role(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
# the forward step: per layer [flat (means), gemm, flat (combine)]
pat = ["flat", "gemm", "flat"] * a.layers
n = len(pat)
blocks = []  # start indices of steps
i = 0
while i + n <= len(seq):
    if [s[0] for s in seq[i:i + n]] == pat:
        blocks.append(i)
        i += n
    else:
        i += 1
# runs of consecutive steps, cut where the GPU idled > --idle-us between two steps (a host sync:
# bench.py syncs after its pre-warm batches of 10, after the warm-up and after the timed region)
runs, cur, after = [], ([blocks[0]] if blocks else []), []
for b in blocks[1:]:
    idle = (seq[b][1] - seq[cur[-1] + n - 1][2]) / 1e3
    if b == cur[-1] + n and idle < a.idle_us:
        cur.append(b)
    else:
        runs.append(cur)
        after.append(idle)
        cur = [b]
if cur:
    runs.append(cur)
    after.append(None)
# bench.py: plan + first step, pre-warm (batches of 10 with a host sync between them), warm-up,
# the timed region, then the per-kernel event pass (--steps steps with a HIP event pair around
# every kernel: each kernel then waits ~8 us behind its events). The timed region is the --steps
# steps right before the first event-pass step (median gap between its kernels > --event-gap-us).
def med_gap(b):
    return st.median((seq[b + k][1] - seq[b + k - 1][2]) / 1e3 for k in range(1, n))


ev = next((j for j, b in enumerate(blocks) if j >= a.steps and med_gap(b) > a.event_gap_us), None)
if ev is None:
    raise SystemExit("no per-kernel event pass found in the trace")
timed = blocks[ev - a.steps:ev]
if any(timed[j + 1] != timed[j] + n for j in range(len(timed) - 1)):
    raise SystemExit("the steps before the event pass are not back to back")
names = ["means L%d" % (k // 3) if k % 3 == 0 else ("gemm L%d" % (k // 3) if k % 3 == 1 else "combine L%d" % (k // 3))
         for k in range(n)]
dur = {k: [] for k in range(n)}
gap = {k: [] for k in range(n)}
for b in timed:
    for k in range(n):
        r, s, e, _ = seq[b + k]
        dur[k].append((e - s) / 1e3)
        if b + k > 0:
            gap[k].append((s - seq[b + k - 1][2]) / 1e3)
t0 = seq[timed[0]][1]
t1 = seq[timed[-1] + n - 1][2]
out = {"steps": len(timed), "trace_step_us": (t1 - t0) / 1e3 / len(timed),
       "kernel_sum_us": sum(st.mean(dur[k]) for k in range(n)),
       "gap_sum_us": sum(st.mean(gap[k]) for k in range(n)),
       "per_launch": [{"launch": names[k], "kernel": seq[timed[0] + k][3][:80],
                       "avg_us": round(st.mean(dur[k]), 2), "min_us": round(min(dur[k]), 2),
                       "max_us": round(max(dur[k]), 2), "gap_before_avg_us": round(st.mean(gap[k]), 2),
                       "gap_before_max_us": round(max(gap[k]), 2)} for k in range(n)]}
for p in out["per_launch"]:
    print(f"{p['launch']:12s} {p['avg_us']:7.2f} us (min {p['min_us']:6.2f} max {p['max_us']:6.2f})  gap before "
          f"{p['gap_before_avg_us']:5.2f} (max {p['gap_before_max_us']:5.2f})")
print(f"step {out['trace_step_us']:.1f} us = kernels {out['kernel_sum_us']:.1f} + gaps {out['gap_sum_us']:.1f}")
if a.json:
    json.dump(out, open(a.json, "w"), indent=1)
