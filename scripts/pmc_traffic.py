#!/usr/bin/env python3
"""profiles/r02_pmc_traffic.json — the bench's roofline `traffic`: HBM bytes per launch of each
forward kernel (role-labelled) from a scripts/pmc_report.py report of the PMC passes
(FETCH_SIZE ×2 + WRITE_SIZE per MI355X_MICROARCH.md §HBM, separate kernel-trace-only passes).
usage: pmc_traffic.py <report.json> <workload> <mode> <feat> [out.json]"""
import json
import sys

rep = json.load(open(sys.argv[1]))
workload, mode, feat = sys.argv[2], sys.argv[3], int(sys.argv[4])
out_path = sys.argv[5] if len(sys.argv) > 5 else "profiles/r02_pmc_traffic.json"
try:
    rows = json.load(open(out_path))
except (OSError, ValueError):
    rows = []
rows = [r for r in rows if not (r["workload"] == workload and r["mode"] == mode and r["feat"] == feat)]
for name, e in rep.items():
    if "hbm_MB_per_launch" not in e:
        continue
    rows.append({"workload": workload, "mode": mode, "feat": feat, "kernel": name,
                 "hbm_bytes_per_launch": int(e["hbm_MB_per_launch"] * 1e6), "profiled_us": e.get("profiled_us"),
                 "l2_hit": e.get("l2_hit"), "mfma_util": e.get("mfma_util"),
                 "source": f"scripts/pmc.sh + scripts/pmc_report.py ({sys.argv[1]})"})
json.dump(rows, open(out_path, "w"), indent=1)
print(json.dumps(rows, indent=1))
