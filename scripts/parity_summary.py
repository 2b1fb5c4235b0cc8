#!/usr/bin/env python3
"""Summary of a parity report (tests/_parity_report.py rows, MPGNN_PARITY_REPORT): how many checks
pass on the elementwise bar against the fp32 reference, how many on the float64-truth fallback,
the largest normwise error, and every check within 1/1.5 of its bar with the pytest node id
that made it. usage: python scripts/parity_summary.py profiles/r06_parity_report.jsonl [--json out]"""
import json
import sys

rows = [json.loads(line) for line in open(sys.argv[1]) if line.strip()]
fallback = [r for r in rows if r.get("decided_by", "").startswith("float64")]
near = sorted([r for r in rows if r.get("bar_ratio") is not None and r["bar_ratio"] >= 1 / 1.5],
              key=lambda r: -r["bar_ratio"])
out = {"checks": len(rows), "decided_on_float64_truth": len(fallback),
       "max_normwise": max((r.get("normwise", 0.0) for r in rows), default=0.0),
       "max_bar_ratio": max((r.get("bar_ratio") or 0.0 for r in rows), default=0.0),
       "within_1.5x_of_bar": [{"test": r.get("test"), "check": r["check"], "bar_ratio": round(r["bar_ratio"], 3),
                               "decided_by": r.get("decided_by")} for r in near]}
if "--json" in sys.argv:
    json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
print(json.dumps(out, indent=1))
