#!/usr/bin/env python3
"""Average each PMC counter per kernel over the dispatches of all passes under a directory."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        name = row.get("Kernel_Name", "")
        short = name.split("(")[0].replace("void ", "")[:60]
        acc[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
out = {}
for k, d in acc.items():
    if not k.startswith("mpgnn::"):
        continue
    out[k] = {c: sum(v) / len(v) for c, v in d.items()}
print(json.dumps(out, indent=1))
