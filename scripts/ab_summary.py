#!/usr/bin/env python3
"""Summarise scripts/ab_libs.sh outputs: gpurun_out/ab_<tag>_<k>.json -> one line per run."""
import json
import sys

tags = sys.argv[1:] or ["base"]
for t in tags:
    for k in (1, 2):
        try:
            d = json.load(open(f"gpurun_out/ab_{t}_{k}.json"))
        except (OSError, ValueError) as e:
            print(t, k, e)
            continue
        kk = d.get("kernels_per_layer", {})
        print(t, k, round(d["value"] / 1e9, 3), d["ms_per_step"], d.get("epoch_ms"),
              {n: round(v["us_per_layer"], 2) for n, v in kk.items()})
