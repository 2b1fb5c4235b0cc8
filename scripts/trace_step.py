#!/usr/bin/env python3
"""Print the kernel sequence (duration, gap, grid) of a window of a rocprofv3 kernel trace."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
start = int(sys.argv[2]) if len(sys.argv) > 2 else 200
count = int(sys.argv[3]) if len(sys.argv) > 3 else 16
r = sorted(csv.DictReader(open(path)), key=lambda x: int(x["Start_Timestamp"]))
prev = None
for x in r[start:start + count]:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    prev = e
    print(f"{x['Kernel_Name'][:58]:58s} {(e - s) / 1e3:8.2f} us  gap {gap:6.2f}  grid {x['Grid_Size_X']:>8} "
          f"vgpr {x['VGPR_Count']:>3} lds {x['LDS_Block_Size']}")
