"""Print the kernel sequence of one window of a rocprofv3 kernel trace (durations in us).
usage: python scripts/trace_seq.py <run_kernel_trace.csv> [anchor-substring] [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
anchor = sys.argv[2] if len(sys.argv) > 2 else "rel_gemm_kernel<2, false"
n = int(sys.argv[3]) if len(sys.argv) > 3 else 14
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
i0 = max(idx[len(idx) // 2] - 3, 0)
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i0 + n]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1000:9.1f} {(e - s) / 1000:8.1f}  {r['Kernel_Name'][:90]}")
