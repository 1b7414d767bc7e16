"""Median duration of each run of consecutive same-name dispatches in a rocprofv3 kernel trace."""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pat = sys.argv[2] if len(sys.argv) > 2 else ""
groups = {}
order = []
for r in rows:
    n = r["Kernel_Name"]
    if pat not in n:
        continue
    key = (n[:60], r["Grid_Size_X"])
    if key not in groups:
        groups[key] = []
        order.append(key)
    groups[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k in order:
    d = groups[k]
    print(f"{k[0]:60s} grid {k[1]:>8s} n={len(d):4d} median {statistics.median(d):8.1f}us")
