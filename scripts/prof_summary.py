"""Summarise a rocprofv3 kernel-stats CSV: top kernels, totals, per-step estimates."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(int(r["TotalDurationNs"]) for r in rows)
calls = sum(int(r["Calls"]) for r in rows)
print(f"total {tot / 1e6:.2f} ms in {calls} launches")
for r in sorted(rows, key=lambda r: -int(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    n = r["Name"]
    n = ("GEMM MT" + n.split("_MT")[1].split("_")[0] + " " + n[:16]) if n.startswith("Cijk") else n[:88]
    print(f"{n:90s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:8.1f}us {int(r['TotalDurationNs']) / 1e6:8.2f}ms"
          f" {int(r['TotalDurationNs']) / 1e6 / steps:7.3f}ms/step")
