"""Print the kernel sequence of one graph-replayed step from a rocprofv3 kernel trace (the
last burst of dispatches whose inter-kernel gaps stay < 50 us and that holds the most
kernels), with per-kernel durations, so every launch can be traced back to its source."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Grid_Size_X"]) for r in rows)
bursts, cur = [], [iv[0]]
for a in iv[1:]:
    if a[0] - cur[-1][1] > 50_000:
        bursts.append(cur)
        cur = []
    cur.append(a)
bursts.append(cur)
big = max(len(b) for b in bursts)
step = [b for b in bursts if len(b) >= 0.9 * big][-1]
for s, e, n, g in step:
    short = n.split("(")[0].replace("void ", "")[:70]
    print(f"{(e - s) / 1e3:8.1f}  {g:>9s}  {short}")
print(f"# {len(step)} kernels, {(step[-1][1] - step[0][0]) / 1e3:.1f} us")
