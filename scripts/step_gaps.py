"""Busy vs idle time of the GPU over one graph-replayed training step in a rocprofv3 kernel trace.

Finds the densest window of consecutive dispatches that contains one step (the longest run
whose inter-kernel gaps are all < 50 us), then reports the kernel-busy time (union of
intervals), the idle gaps, and their distribution."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:50]) for r in rows)
# split into bursts at gaps > 50 us
bursts, cur = [], [iv[0]]
for a in iv[1:]:
    if a[0] - max(x[1] for x in cur[-4:]) > 50_000:
        bursts.append(cur)
        cur = []
    cur.append(a)
bursts.append(cur)
bursts.sort(key=lambda b: -len(b))
for b in bursts[:3]:
    t0, t1 = b[0][0], max(x[1] for x in b)
    busy, end, gaps = 0, b[0][0], []
    for s, e, _ in b:
        if s > end:
            gaps.append(s - end)
        busy += max(0, e - max(s, end))
        end = max(end, e)
    gaps.sort()
    print(f"burst: {len(b)} kernels, span {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, "
          f"idle {sum(gaps) / 1e3:.1f} us in {len(gaps)} gaps (median {gaps[len(gaps) // 2] / 1e3 if gaps else 0:.2f} us,"
          f" p90 {gaps[int(len(gaps) * .9)] / 1e3 if gaps else 0:.2f} us)")
