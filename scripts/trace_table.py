"""Per-step kernel table from a rocprofv3 kernel trace of bench.py --step-only (training or inference):
the largest burst of dispatches, per step = its totals / the launches of a once-per-step kernel
(edge_basis_kernel).  Usage: python scripts/trace_table.py run_kernel_trace.csv [rows]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
bursts, cur = [], [iv[0]]
for a in iv[1:]:
    if a[0] - cur[-1][1] > 200_000:
        bursts.append(cur)
        cur = []
    cur.append(a)
bursts.append(cur)
b = max(bursts, key=len)
nsteps = sum(1 for _, _, n in b if "edge_basis_kernel" in n)
d, c = collections.defaultdict(float), collections.Counter()
for s, e, n in b:
    k = n.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:64]
    d[k] += (e - s) / 1e3
    c[k] += 1
print(f"steps {nsteps}: kernel time per step {sum(d.values()) / nsteps:.1f} us, "
      f"span per step {(b[-1][1] - b[0][0]) / 1e3 / nsteps:.1f} us")
for k, v in sorted(d.items(), key=lambda kv: -kv[1])[:int(sys.argv[2]) if len(sys.argv) > 2 else 24]:
    print(f"{v / nsteps:9.1f} us {c[k] / nsteps:5.1f} x  {k}")
