"""Per-step kernel breakdown from a rocprofv3 kernel trace of bench.py: one step = the dispatches
between two consecutive `adam_ema` launches (the last kernel of a training step).  Prints the
median over the timed steps of each kernel's per-step time and launch count, plus busy/span."""
import csv
import statistics
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
marks = [i for i, a in enumerate(iv) if "adam_ema" in a[2]]
steps = [iv[a + 1:b + 1] for a, b in zip(marks[:-1], marks[1:])]
steps = steps[-8:]
per = defaultdict(list)
cnt = defaultdict(list)
busy, span = [], []
for st in steps:
    d = defaultdict(float)
    c = defaultdict(int)
    for s, e, n in st:
        k = n.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:72]
        d[k] += (e - s) / 1e3
        c[k] += 1
    for k in d:
        per[k].append(d[k])
        cnt[k].append(c[k])
    busy.append(sum((e - s) for s, e, _ in st) / 1e3)
    span.append((st[-1][1] - st[0][0]) / 1e3)
tot = 0
for k, v in sorted(per.items(), key=lambda kv: -statistics.median(kv[1])):
    m = statistics.median(v)
    tot += m
    print(f"{m:9.1f} us {statistics.median(cnt[k]):6.0f} x  {k}")
print(f"# steps {len(steps)}: kernel time {statistics.median(busy):.1f} us, span {statistics.median(span):.1f} us, "
      f"launches {statistics.median([len(s) for s in steps])}")
