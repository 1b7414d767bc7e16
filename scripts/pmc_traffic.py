"""HBM traffic per dispatch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs).

    python scripts/pmc_traffic.py gpurun_out/pmc_fetch_TAG gpurun_out/pmc_write_TAG profiles/TAG_pmc_traffic.json

Both counters are in KiB.  gfx950 tallies 128-B read requests at 64 B, so FETCH_SIZE reports
half the bytes of wide (16 B/lane) streaming reads: it is doubled here (MI355X_MICROARCH.md,
HBM section).  WRITE_SIZE is exact for 16-B-per-lane stores and used as is.  The JSON maps
"<kernel name>|<grid size>" to the LARGEST bytes per dispatch: bench.py's probes time the step's
largest launch of each kernel (config 5: the whole-batch attention launch, while the step runs it in
triplet tiles of the same grid size), so the PMC figure paired with a probe time must be that launch's,
not the median over the tiles (round 3's config-5 line paired a tile's bytes with a whole-batch time).
"""
import collections
import csv
import json
import os
import sys


def per_dispatch(d):
    path = os.path.join(d, "run_counter_collection.csv")
    g = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        g[f"{r['Kernel_Name']}|{r['Grid_Size']}"].append(float(r["Counter_Value"]))
    return {k: (max(v), len(v)) for k, v in g.items()}


fetch, write = per_dispatch(sys.argv[1]), per_dispatch(sys.argv[2])
out = {}
for k in sorted(set(fetch) | set(write)):
    f = fetch.get(k, (None, 0))
    w = write.get(k, (None, 0))
    out[k] = {"fetch_bytes": None if f[0] is None else round(2 * 1024 * f[0]),
              "write_bytes": None if w[0] is None else round(1024 * w[0]),
              "dispatches": [f[1], w[1]]}
meta = {"commit": os.environ.get("X2G_COMMIT"), "source": [sys.argv[1], sys.argv[2]], "correction": "FETCH_SIZE x2 (gfx950), KiB -> bytes",
        "per_dispatch": "max over the key's dispatches (the probes' launches)"}
json.dump({"meta": meta, "kernels": out}, open(sys.argv[3], "w"), indent=1)
print(f"{len(out)} kernel/grid entries -> {sys.argv[3]}")
