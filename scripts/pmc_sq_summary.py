"""Per-kernel summary of the SQ counter passes of scripts/pmc_sq.sh.

    python scripts/pmc_sq_summary.py gpurun_out/pmc_sqa_TAG [gpurun_out/pmc_sqb_TAG ...]

For every kernel: the per-dispatch mean of each counter and the derived shares —
  parked  = SQ_WAIT_ANY / SQ_WAVE_CYCLES       (waiting on s_waitcnt / s_barrier)
  stalled = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES  (ready but not issued: MFMA dependency / pipe busy)
  issuing = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  mfma    = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs): the matrix pipes' busy
            share of the kernel's duration (GRBM_GUI_ACTIVE is summed over the 8 XCDs; the MFMA busy
            counter over every SIMD)
  clock   = GRBM_GUI_ACTIVE / 8 / duration, when the trace gives the duration
"""
import collections
import csv
import os
import re
import sys


def short(name):
    m = re.search(r"x2g::(?:\(anonymous namespace\)::)?(\w+)", name)
    return m.group(1) if m else name[:40]


def load(d):
    path = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(path):
        for root, _, files in os.walk(d):
            for f in files:
                if f.endswith("counter_collection.csv"):
                    path = os.path.join(root, f)
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
        if "End_Timestamp" in r and "Start_Timestamp" in r:
            dur[k].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    return {k: {c: v / max(1, len(disp[k])) for c, v in cs.items()} for k, cs in vals.items()}, disp


merged = collections.defaultdict(dict)
ndisp = {}
for d in sys.argv[1:]:
    v, disp = load(d)
    for k, cs in v.items():
        merged[k].update(cs)
        ndisp[k] = len(disp[k])

for k in sorted(merged, key=lambda k: -merged[k].get("GRBM_GUI_ACTIVE", 0)):
    c = merged[k]
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    line = [f"{k:32s} n={ndisp.get(k, 0):3d}"]
    if "SQ_WAVE_CYCLES" in c:
        line.append(f"parked {c.get('SQ_WAIT_ANY', 0) / wc:5.2f} stalled {c.get('SQ_WAIT_INST_ANY', 0) / wc:5.2f} "
                    f"issuing {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:5.2f} lds-stall {c.get('SQ_WAIT_INST_LDS', 0) / wc:5.2f}")
    g = c.get("GRBM_GUI_ACTIVE")
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
        line.append(f"mfma {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (g / 8 * 1024):5.2f} "
                    f"(cycles {g / 8:9.0f})")
    if "SQ_LDS_IDX_ACTIVE" in c and c["SQ_LDS_IDX_ACTIVE"]:
        line.append(f"lds-conflict {c.get('SQ_LDS_BANK_CONFLICT', 0) / c['SQ_LDS_IDX_ACTIVE']:5.3f}")
    if "SQ_INSTS_VALU" in c:
        line.append(f"valu {c['SQ_INSTS_VALU']:.3g} lds {c.get('SQ_INSTS_LDS', 0):.3g} "
                    f"vmem-wr {c.get('SQ_INSTS_VMEM_WR', 0):.3g} vmem-rd {c.get('SQ_INSTS_VMEM_RD', 0):.3g}")
    print("  ".join(line))
print()
for k in sorted(merged):
    print(k, {c: round(v) for c, v in sorted(merged[k].items())})
