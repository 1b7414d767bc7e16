"""The training step's per-kernel work table (GPU box): HBM bytes per step from two rocprofv3 PMC passes
(FETCH_SIZE, WRITE_SIZE) over eager steps of `bench.py --step-only --eager`, the matrix FLOPs per step
of every MFMA kernel from the config-2 shapes, and the kernel time per step from a kernel trace.
bench.py reads the table to state `step_roofline`: the sum over kernels of max(FLOP / f32 MFMA peak,
HBM bytes / HBM peak) — each kernel at its own roofline, run back to back — divided by the measured
step time.

    python scripts/step_work.py PMC_FETCH_DIR PMC_WRITE_DIR TRACE_DIR OUT.json

FETCH_SIZE is doubled (gfx950 counts 128-B reads at 64 B; MI355X_MICROARCH.md HBM section), both
counters are KiB.  Steps are counted by the optimizer's last kernel (adam_ema), one per step.
"""
import collections
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "x2-gnn_amd")]

D = 128


def short(name):
    m = re.search(r"x2g::(?:\(anonymous namespace\)::)?(\w+)", name)
    return m.group(1) if m else name.split("(")[0][:48]


def find_csv(d, suffix):
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith(suffix):
                return os.path.join(root, f)
    raise FileNotFoundError(f"{suffix} under {d}")


def per_kernel_counter(d):
    tot = collections.defaultdict(float)
    for r in csv.DictReader(open(find_csv(d, "counter_collection.csv"))):
        tot[short(r["Kernel_Name"])] += float(r["Counter_Value"])
    return tot


def trace(d, last=8):
    """(us per step, launches per step) per kernel over the last `last` steps of a kernel trace (a step =
    the dispatches after one adam_ema up to and including the next), and the step count used."""
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                for r in csv.DictReader(open(find_csv(d, "kernel_trace.csv"))))
    marks = [i for i, a in enumerate(iv) if a[2] == "adam_ema"]
    steps = [iv[a + 1:b + 1] for a, b in zip(marks[:-1], marks[1:])][-last:]
    tot, cnt = collections.defaultdict(float), collections.defaultdict(int)
    for stp in steps:
        for s0, s1, k in stp:
            tot[k] += (s1 - s0) / 1e3
            cnt[k] += 1
    n = max(1, len(steps))
    return {k: v / n for k, v in tot.items()}, {k: v / n for k, v in cnt.items()}, n


def flops_per_step(E, T, N, flat_launches):
    """Matrix FLOPs (2 per multiply-add) per training step of each MFMA kernel at this batch's shape."""
    L = 4
    flat = sum(2 * R * D * c for launch in flat_launches for R, c in launch)  # [(rows, cols) per job] per launch
    return {
        "chain_fwd_v4_ln": L * 7 * 2 * E * D * D,           # trunk tail: 7 D x D stages per layer
        "chain_fwd_v4_batch": 5 * 2 * 2 * N * D * D,        # 5 readout MLPs x 2 hidden layers on the atom rows
        "chain_bwd_v3_batch": L * 7 * 2 * E * D * D + 5 * 2 * 2 * N * D * D,  # their data gradients
        "conv_proj_fwd_kernel": L * (4 * 2 * E * D * D + 2 * E * D * 6),      # q, k, v, skip + the rbf gate
        "conv_proj_bwd_gate_kernel": L * (4 * 2 * E * D * D + 2 * 2 * E * D * 6),
        "feat_fwd_kernel": 2 * E * (338 * 256 + 256 * 128),
        "feat_bwd_kernel": 2 * E * 256 * 128,
        "sbf_project_waves": L * 2 * T * 42 * D,
        "tiled_flat_kernel": flat,                          # every T-layout weight gradient of the backward
    }


def main():
    fetch_d, write_d, trace_d, out = sys.argv[1:5]
    import torch

    import x2gnn
    from x2gnn.data import collate
    from x2gnn.synth import synthetic_molecules
    from x2gnn.train import Trainer

    fetch, write = per_kernel_counter(fetch_d), per_kernel_counter(write_d)
    t_us, t_cnt, st = trace(trace_d)
    # steps in each pass: adam_ema dispatches (one per step)
    def steps_in(d):
        n = sum(1 for r in csv.DictReader(open(find_csv(d, "counter_collection.csv"))) if "adam_ema" in r["Kernel_Name"])
        return max(1, n)
    sf, sw = steps_in(fetch_d), steps_in(write_d)
    cfg = dict(conv_layers=4, sbf_dim=7, rbf_dim=6, in_channels=128, heads=16, embedding_size=128)
    batch = collate(synthetic_molecules(128, "S160", seed=1000))
    meta = batch.host_meta()
    E, T, N = int(meta["edges"].sum()), int(meta["triplets"].sum()), int(meta["nodes"].sum())
    torch.manual_seed(0)
    tr = Trainer(x2gnn.xgnn_poly(device="cuda", **cfg).cuda())
    tr.forward_backward(batch.to("cuda"))
    torch.cuda.synchronize()
    fl = flops_per_step(E, T, N, tr.flat_launches)
    kernels = {}
    for k in sorted(set(fetch) | set(write) | set(t_us)):
        b = 2 * 1024 * fetch.get(k, 0.0) / sf + 1024 * write.get(k, 0.0) / sw
        kernels[k] = {"hbm_bytes": int(b), "flops": int(fl.get(k, 0)), "us": round(t_us.get(k, 0.0), 2),
                      "launches": round(t_cnt.get(k, 0), 2)}
    from bench import product_digest

    json.dump({"meta": {"commit": os.environ.get("X2G_COMMIT"),  # the tree measured (.git does not travel to the box)
                        "digest": product_digest(),  # bench.py states step_roofline only on these sources
                        "shape": {"E": E, "T": T, "N": N, "B": 128}, "steps": {"fetch": sf, "write": sw, "trace": st},
                        "sources": [fetch_d, write_d, trace_d],
                        "note": "HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB) per step; flops = matrix FLOPs per "
                                "step of the MFMA kernels (scripts/step_work.py flops_per_step); us = kernel time "
                                "per step in a kernel trace of graph-replayed steps (median-free mean of the last 8)"},
               "kernels": kernels}, open(out, "w"), indent=1)
    print(f"{len(kernels)} kernels -> {out}")


if __name__ == "__main__":
    main()
