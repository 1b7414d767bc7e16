"""CPU-baseline calibration (BASELINE.md "Plan for the CPU baseline", item 2) — build container only.

The reference's Python cannot travel to the GPU box, so bench.py times the oracle restatement
(``oracle/ref_cpu.py``) there.  This script times BOTH on the same host cores here — the
reference itself imported through the fixture harness (tests/golden/ref_import.py, the shims of
SURVEY.md §8c) and the restatement — on the same batch (bench.py's config-2 batch: 128 S160
molecules, seed 1000), the same seeded weights, fwd + smooth_l1 + bwd, median of 5 steps after
1 warm-up, at 8 threads (this container's cores) and 4 (config.json ``num_thread``), and writes
the reference / restatement rate ratio per thread count:

    python scripts/calibrate_cpu_baseline.py [out.json] [seed ...]
        (default profiles/r4_cpu_calibration.json; seeds default: 1000 = bench.py's batch, 0 = the survey's)

Round 4: the batch seed is a parameter and both the survey's seed-0 batch (BASELINE.md:25, 106.9 mol/s
at 8 threads) and bench.py's seed-1000 batch are timed, so the two figures can be compared on one host.

bench.py multiplies the restatement's rate on the GPU box's host by this ratio to state a
reference-equivalent CPU figure beside its own measurement.
"""
from __future__ import annotations

import json
import os
import platform
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "x2-gnn_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)

from ref_import import import_reference  # noqa: E402
from weights import load_seeded  # noqa: E402

from oracle import ref_cpu  # noqa: E402
from x2gnn.data import collate  # noqa: E402
from x2gnn.synth import synthetic_molecules  # noqa: E402

CFG = dict(conv_layers=4, sbf_dim=7, rbf_dim=6, in_channels=128, heads=16, embedding_size=128)
SEED_W = 900


def time_steps(step, reps=5):
    step()  # warm-up
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        step()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), [round(t, 4) for t in ts]


def calibrate(ref, seed):
    mols = synthetic_molecules(128, "S160", seed=seed)  # seed 1000: bench.py's config-2 batch at N = 1
    b = collate(mols)
    ref_model = ref.xgnn.xgnn_poly(device="cpu", **CFG)
    port_model = ref_cpu.XGNN(**CFG)
    load_seeded(ref_model, SEED_W)
    load_seeded(port_model, SEED_W)

    def ref_step():
        ref_model.zero_grad(set_to_none=True)
        res = ref_model(b)
        torch.nn.functional.smooth_l1_loss(res, b.y).backward()
        return res

    def port_step():
        port_model.zero_grad(set_to_none=True)
        res = ref_cpu.run_batch(port_model, b)
        torch.nn.functional.smooth_l1_loss(res, b.y).backward()
        return res

    with torch.no_grad():
        e_ref = ref_model(b)
        e_port = ref_cpu.run_batch(port_model, b)
    rel = float((e_ref - e_port).abs().max() / e_ref.abs().max())
    rows = {}
    for threads in (8, 4):
        torch.set_num_threads(threads)
        t_ref, ts_ref = time_steps(ref_step)
        t_port, ts_port = time_steps(port_step)
        rows[str(threads)] = {"reference_mol_s": round(len(mols) / t_ref, 2), "port_mol_s": round(len(mols) / t_port, 2),
                              "reference_over_port": round(t_port / t_ref, 4), "reference_step_s": ts_ref,
                              "port_step_s": ts_port}
        print(seed, threads, rows[str(threads)], flush=True)
    meta = b.host_meta()
    return {"batch": f"128 synthetic S160 molecules, seed {seed}",
            "per_molecule": {"atoms": float(meta["nodes"].mean()), "edges": float(meta["edges"].mean()),
                             "triplets": float(meta["triplets"].mean())},
            "energies_max_rel_diff": rel, "threads": rows}


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r4_cpu_calibration.json")
    seeds = [int(x) for x in sys.argv[2:]] or [1000, 0]
    ref = import_reference()
    per_seed = {str(s): calibrate(ref, s) for s in seeds}
    first = per_seed[str(seeds[0])]
    res = {"what": "reference (shimmed import) vs oracle/ref_cpu.py restatement, fwd+smooth_l1+bwd, same batch / "
                   "weights / cores; median of 5 after 1 warm-up",
           "host": {"cpus": os.cpu_count(), "machine": platform.processor() or platform.machine(),
                    "torch": torch.__version__},
           # bench.py reads these two (its batch: seed 1000)
           "batch": first["batch"], "energies_max_rel_diff": first["energies_max_rel_diff"],
           "threads": first["threads"], "seeds": per_seed}
    json.dump(res, open(out_path, "w"), indent=1)
    print("->", out_path)


if __name__ == "__main__":
    main()
