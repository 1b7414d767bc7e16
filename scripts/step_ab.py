"""Interleaved A/B of whole training steps: bench.py --step-only under each variant's environment,
round-robin for several rounds on one box (box-to-box spread is ~1 %, so steps are compared only
within one call).  Usage: python scripts/step_ab.py ROUNDS NAME=ENV[;ENV...] ...
e.g.  python scripts/step_ab.py 3 base=X2G_LIB=x2-gnn_amd/lib/ab/libx2g_base.so new="""
import json
import os
import subprocess
import sys

rounds = int(sys.argv[1])
variants = []
for spec in sys.argv[2:]:
    name, _, envs = spec.partition("=")
    env = {}
    for kv in filter(None, envs.split(";")):
        k, _, v = kv.partition("=")
        env[k] = os.path.expandvars(v)
    variants.append((name, env))
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
res = {name: [] for name, _ in variants}
for r in range(rounds):
    for name, env in variants:
        e = dict(os.environ, **env)
        # AB_ROOT: run that tree's bench.py (and so its x2gnn package), e.g. ab_base/ from
        # scripts/build_base_tree.sh for a host-side change
        broot = os.path.join(root, env["AB_ROOT"]) if "AB_ROOT" in env else root
        # AB_ARGS: extra bench.py arguments for every variant (e.g. "--workload aid_infer --steps 30")
        # (a variant's own BENCH_ARGS entry adds arguments for that variant alone)
        extra = os.environ.get("AB_ARGS", "").split() + env.get("BENCH_ARGS", "").split()
        out = subprocess.run([sys.executable, os.path.join(broot, "bench.py"), "--step-only", "--steps", "200",
                              "--warmup", "10", *extra], env=e, capture_output=True, text=True, timeout=300)
        line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
        if out.returncode != 0 or not line:
            print(name, "FAILED", out.returncode, out.stderr[-2000:], flush=True)
            sys.exit(1)
        d = json.loads(line[-1])
        res[name].append(d["value"])
        print(f"round {r} {name:>10s} {d['value']:10.1f} mol/s  {d['ms_per_step']:.4f} ms  loss {d['final_loss']}",
              flush=True)
for name, v in res.items():
    print(f"{name:>10s} median {sorted(v)[len(v) // 2]:10.1f}  all {v}")
