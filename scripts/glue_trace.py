"""Which Python call site launches each small kernel of the training step?  One eager step of
bench.py's Trainer under torch.profiler (with stacks); prints every GPU kernel shorter than
LIMIT_US with the innermost x2gnn / bench frame that issued it, in launch order."""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "x2-gnn_amd"))
import bench  # noqa: E402
import x2gnn  # noqa: E402
from x2gnn.data import collate  # noqa: E402
from x2gnn.synth import synthetic_molecules  # noqa: E402

LIMIT_US = float(os.environ.get("LIMIT_US", "12"))
dev = torch.device("cuda")
torch.manual_seed(0)
model = x2gnn.xgnn_poly(device="cuda", **bench.CFG).to(dev)
batch = collate(synthetic_molecules(128, "S160", seed=1000)).to(dev)
tr = bench.Trainer(model)
for _ in range(2):
    tr.step(batch)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    tr.step(batch)
    torch.cuda.synchronize()

events = prof.events()


def site(stack):
    for fr in stack or []:
        if ("x2gnn" in fr or "bench.py" in fr) and "_lib.py" not in fr:
            return fr
    return (stack or ["?"])[0]


# every CPU-side op that launched kernels, innermost first so each kernel is attributed once
seen, rows = set(), []
cpu = [e for e in events if e.device_type == torch.autograd.DeviceType.CPU and e.kernels]
cpu.sort(key=lambda e: -e.time_range.start)  # children start after parents: innermost first
for e in sorted(cpu, key=lambda e: e.time_range.elapsed_us()):
    for k in e.kernels:
        key = (k.name, k.device, getattr(k, "time_range", None) and k.time_range.start)
        if key in seen:
            continue
        seen.add(key)
        st = e
        while st is not None and not st.stack:
            st = st.cpu_parent
        rows.append((getattr(k, "time_range", None).start if getattr(k, "time_range", None) else 0,
                     k.duration if hasattr(k, "duration") else 0, k.name, e.name, site(st.stack if st else None)))
rows.sort()
n = 0
for t, us, kname, op, src in rows:
    if us > LIMIT_US:
        continue
    n += 1
    print(f"{us:6.1f}  {kname[:50]:50s}  {op[:28]:28s}  {src}")
print(f"# {n} kernels under {LIMIT_US} us of {len(rows)}")
