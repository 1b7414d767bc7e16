"""Phase timeline of the fused-projection center forward (x2g_sbf_attention_fwd_center_sf; A/B trace build
only: python scripts/make_ctrace_copy.py && make -C x2-gnn_amd ab AB_UNIT=attention_center AB_NAME=ctrace
AB_FLAGS=-DX2G_TRACE, run with X2G_LIB=.../libx2g_ctrace.so).  Thread 0 of every workgroup (one per unit: a
pack of center atoms, or one atom) stamps a 100 MHz clock at: start, row tables built, rows staged, P products
done, end (after a trace-build-only barrier).  Prints per-phase medians / p90 and the workgroups' overlap.

    python scripts/trace_center_fwd.py [molecules] [packs|degree]"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "x2-gnn_amd"))
from x2gnn import _lib, ops  # noqa: E402
from x2gnn._lib import call, ptr, stream_ptr  # noqa: E402
from x2gnn.data import center_packs, collate  # noqa: E402
from x2gnn.synth import synthetic_molecules  # noqa: E402

nmol = int(sys.argv[1]) if len(sys.argv) > 1 else 128
mode = sys.argv[2] if len(sys.argv) > 2 else "packs"
dev = torch.device("cuda")
b = collate(synthetic_molecules(nmol, "S160", seed=1000))
ei = b.edge_index.to(dev)
n = b.num_nodes
T = int(b._meta["triplets"].sum())
e32 = ops._i32(ei)
lg = ops.LineGraph(e32[0].contiguous(), e32[1].contiguous(), n, T, symmetric=True)
z = b.x.to(dev)
lg.src_type = ops._i32(z[ei[0]])
deg_all = np.bincount(b.edge_index[0].numpy(), minlength=n)
md = int(deg_all.max())
if mode == "packs":
    po, pp, rows = center_packs(deg_all)
    order, packs, units = torch.from_numpy(po).to(dev), torch.from_numpy(pp).to(dev), len(pp) - 1
    info = b._store["_x2g_pack_info"].to(dev)  # (collate's: the same packs)
    unit_rows = np.array([deg_all[po[pp[u]:pp[u + 1]]].sum() for u in range(units)])
else:
    po = np.argsort(-deg_all, kind="stable").astype(np.int32)
    order, packs, units, rows, info = torch.from_numpy(po).to(dev), None, n, md, None
    unit_rows = deg_all[po]
E, H, C, D = lg.E, 16, 8, 128
g = torch.Generator(device=dev).manual_seed(3)
q, k, v, skip = (torch.randn(E, D, device=dev, generator=g) for _ in range(4))
table = torch.randn(10, D, device=dev, generator=g)
radial = torch.randn(E, 42, device=dev, generator=g)
y = torch.randn(T, 8, device=dev, generator=g)
W = 0.2 * torch.randn(D, 42, device=dev, generator=g)
bias = 0.1 * torch.randn(D, device=dev, generator=g)
f = dict(device=dev, dtype=torch.float32)
out, alpha, S = torch.empty(E, D, **f), torch.empty(T, H, **f), torch.empty(T, D, **f)
smax, sden, rs = torch.empty(E, H, **f), torch.empty(E, H, **f), torch.empty(E, 2, **f)
lib = _lib.load()
lib.x2g_ftrace_fetch.argtypes = [ctypes.c_void_p, ctypes.c_int]
def run(store):
    ev = []
    for it in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        call("x2g_sbf_attention_fwd_center_sf", ptr(q), ptr(k), ptr(v), ptr(skip), ptr(table), ptr(lg.src_type),
             ops.EDGE_PER_DST, ptr(radial), ptr(y), ptr(W), ptr(bias), ptr(lg.atom_rowptr), ptr(lg.edge_rev),
             ptr(lg.rev_trip), ptr(order), ptr(packs), ptr(info), 0, units, rows, E, T, H, C, ptr(out), ptr(alpha), ptr(smax),
             ptr(sden), ptr(rs), ptr(S) if store else None, None, stream_ptr())
        e1.record()
        torch.cuda.synchronize()
        ev.append(e0.elapsed_time(e1) * 1e3)
    return ev


# without the S rows a backward reads (inference) first, for the comparison; the stamps are the training form's
print(f"kernel (events) without the S store: {np.median(run(False)):.1f} us")
ev = run(True)
buf = np.zeros(8192 * 8, dtype=np.uint64)
assert lib.x2g_ftrace_fetch(buf.ctypes.data, buf.size) == 0
t = buf.reshape(8192, 8)[:units].astype(np.int64)
live = unit_rows > 0
t, ur = t[live], unit_rows[live]
t0 = t[:, 0].min()
print(f"{mode}: workgroups {units}, rows max {rows}; kernel (events) {np.median(ev):.1f} us; "
      f"span of the stamps {(t[:, 4].max() - t0) / 100:.1f} us")
for kk, name in enumerate(["tables", "staging", "P products", "owner loop + end"]):
    d = (t[:, kk + 1] - t[:, kk]) / 100.0
    print(f"  {name:18s} median {np.median(d):7.2f} us  p90 {np.percentile(d, 90):7.2f}  max {d.max():7.2f}")
life = (t[:, 4] - t[:, 0]) / 100.0
print(f"  workgroup life     median {np.median(life):7.2f} us  p90 {np.percentile(life, 90):7.2f}  max {life.max():7.2f}")
starts = np.sort((t[:, 0] - t0) / 100.0)
print("  start-time percentiles (us):", " ".join(f"{np.percentile(starts, p):.1f}" for p in (0, 10, 25, 50, 75, 90, 100)))
span = int((t[:, 4].max() - t0) / 100) + 1
alive = np.zeros(span + 1)
for s0, s1 in zip((t[:, 0] - t0) // 100, (t[:, 4] - t0) // 100):
    alive[s0:s1 + 1] += 1
print("  workgroups alive (every 5 us):", " ".join(str(int(a)) for a in alive[::5]))
