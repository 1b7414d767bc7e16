"""Phase timeline of the center-atom attention backward (x2g_sbf_attention_bwd_center; A/B trace build
only: make -C x2-gnn_amd ab AB_UNIT=attention_center AB_NAME=ctrace AB_FLAGS=-DX2G_TRACE, run with
X2G_LIB=.../libx2g_ctrace.so).  Thread 0 of every workgroup (one per center atom) stamps a 100 MHz clock at
its phase boundaries: start, staging done, pass 1 done (its own), fence + barrier, rho + barrier, pass 2
done, end.  Prints per-phase medians / p90 over the workgroups and how the workgroups overlap in time.

    python scripts/trace_center_bwd.py [molecules] [degree|ident]"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "x2-gnn_amd"))
from x2gnn import _lib, ops  # noqa: E402
from x2gnn._lib import call, ptr, stream_ptr  # noqa: E402
from x2gnn.data import collate  # noqa: E402
from x2gnn.synth import synthetic_molecules  # noqa: E402

nmol = int(sys.argv[1]) if len(sys.argv) > 1 else 128
dev = torch.device("cuda")
b = collate(synthetic_molecules(nmol, "S160", seed=1000))
ei = b.edge_index.to(dev)
n = b.num_nodes
T = int(b._meta["triplets"].sum())
e32 = ops._i32(ei)
lg = ops.LineGraph(e32[0].contiguous(), e32[1].contiguous(), n, T, symmetric=True)
z = b.x.to(dev)
lg.src_type, lg.dst_type, lg.atom_type = ops._i32(z[ei[0]]), ops._i32(z[ei[1]]), ops._i32(z)
deg_all = np.bincount(b.edge_index[0].numpy(), minlength=n)
md = int(deg_all.max())
# launch order: by decreasing degree (the model's), or the identity with "ident" as the second argument
mode = sys.argv[2] if len(sys.argv) > 2 else "degree"
rows, units = md, n
order = None if mode == "ident" else torch.from_numpy(np.argsort(-deg_all, kind="stable").astype(np.int32)).to(dev)
ordn = order.cpu().numpy() if order is not None else np.arange(n)
unit_rows = unit_maxdeg = deg_all[ordn]
E, H, C, D = lg.E, 16, 8, 128
g = torch.Generator(device=dev).manual_seed(3)
q, k, v, skip, dout = (torch.randn(E, D, device=dev, generator=g) for _ in range(5))
S = torch.randn(T, D, device=dev, generator=g)
table = torch.randn(10, D, device=dev, generator=g)
y = torch.randn(T, 8, device=dev, generator=g)
f = dict(device=dev, dtype=torch.float32)
out, alpha = torch.empty(E, D, **f), torch.empty(T, H, **f)
smax, sden = torch.empty(E, H, **f), torch.empty(E, H, **f)
call("x2g_sbf_attention_fwd_center", ptr(q), ptr(k), ptr(v), ptr(skip), ptr(table), ptr(lg.src_type),
     ops.EDGE_PER_DST, ptr(S), 0, ptr(lg.atom_rowptr), ptr(lg.edge_rev), ptr(lg.rev_trip), None, 0, n, md, E, T,
     H, C, ptr(out), ptr(alpha), ptr(smax), ptr(sden), None, stream_ptr())
dq, dk, dv = (torch.empty(E, D, **f) for _ in range(3))
G, de, gw = torch.empty(E, 8, D, **f), torch.empty(n, D, **f), torch.empty(2, T, H, **f)
lib = _lib.load()
lib.x2g_ctrace_fetch.argtypes = [ctypes.c_void_p, ctypes.c_int]
ev = []
for it in range(6):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    call("x2g_sbf_attention_bwd_center", ptr(q), ptr(k), ptr(v), ptr(table), ptr(lg.src_type), ops.EDGE_PER_DST,
         ptr(S), None, None, ptr(y), ptr(lg.atom_rowptr), ptr(lg.edge_rev), ptr(lg.rev_trip), ptr(order), ptr(alpha),
         ptr(smax), ptr(sden), ptr(dout), units, rows, E, T, H, C, ptr(dq), ptr(dk), ptr(dv), ptr(G), ptr(de), ptr(gw),
         stream_ptr())
    e1.record()
    torch.cuda.synchronize()
    ev.append(e0.elapsed_time(e1) * 1e3)
buf = np.zeros(8192 * 8, dtype=np.uint64)
assert lib.x2g_ctrace_fetch(buf.ctypes.data, buf.size) == 0
t = buf.reshape(8192, 8)[:units].astype(np.int64)
# stamps are per workgroup: workgroup w ran unit w (its rows: the degrees of its atoms summed)
deg = unit_maxdeg
live = unit_rows > 0
t, deg = t[live], deg[live]
t0 = t[:, 0].min()
print(f"{mode}: atoms {n}, workgroups {units} (with rows {live.sum()}), E {E}, T {T}, max degree {md}, max rows {rows}; "
      f"kernel (events) "
      f"{np.median(ev):.1f} us; span of the stamps {(t[:, 6].max() - t0) / 100:.1f} us")
names = ["staging", "pass 1 (own)", "fence + barrier", "rho + barrier", "pass 2", "d_edge + end"]
for kk, name in enumerate(names):
    d = (t[:, kk + 1] - t[:, kk]) / 100.0
    print(f"  {name:16s} median {np.median(d):7.2f} us  p90 {np.percentile(d, 90):7.2f}  max {d.max():7.2f}")
life = (t[:, 6] - t[:, 0]) / 100.0
print(f"  workgroup life   median {np.median(life):7.2f} us  p90 {np.percentile(life, 90):7.2f}  max {life.max():7.2f}")
for lo, hi in ((2, 8), (9, 12), (13, 17)):
    sel = (deg >= lo) & (deg <= hi)
    if sel.any():
        print(f"  largest degree {lo:2d}-{hi:2d}: {sel.sum():5d} workgroups, life median {np.median(life[sel]):6.2f} us, "
              f"pass 1 median {np.median((t[sel, 2] - t[sel, 1]) / 100):6.2f} us")
starts = np.sort((t[:, 0] - t0) / 100.0)
print("  start-time percentiles (us):", " ".join(f"{np.percentile(starts, p):.1f}" for p in (0, 10, 25, 50, 75, 90, 100)))
# concurrency: workgroups alive at each microsecond
span = int((t[:, 6].max() - t0) / 100) + 1
alive = np.zeros(span + 1)
for s0, s1 in zip((t[:, 0] - t0) // 100, (t[:, 6] - t0) // 100):
    alive[s0:s1 + 1] += 1
print("  workgroups alive (every 10 us):", " ".join(str(int(a)) for a in alive[::10]))
