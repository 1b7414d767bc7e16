"""Phase timeline of the gate-backward projection kernel (A/B trace build only: make -C x2-gnn_amd ab
AB_NAME=trace AB_FLAGS=-DX2G_TRACE; run with X2G_LIB=.../libx2g_trace.so).  Thread 0 of every
workgroup stamps a 100 MHz clock at each phase boundary; prints the per-phase median / max over
workgroups in microseconds.  Usage: python scripts/trace_gate.py [rows]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "x2-gnn_amd"))
from x2gnn import _lib, ops  # noqa: E402
from x2gnn._lib import call, ptr, stream_ptr  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 21120
D, RR = 128, 6
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(7)
G = [torch.randn(R, D, device=dev, generator=g) for _ in range(4)]
W = [torch.randn(D, D, device=dev, generator=g) / 11.3 for _ in range(4)]
WT = [w.t().contiguous() for w in W]
tf = int(_lib.load().x2g_chain_t_floats(R, D))
GT = [torch.empty(tf, device=dev) for _ in range(4)]
x = torch.randn(R, D, device=dev, generator=g)
rbf = torch.randn(R, RR, device=dev, generator=g)
wr = torch.randn(D, RR, device=dev, generator=g)
dx = torch.zeros(R, D, device=dev)
drbf = torch.empty(R, RR, device=dev)
dw = torch.empty(D, RR, device=dev)
wsb = int(_lib.load().x2g_conv_proj_bwd_gate_workspace(R, RR))
ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
grads = (ops.ProjGrad * 4)(*[ops.ProjGrad(G[p].data_ptr(), W[p].data_ptr(), WT[p].data_ptr(), GT[p].data_ptr())
                             for p in range(4)])
lib = _lib.load()
lib.x2g_trace_fetch.argtypes = [ctypes.c_void_p, ctypes.c_int]
grid = int(lib.x2g_conv_proj_bwd_gate_splits(R))
names = ["start"] + [f"c{k} {n}" for k in range(2) for n in ("kv landed", "kv products", "qs landed", "qs products+epi", "dx stored", "-")] + ["", "", ""]
for it in range(6):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    call("x2g_conv_proj_bwd_gate", grads, R, D, ptr(x), ptr(rbf), RR, ptr(wr), ptr(dx), ptr(dx), ptr(drbf), ptr(dw),
         0, ptr(ws), wsb, stream_ptr())
    en.record()
    torch.cuda.synchronize()
    ms = st.elapsed_time(en)
buf = np.zeros(1024 * 16, dtype=np.uint64)
assert lib.x2g_trace_fetch(buf.ctypes.data, buf.size) == 0
t = buf.reshape(1024, 16)[:grid, :13].astype(np.int64)
t0 = t[:, 0].min()
print(f"rows {R} grid {grid} event {ms * 1e3:.1f} us; stamps relative to the first workgroup's start (us)")
for k in range(13):
    rel = (t[:, k] - t0) / 100.0
    d = (t[:, k] - t[:, k - 1]) / 100.0 if k else rel
    print(f"{k:2d} {names[k]:>14s}  at med {np.median(rel):7.2f} max {rel.max():7.2f}   phase med {np.median(d):6.2f} "
          f"max {d.max():6.2f}")
