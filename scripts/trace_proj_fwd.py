"""Phase timeline of the projection forward (x2g_conv_proj_fwd; A/B trace build only: make -C
x2-gnn_amd ab AB_NAME=trace AB_FLAGS=-DX2G_TRACE, run with X2G_LIB=.../libx2g_trace.so)."""
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
g = torch.Generator(device=dev).manual_seed(9)
x = torch.randn(R, D, device=dev, generator=g)
rbf = torch.randn(R, RR, device=dev, generator=g)
wr = torch.randn(D, RR, device=dev, generator=g)
W = [torch.randn(D, D, device=dev, generator=g) / 11.3 for _ in range(4)]
Bs = [torch.randn(D, device=dev, generator=g) for _ in range(4)]
out = [torch.empty(R, D, device=dev) for _ in range(4)]
WT = [torch.empty(D, D, device=dev) for _ in range(4)]
lib = _lib.load()
tf = int(lib.x2g_chain_t_floats(R, D))
x_t, xs_t = torch.empty(tf, device=dev), torch.empty(tf, device=dev)
proj = (ops.Proj * 4)(*[ops.Proj(W[p].data_ptr(), Bs[p].data_ptr(), out[p].data_ptr(), WT[p].data_ptr())
                        for p in range(4)])
lib.x2g_trace_fetch.argtypes = [ctypes.c_void_p, ctypes.c_int]
for it in range(6):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    call("x2g_conv_proj_fwd", ptr(x), ptr(rbf), RR, ptr(wr), proj, R, D, ptr(x_t), ptr(xs_t), stream_ptr())
    e1.record()
    torch.cuda.synchronize()
buf = np.zeros(1024 * 16, dtype=np.uint64)
assert lib.x2g_trace_fetch(buf.ctypes.data, buf.size) == 0
grid = min(256, (R + 15) // 16)
names = ["start"] + [f"c{k} {n}" for k in range(2) for n in ("landed", "x_src+copy", "q+skip", "barrier", "k+v")]
t = buf.reshape(1024, 16)[:grid, :len(names)].astype(np.int64)
t0 = t[:, 0].min()
print(f"rows {R} grid {grid} event {e0.elapsed_time(e1) * 1e3:.1f} us; relative to the first stamp (us)")
for k in range(len(names)):
    rel = (t[:, k] - t0) / 100.0
    d = (t[:, k] - t[:, k - 1]) / 100.0 if k else rel
    print(f"{k:2d} {names[k]:>14s}  at med {np.median(rel):7.2f} max {rel.max():7.2f}   phase med {np.median(d):6.2f} "
          f"max {d.max():6.2f}")
