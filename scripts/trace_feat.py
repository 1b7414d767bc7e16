"""Phase timeline of the featurisation forward (x2g_feat_fwd at config 2: 21,058 line nodes, 338 -> 256 ->
128; A/B trace build only: make -C x2-gnn_amd ab AB_UNIT=feature AB_NAME=ftrace AB_FLAGS=-DX2G_TRACE,
run with X2G_LIB=.../libx2g_ftrace.so).  Thread 0 of every workgroup stamps a 100 MHz clock at 7
points of its first two 32-row tiles: tile start (after the top barrier), staged (scatter + barrier),
x*env T-layout stores, product 1, epilogue 1 + barrier, product 2, epilogue 2."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "x2-gnn_amd"))
from x2gnn import _lib, ops  # noqa: E402
from x2gnn.layers import Linear  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 21058
dev = torch.device("cuda")
torch.manual_seed(0)
x = 0.3 * torch.randn(R, 338, device=dev)
env = torch.rand(R, device=dev) + 0.5
l1, l2 = Linear(338, 256).to(dev), Linear(256, 128).to(dev)
lib = _lib.load()
lib.x2g_feat_trace_fetch.argtypes = [ctypes.c_void_p, ctypes.c_int]
ts = []
for it in range(6):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    y = ops.featurize(x, env, l1, l2)  # parameters require grad: the T-layout operands are written
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) * 1e3)
buf = np.zeros(1024 * 16, dtype=np.uint64)
assert lib.x2g_feat_trace_fetch(buf.ctypes.data, buf.size) == 0
grid = min(256, (R + 31) // 32)
t = buf.reshape(1024, 16)[:grid, :14].astype(np.int64)
t0 = t[:, 0].min()
names = ["start", "staged", "xs_t stored", "product 1", "epi 1 + bar", "product 2", "epi 2"]
print(f"rows {R} grid {grid} featurize (incl. launch overheads) {np.median(ts):.1f} us; relative to the first stamp (us)")
for k in range(14):
    rel = (t[:, k] - t0) / 100.0
    d = (t[:, k] - t[:, k - 1]) / 100.0 if k else rel
    print(f"{k:2d} tile{k // 7} {names[k % 7]:>12s}  at med {np.median(rel):7.2f} max {rel.max():7.2f}   "
          f"phase med {np.median(d):6.2f} max {d.max():6.2f}")
