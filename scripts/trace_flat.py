"""Where the flat weight-gradient kernel's time goes (A/B trace build only: make -C x2-gnn_amd ab
AB_NAME=trace AB_FLAGS=-DX2G_TRACE, run with X2G_LIB=.../libx2g_trace.so): thread 0 of every
workgroup sums, over its steps, the time from the end of one step's MFMA issue to the step
barrier's release (copies + barrier) and from there to the end of the next MFMA issue."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "x2-gnn_amd"))
from x2gnn import _lib, ops  # noqa: E402
from x2gnn._lib import call, ptr, stream_ptr  # noqa: E402

R, n, D = 21058, 52, 128
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(5)
lib = _lib.load()
tf = int(lib.x2g_chain_t_floats(R, D))
x_t = [torch.randn(tf, device=dev, generator=g) for _ in range(n)]
dz_t = [torch.randn(tf, device=dev, generator=g) for _ in range(n)]
dw = [torch.zeros(D, D, device=dev) for _ in range(n)]
db = [torch.zeros(D, device=dev) for _ in range(n)]
jobs = (ops.TiledJob * n)(*[ops.TiledJob(dz_t[j].data_ptr(), x_t[j].data_ptr(), dw[j].data_ptr(), db[j].data_ptr(),
                                         0, 0) for j in range(n)])
wsb = int(lib.x2g_tiled_wgrad_flat_workspace(R, D, n))
ws = torch.empty(max(wsb, 4), dtype=torch.uint8, device=dev)
out = (ops.SlabJob * n)()
lib.x2g_trace_fetch.argtypes = [ctypes.c_void_p, ctypes.c_int]
reps = 5
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    call("x2g_tiled_wgrad_flat", jobs, n, R, D, ops.ACCUM_WGRAD | ops.DEFER_SLAB_SUM, out, ptr(ws), wsb, stream_ptr())
e1.record()
torch.cuda.synchronize()
buf = np.zeros(1024 * 16, dtype=np.uint64)
assert lib.x2g_trace_fetch(buf.ctypes.data, buf.size) == 0
t = buf.reshape(1024, 16).astype(np.float64)
t = t[t[:, 2] > 0]  # the launch's workgroups (two per CU)
wait, comp, steps = t[:, 0] / 100.0 / reps, t[:, 1] / 100.0 / reps, t[:, 2] / reps
print(f"{e0.elapsed_time(e1) * 1e3 / reps:.1f} us per launch; {len(t)} workgroups; per workgroup: steps {np.median(steps):.0f}, "
      f"copies+barrier {np.median(wait):.1f} us (max {wait.max():.1f}), MFMA issue {np.median(comp):.1f} us "
      f"(max {comp.max():.1f}); per step {np.median(wait / steps) * 1e3:.0f} + {np.median(comp / steps) * 1e3:.0f} ns")
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import clk_report  # noqa: E402

clk_report.report(lib, "flat")
