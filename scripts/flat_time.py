"""Kernel time of the flat T-layout weight-gradient launch (x2g_tiled_wgrad_flat, the config-2 step's
52 jobs over 21,058 rows) for the library X2G_LIB names: median of 10 launches, HIP events.

    X2G_LIB=x2-gnn_amd/lib/ab/libx2g_NAME.so python scripts/flat_time.py"""
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
ts = []
for it in range(12):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    call("x2g_tiled_wgrad_flat", jobs, n, R, D, ops.ACCUM_WGRAD | ops.DEFER_SLAB_SUM, out, ptr(ws), wsb, stream_ptr())
    e1.record()
    torch.cuda.synchronize()
    if it >= 2:
        ts.append(e0.elapsed_time(e1) * 1e3)
print(f"{os.path.basename(_lib.LIB_PATH)}: flat {np.median(ts):.1f} us (min {min(ts):.1f}) "
      f"{35.4e9 / (np.median(ts) * 1e-6) / 1e12:.1f} TF/s")
