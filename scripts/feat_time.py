"""Kernel time of the featurisation forward (x2g_feat_fwd through ops.featurize, training mode: the
T-layout operands written) at config 2 (21,058 line nodes, 338 -> 256 -> 128) for the library X2G_LIB
names: median of 20 launches, HIP events, plus an output checksum.

    X2G_LIB=x2-gnn_amd/lib/ab/libx2g_NAME.so python scripts/feat_time.py"""
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
ts = []
for it in range(22):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    y = ops.featurize(x, env, l1, l2)
    e1.record()
    torch.cuda.synchronize()
    if it >= 2:
        ts.append(e0.elapsed_time(e1) * 1e3)
print(f"{os.path.basename(_lib.LIB_PATH)}: featurize fwd {np.median(ts):.1f} us (min {min(ts):.1f}); "
      f"checksum {float(y.double().abs().sum()):.6e}")
