"""Microbenchmark of the dense kernels vs torch (hipBLASLt + elementwise) at the step's shapes."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "x2-gnn_amd"))
from x2gnn import ops  # noqa: E402

dev = torch.device("cuda")


def t(fn, reps=30):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


for R, K, N in [(21058, 128, 128), (2304, 128, 128), (10, 128, 128), (21058, 6, 128), (21058, 338, 256)]:
    x = torch.randn(R, K, device=dev)
    w = torch.randn(N, K, device=dev) * 0.1
    b = torch.randn(N, device=dev)
    res = torch.randn(R, N, device=dev)
    gy = torch.randn(R, N, device=dev)
    xr = x.clone().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    mine_f = t(lambda: ops.dense(x, w, b, act=1, res=res))
    ref_f = t(lambda: torch.nn.functional.silu(torch.nn.functional.linear(x, w, b)) + res)
    y = ops.dense(xr, wr, br, act=1, res=res)
    mine_b = t(lambda: torch.autograd.grad(y, (xr, wr, br), gy, retain_graph=True))
    yr = torch.nn.functional.silu(torch.nn.functional.linear(xr, wr, br)) + res
    ref_b = t(lambda: torch.autograd.grad(yr, (xr, wr, br), gy, retain_graph=True))
    print(f"R={R:6d} K={K:3d} N={N:3d}  fwd mine {mine_f:7.1f}us torch {ref_f:7.1f}us | "
          f"bwd mine {mine_b:7.1f}us torch {ref_b:7.1f}us", flush=True)
