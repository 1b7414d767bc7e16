"""Kernel-only timing of the dense forward variants (x2g_tuning key 0) vs hipBLASLt."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "x2-gnn_amd"))
from x2gnn import _lib, ops  # noqa: E402
from x2gnn._lib import call, ptr, stream_ptr  # noqa: E402

dev = torch.device("cuda")
lib = _lib.load()


def t(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


for R, K, N in [(21058, 128, 128), (2304, 128, 128), (21058, 6, 128), (10, 128, 128)]:
    x = torch.randn(R, K, device=dev)
    w = torch.randn(N, K, device=dev) * 0.1
    b = torch.randn(N, device=dev)
    res = torch.randn(R, N, device=dev)
    y = torch.empty(R, N, device=dev)
    z = torch.empty(R, N, device=dev)
    ref = torch.nn.functional.silu(torch.nn.functional.linear(x, w, b)) + res
    line = f"R={R:6d} K={K:3d} N={N:3d} "
    for v in (0, 1, 2):
        lib.x2g_tuning(0, v)
        fn = lambda: call("x2g_dense_fwd", ptr(x), ptr(w), ptr(b), R, K, N, 1, ptr(res), ptr(y), ptr(z), stream_ptr())
        us = t(fn)
        err = float((y - ref).abs().max())
        line += f"| v{v} {us:7.1f}us err {err:.1e} "
    lib.x2g_tuning(0, 0)
    line += f"| torch gemm {t(lambda: torch.nn.functional.linear(x, w, b)):7.1f}us"
    print(line, flush=True)
