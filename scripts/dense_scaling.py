"""Dense fwd/bwd kernel time vs row count (separates the fixed start-up cost from per-tile cost)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "x2-gnn_amd"))
from x2gnn import _lib  # noqa: E402
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


K = N = 128
for R in (32, 8192, 21058, 65536, 262144):
    x = torch.randn(R, K, device=dev)
    w = torch.randn(N, K, device=dev) * 0.1
    b = torch.randn(N, device=dev)
    res = torch.randn(R, N, device=dev)
    y = torch.empty(R, N, device=dev)
    z = torch.empty(R, N, device=dev)
    dy = torch.randn(R, N, device=dev)
    dx = torch.empty(R, K, device=dev)
    dw = torch.empty(N, K, device=dev)
    db = torch.empty(N, device=dev)
    wsb = lib.x2g_dense_bwd_workspace(R, K, N)
    ws = torch.empty(max(wsb, 4) // 4 + 1, device=dev)
    fwd_v = []
    for v in (1, 0):  # key 3: 1 = v5, 0 = v6 (default)
        lib.x2g_tuning(3, v)
        fwd_v.append(t(lambda: call("x2g_dense_fwd", ptr(x), ptr(w), ptr(b), R, K, N, 1, ptr(res), ptr(y), ptr(z),
                                    stream_ptr())))
    lib.x2g_tuning(3, 0)
    fwd = fwd_v[-1]
    bwd = t(lambda: call("x2g_dense_bwd", ptr(dy), ptr(z), 1, ptr(x), ptr(w), R, K, N, ptr(dx), ptr(dw), ptr(db),
                         ptr(ws), wsb, stream_ptr()))
    ref = torch.nn.functional.silu(torch.nn.functional.linear(x, w, b)) + res
    err = float((y - ref).abs().max())
    gemm = t(lambda: torch.nn.functional.linear(x, w, b))
    fl = 2 * R * K * N
    print(f"R={R:7d} fwd(v5) {fwd_v[0]:8.1f}us fwd(v6) {fwd:8.1f}us ({fl / fwd / 1e6:6.1f} TF/s, {4 * R * (K + 3 * N) / fwd / 1e3:6.0f} GB/s) "
          f"bwd {bwd:8.1f}us ({2 * fl / bwd / 1e6:6.1f} TF/s) | torch linear {gemm:7.1f}us | err {err:.1e}",
          flush=True)
