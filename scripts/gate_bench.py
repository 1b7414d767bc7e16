"""Graph-replayed timing of the rbf-gate kernels at config-2 size (no host launch overhead):
backward variants (all outputs / no drbf / no dx / weights only) x workgroup caps."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "x2-gnn_amd"))
from x2gnn import _lib  # noqa: E402
from x2gnn._lib import call, ptr, stream_ptr  # noqa: E402

dev = torch.device("cuda")
lib = _lib.load()
E, D, R = 21058, 128, 6
x = torch.randn(E, D, device=dev)
g = torch.randn(E, D, device=dev)
rbf = torch.randn(E, R, device=dev)
w = torch.randn(D, R, device=dev)
b = torch.randn(D, device=dev)
dx = torch.empty(E, D, device=dev)
drbf = torch.empty(E, R, device=dev)
dw = torch.empty(D, R, device=dev)
db = torch.empty(D, device=dev)
out = torch.empty(E, D, device=dev)
owner = torch.arange(E, device=dev, dtype=torch.int32) // 9
n_seg = int(owner[-1]) + 1
rowptr = torch.searchsorted(owner, torch.arange(n_seg + 1, device=dev, dtype=torch.int32)).to(torch.int32)
pooled = torch.randn(n_seg, D, device=dev)


def timed(fn, reps=40):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(reps):
            fn()
    gr.replay()
    torch.cuda.synchronize()
    a, bb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    gr.replay()
    bb.record()
    bb.synchronize()
    return a.elapsed_time(bb) / reps * 1e3


print(f"gate fwd   {timed(lambda: call('x2g_rbf_gate_fwd', ptr(x), ptr(rbf), ptr(w), ptr(b), E, D, R, ptr(out), stream_ptr())):7.1f} us")
print(f"pool fwd   {timed(lambda: call('x2g_rbf_pool_fwd', ptr(x), ptr(rbf), ptr(w), ptr(b), ptr(rowptr), n_seg, D, R, ptr(pooled), stream_ptr())):7.1f} us")
for cap in (256, 512, 1024, 2048):
    lib.x2g_tuning(4, cap)
    wsb = int(lib.x2g_rbf_gate_bwd_workspace(E, D, R))
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    res = []
    for name, o, gg, dxp, drp in (("full", None, g, dx, drbf), ("no-drbf", None, g, dx, None),
                                  ("no-dx", None, g, None, drbf), ("w-only", None, g, None, None),
                                  ("pool", owner, pooled, dx, drbf)):
        t = timed(lambda: call("x2g_rbf_gate_bwd", ptr(gg), ptr(o), ptr(x), ptr(rbf), ptr(w), ptr(b), E, D, R, ptr(dxp),
                               None, ptr(drp), ptr(dw), ptr(db), 2, ptr(ws), wsb, stream_ptr()))
        res.append(f"{name} {t:6.1f}")
    print(f"bwd cap {cap:5d}: " + "  ".join(res) + " us (slab sum deferred)")
lib.x2g_tuning(4, 0)
