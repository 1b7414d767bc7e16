"""Phase timeline of the trunk chain backward (x2g_chain_bwd, 7 stages; A/B trace build only:
make -C x2-gnn_amd ab AB_NAME=trace AB_FLAGS=-DX2G_TRACE, run with X2G_LIB=.../libx2g_trace.so).
Thread 0 of every workgroup stamps a 100 MHz clock before / after each stage's barrier.

    python scripts/trace_chain.py [rows] [fwd]   (fwd: the forward x2g_chain_fwd instead)"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "x2-gnn_amd"))
from x2gnn import _lib, ops  # noqa: E402
from x2gnn._lib import call, ptr, stream_ptr  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 21120
FWD = len(sys.argv) > 2 and sys.argv[2] == "fwd"
D, n = 128, 7
S, H, RH, RE = ops.CHAIN_SILU, ops.CHAIN_HOLD, ops.CHAIN_RES_HELD, ops.CHAIN_RES_EXT
flags = [S | H, S | RH, S | RE, S | H, S | RH, S | H, S | RH]
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(4)
x, res, dy = (torch.randn(R, D, device=dev, generator=g) for _ in range(3))
W = [torch.randn(D, D, device=dev, generator=g) / 11.3 for _ in range(n)]
B = [0.1 * torch.randn(D, device=dev, generator=g) for _ in range(n)]
Z = [torch.empty(R, D, device=dev) for _ in range(n)]
y, dx, dres = (torch.empty(R, D, device=dev) for _ in range(3))
WT = torch.empty(n, D, D, device=dev)
lib = _lib.load()
tf = int(lib.x2g_chain_t_floats(R, D))
in_t, dz_t = torch.empty(n, tf, device=dev), torch.empty(n, tf, device=dev)
st = (ops.ChainStage * n)(*[ops.ChainStage(W[i].data_ptr(), B[i].data_ptr(), Z[i].data_ptr(),
                                           y.data_ptr() if i == n - 1 else None, WT[i].data_ptr(), flags[i])
                            for i in range(n)])
bst = (ops.ChainBwdStage * n)(*[ops.ChainBwdStage(W[i].data_ptr(), WT[i].data_ptr(), Z[i].data_ptr(), None, flags[i])
                                for i in range(n)])
call("x2g_chain_fwd", ptr(x), ptr(res), st, n, R, D, ptr(in_t), stream_ptr())
lib.x2g_trace_fetch.argtypes = [ctypes.c_void_p, ctypes.c_int]
for it in range(6):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    if FWD:
        call("x2g_chain_fwd", ptr(x), ptr(res), st, n, R, D, ptr(in_t), stream_ptr())
    else:
        call("x2g_chain_bwd", ptr(dy), None, bst, n, R, D, ptr(dx), ptr(dres), ptr(dz_t), stream_ptr())
    e1.record()
    torch.cuda.synchronize()
buf = np.zeros(1024 * 16, dtype=np.uint64)
assert lib.x2g_trace_fetch(buf.ctypes.data, buf.size) == 0
grid = min(256, (R + 15) // 16)
t = buf.reshape(1024, 16)[:grid].astype(np.int64)
t0 = t[:, 0].min()
if FWD:
    names = ["start", "staged+bar"] + [f"stage{i} {w}" for i in range(n) for w in ("done", "barrier")]
else:
    names = ["start", "stage6 elem+bar"] + [f"stage{n - 1 - i} {w}" for i in range(n) for w in ("done", "barrier")]
print(f"rows {R} grid {grid} event {e0.elapsed_time(e1) * 1e3:.1f} us; relative to the first stamp (us)")
for k in range(len(names)):
    rel = (t[:, k] - t0) / 100.0
    d = (t[:, k] - t[:, k - 1]) / 100.0 if k else rel
    print(f"{k:2d} {names[k]:>16s}  at med {np.median(rel):7.2f} max {rel.max():7.2f}   phase med {np.median(d):6.2f} "
          f"max {d.max():6.2f}")
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import clk_report  # noqa: E402

clk_report.report(lib, "chain fwd" if FWD else "chain bwd")
