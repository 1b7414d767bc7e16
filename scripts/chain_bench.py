"""Row-chain kernels at config-2 size (E = 21,058 rows): time per launch of x2g_chain_fwd /
x2g_chain_bwd / x2g_wgrad_batched for 1..7 stages and both kernel variants (x2g_tuning key 6)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "x2-gnn_amd"))
from x2gnn import _lib, ops  # noqa: E402
from x2gnn._lib import ptr, stream_ptr  # noqa: E402

dev = torch.device("cuda")
lib = _lib.load()
R = int(os.environ.get("ROWS", "21058"))
D = 128
S, H, RH, RE = ops.CHAIN_SILU, ops.CHAIN_HOLD, ops.CHAIN_RES_HELD, ops.CHAIN_RES_EXT
TRUNK = [S | H, S | RH, S | RE, S | H, S | RH, S | H, S | RH]


def t(fn, reps=30):
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


x = torch.randn(R, D, device=dev)
res = torch.randn(R, D, device=dev)
W = [torch.randn(D, D, device=dev) / 11.3 for _ in range(7)]
B = [torch.randn(D, device=dev) * 0.1 for _ in range(7)]
Z = [torch.empty(R, D, device=dev) for _ in range(7)]
Y = [torch.empty(R, D, device=dev) for _ in range(7)]
DZ = [torch.empty(R, D, device=dev) for _ in range(7)]
dx = torch.empty(R, D, device=dev)
dres = torch.empty(R, D, device=dev)
dy = torch.randn(R, D, device=dev)
DW = [torch.empty(D, D, device=dev) for _ in range(7)]
WT = [torch.empty(D, D, device=dev) for _ in range(7)]
DB = [torch.empty(D, device=dev) for _ in range(7)]
for knob in (0, 2, 1):
    lib.x2g_tuning(6, knob)
    for n in (1, 2, 7):
        flags = TRUNK[:n] if n != 1 else [S]
        if n == 2:
            flags = [S | H, S | RH]
        # as the model runs it (ops._ChainFn): v2 keeps the stage inputs / dz in the T layout only
        t_only = knob in (0, 2)
        st = (ops.ChainStage * n)(*[ops.ChainStage(W[i].data_ptr(), B[i].data_ptr(), Z[i].data_ptr(),
                                                   Y[i].data_ptr() if (i == n - 1 or not t_only) else None,
                                                   WT[i].data_ptr(), flags[i]) for i in range(n)])
        bst = (ops.ChainBwdStage * n)(*[ops.ChainBwdStage(W[i].data_ptr(), WT[i].data_ptr() if t_only else None,
                                                          Z[i].data_ptr(), None if t_only else DZ[i].data_ptr(),
                                                          flags[i]) for i in range(n)])
        tf = int(lib.x2g_chain_t_floats(R, D))
        in_t = torch.empty(n, tf, device=dev) if knob in (0, 2) else None
        dz_t = torch.empty(n, tf, device=dev) if knob in (0, 2) else None
        f = t(lambda: lib.x2g_chain_fwd(ptr(x), ptr(res), st, n, R, D, ptr(in_t), stream_ptr()))
        b = t(lambda: lib.x2g_chain_bwd(ptr(dy), None, bst, n, R, D, ptr(dx), ptr(dres), ptr(dz_t), stream_ptr()))
        if knob == 0:
            wsz = int(lib.x2g_chain_wgrad_workspace(R, D, n))
            wsb = torch.empty(wsz, dtype=torch.uint8, device=dev)
            dwa = (ctypes.c_void_p * n)(*[DW[i].data_ptr() for i in range(n)])
            dba = (ctypes.c_void_p * n)(*[DB[i].data_ptr() for i in range(n)])
            cw = t(lambda: lib.x2g_chain_wgrad(ptr(in_t), ptr(dz_t), n, R, D, dwa, dba, 2, ptr(wsb), wsz, stream_ptr()))
            print(f"  chain_wgrad stages {n}: {cw:7.1f} us deferred ({2 * R * D * D * n / cw / 1e6:5.1f} TF/s), "
                  f"splits {lib.x2g_chain_wgrad_splits(R, D, n)}", flush=True)
        print(f"knob {knob} stages {n}: fwd {f:7.1f} us ({f / n:5.1f}/stage, {2 * R * D * D * n / f / 1e6:5.1f} TF/s)  "
              f"bwd-data {b:7.1f} us ({b / n:5.1f}/stage)", flush=True)
lib.x2g_tuning(6, 0)
for G in (1, 7):
    ws = int(lib.x2g_wgrad_batched_workspace(R, D, G))
    wsb = torch.empty(ws, dtype=torch.uint8, device=dev)
    jobs = (ops.WgradJob * G)(*[ops.WgradJob(DZ[g].data_ptr(), Y[g].data_ptr(), DW[g].data_ptr(), DB[g].data_ptr())
                                for g in range(G)])
    w = t(lambda: lib.x2g_wgrad_batched(jobs, G, R, D, 0, ptr(wsb), ws, stream_ptr()))
    w2 = t(lambda: lib.x2g_wgrad_batched(jobs, G, R, D, 2, ptr(wsb), ws, stream_ptr()))
    print(f"wgrad_batched G={G}: {w:7.1f} us with slab sum, {w2:7.1f} us deferred "
          f"({2 * R * D * D * G / w2 / 1e6:5.1f} TF/s), splits {lib.x2g_wgrad_batched_splits(R, D, G)}", flush=True)
# ablations of the run-time-flag forward (x2g_tuning key 7): what each phase of a stage costs
lib.x2g_tuning(6, 0)
n = 7
st = (ops.ChainStage * n)(*[ops.ChainStage(W[i].data_ptr(), B[i].data_ptr(), Z[i].data_ptr(), Y[i].data_ptr(), None,
                                           TRUNK[i]) for i in range(n)])
for dbg in (0, 2, 4, 8, 2 | 4 | 8, 16, 2 | 16, 2 | 4 | 8 | 16):
    lib.x2g_tuning(7, dbg)
    f = t(lambda: lib.x2g_chain_fwd(ptr(x), ptr(res), st, n, R, D, None, stream_ptr()))
    print(f"ablation {dbg:2d}: fwd {f:7.1f} us ({f / n:5.1f}/stage)", flush=True)
lib.x2g_tuning(7, 0)
