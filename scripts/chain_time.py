"""Kernel time of the trunk chain forward and backward (x2g_chain_fwd / x2g_chain_bwd, 7 stages at the
config-2 row count) for the library X2G_LIB names: median of 20 launches each, HIP events on the
launching stream.

    X2G_LIB=x2-gnn_amd/lib/ab/libx2g_NAME.so python scripts/chain_time.py [rows]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "x2-gnn_amd"))
from x2gnn import _lib, ops  # noqa: E402
from x2gnn._lib import call, ptr, stream_ptr  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 21058
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


def fwd():
    call("x2g_chain_fwd", ptr(x), ptr(res), st, n, R, D, ptr(in_t), stream_ptr())


def bwd():
    call("x2g_chain_bwd", ptr(dy), None, bst, n, R, D, ptr(dx), ptr(dres), ptr(dz_t), stream_ptr())


def timed(f, reps=20):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return float(np.median(ts))


fwd()
bwd()
torch.cuda.synchronize()
out = (float(y.double().abs().sum()), float(dx.double().abs().sum()))
print(f"{os.path.basename(_lib.LIB_PATH)}: rows {R} fwd {timed(fwd):.1f} us bwd {timed(bwd):.1f} us "
      f"(checksums {out[0]:.6e} {out[1]:.6e})")
