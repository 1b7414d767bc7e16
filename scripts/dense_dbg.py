"""Phase costs of dense_fwd_staged: time it with parts switched off (x2g_tuning key 3 bitmask:
1 = no weight staging, 2 = 1/16 of the MFMA loop, 4 = no epilogue stores)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "x2-gnn_amd"))
from x2gnn import _lib  # noqa: E402
from x2gnn._lib import call, ptr, stream_ptr  # noqa: E402

dev = torch.device("cuda")
lib = _lib.load()
K = N = 128
for R in (21058, 262144):
    x = torch.randn(R, K, device=dev)
    w = torch.randn(N, K, device=dev) * 0.1
    b = torch.randn(N, device=dev)
    res = torch.randn(R, N, device=dev)
    y = torch.empty(R, N, device=dev)
    z = torch.empty(R, N, device=dev)
    for dbg in (0, 1, 2, 4, 6, 7):
        lib.x2g_tuning(3, dbg)
        for _ in range(20):
            call("x2g_dense_fwd", ptr(x), ptr(w), ptr(b), R, K, N, 1, ptr(res), ptr(y), ptr(z), stream_ptr())
    torch.cuda.synchronize()
    lib.x2g_tuning(3, 0)
    print("R", R, "done", flush=True)
