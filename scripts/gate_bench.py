"""rbf gate / pool backward (x2g_rbf_gate_bwd) at config-2 size: E = 21,058 rows, D = 128, R = 6;
gate (owner = NULL) and pool (owner = atom) forms, per split count (x2g_tuning key 4), A/B
interleaved, minimum over rounds."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "x2-gnn_amd"))
from x2gnn import _lib  # noqa: E402
from x2gnn._lib import ptr, stream_ptr  # noqa: E402

dev = torch.device("cuda")
lib = _lib.load()
E, D, R, N = 21058, 128, 6, 2304
g = torch.randn(E, D, device=dev)
gp = torch.randn(N, D, device=dev)
owner = torch.sort(torch.randint(0, N, (E,), device=dev))[0].int()
x = torch.randn(E, D, device=dev)
rbf = torch.rand(E, R, device=dev)
w = torch.randn(D, R, device=dev)
b = torch.randn(D, device=dev)
dx, drbf = torch.empty(E, D, device=dev), torch.empty(E, R, device=dev)
dw, db = torch.zeros(D, R, device=dev), torch.zeros(D, device=dev)


def t(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, c = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    c.record()
    c.synchronize()
    return a.elapsed_time(c) / reps * 1e3


best = {}
for rnd in range(3):
    for splits in (256, 512, 1024, 2048):
        lib.x2g_tuning(4, splits)
        wsz = int(lib.x2g_rbf_gate_bwd_workspace(E, D, R))
        ws = torch.empty(wsz, dtype=torch.uint8, device=dev)
        for kind, gg, ow, add in (("gate", g, None, dx), ("pool", gp, owner, None)):
            f = lambda: lib.x2g_rbf_gate_bwd(ptr(gg), ptr(ow), ptr(x), ptr(rbf), ptr(w), ptr(b), E, D, R, ptr(dx),  # noqa
                                             ptr(add), ptr(drbf), ptr(dw), ptr(db), 3, ptr(ws), wsz, stream_ptr())
            us = t(f)
            best[(kind, splits)] = min(best.get((kind, splits), 1e9), us)
lib.x2g_tuning(4, 0)
for (kind, splits), us in sorted(best.items()):
    print(f"{kind} splits {splits:5d}: {us:6.1f} us ({(3 * E * D * 4 + E * R * 8) / us / 1e3:6.0f} GB/s nominal)")
