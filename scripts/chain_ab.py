"""A/B of the row-chain kernel variants (x2g_tuning key 6) at config-2 size, interleaved so clock /
cache warm-up does not favour either: 7-stage trunk chain forward and backward, T-layout outputs
as the model runs them.  Prints the minimum over rounds for each variant."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "x2-gnn_amd"))
from x2gnn import _lib, ops  # noqa: E402
from x2gnn._lib import ptr, stream_ptr  # noqa: E402

dev = torch.device("cuda")
lib = _lib.load()
R, D, n = int(os.environ.get("ROWS", "21058")), 128, 7
S, H, RH, RE = ops.CHAIN_SILU, ops.CHAIN_HOLD, ops.CHAIN_RES_HELD, ops.CHAIN_RES_EXT
flags = [S | H, S | RH, S | RE, S | H, S | RH, S | H, S | RH]
x, res, dy = (torch.randn(R, D, device=dev) for _ in range(3))
W = [torch.randn(D, D, device=dev) / 11.3 for _ in range(n)]
B = [torch.randn(D, device=dev) * 0.1 for _ in range(n)]
Z = [torch.empty(R, D, device=dev) for _ in range(n)]
WT = [torch.empty(D, D, device=dev) for _ in range(n)]
y, dx, dres = (torch.empty(R, D, device=dev) for _ in range(3))
tf = int(lib.x2g_chain_t_floats(R, D))
in_t, dz_t = torch.empty(n, tf, device=dev), torch.empty(n, tf, device=dev)
st = (ops.ChainStage * n)(*[ops.ChainStage(W[i].data_ptr(), B[i].data_ptr(), Z[i].data_ptr(),
                                           y.data_ptr() if i == n - 1 else None, WT[i].data_ptr(), flags[i])
                            for i in range(n)])
bst = (ops.ChainBwdStage * n)(*[ops.ChainBwdStage(W[i].data_ptr(), WT[i].data_ptr(), Z[i].data_ptr(), None, flags[i])
                                for i in range(n)])


def t(fn, reps=40):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


fwd = lambda: lib.x2g_chain_fwd(ptr(x), ptr(res), st, n, R, D, ptr(in_t), stream_ptr())  # noqa: E731
bwd = lambda: lib.x2g_chain_bwd(ptr(dy), None, bst, n, R, D, ptr(dx), ptr(dres), ptr(dz_t), stream_ptr())  # noqa: E731
names = {0: "default (fwd v4)", 2: "v2", 3: "fwd v3"}
knobs = [int(k) for k in os.environ.get("KNOBS", "2,0").split(",")]
outs = {}
for k in knobs:  # outputs of each variant (y, z, T-layout inputs; dx, d res, T-layout dz) for a bitwise comparison
    lib.x2g_tuning(6, k)
    fwd()
    bwd()
    torch.cuda.synchronize()
    outs[k] = [y.clone(), in_t.clone()] + [z.clone() for z in Z] + [dx.clone(), dres.clone(), dz_t.clone()]
for k in knobs[1:]:
    same = all(torch.equal(a, b) for a, b in zip(outs[knobs[0]], outs[k]))
    err = max(float((a - b).abs().max()) for a, b in zip(outs[knobs[0]], outs[k]))
    print(f"{names[k]} vs {names[knobs[0]]}: forward + backward outputs bitwise equal: {same} (max abs diff {err:.3g})", flush=True)
best = {k: [1e9, 1e9] for k in knobs}
for rnd in range(4):
    for k in (knobs if rnd % 2 == 0 else knobs[::-1]):
        lib.x2g_tuning(6, k)
        best[k][0] = min(best[k][0], t(fwd))
        best[k][1] = min(best[k][1], t(bwd))
lib.x2g_tuning(6, 0)
for k, (f, b) in best.items():
    print(f"{names[k]:14s}: fwd {f:6.1f} us  bwd {b:6.1f} us", flush=True)
