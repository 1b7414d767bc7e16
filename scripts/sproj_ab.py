"""S projection (x2g_sbf_project, S = lin_sbf(sbf) [T,42] -> [T,128]) at config-2 size: the
wave-independent MFMA kernel (default) vs the tile-staged dense_fwd_narrow (x2g_tuning key 2 = 2),
interleaved rounds, minimum; and parity of the two against fp64 torch."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "x2-gnn_amd"))
from x2gnn import _lib  # noqa: E402
from x2gnn._lib import ptr, stream_ptr  # noqa: E402

dev = torch.device("cuda")
lib = _lib.load()
T = int(os.environ.get("TRIPLETS", "194060"))
sbf = torch.randn(T, 42, device=dev)
w = torch.randn(128, 42, device=dev) / 6.5
b = torch.randn(128, device=dev) * 0.1
out = torch.empty(T, 128, device=dev)


def t(fn, reps=40):
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


f = lambda: lib.x2g_sbf_project(ptr(sbf), T, 42, ptr(w), ptr(b), 128, ptr(out), stream_ptr())  # noqa: E731
ref = (sbf.double() @ w.double().t() + b.double())
best = {}
for rnd in range(4):
    for k in ((0, 2) if rnd % 2 == 0 else (2, 0)):
        lib.x2g_tuning(2, k)
        best[k] = min(best.get(k, 1e9), t(f))
        err = float((out.double() - ref).abs().max())
        assert err < 1e-4, (k, err)
lib.x2g_tuning(2, 0)
nbytes = T * (42 + 128) * 4
for k, us in sorted(best.items()):
    print(f"{'waves (default)' if k == 0 else 'dense_fwd_narrow'}: {us:6.1f} us  {nbytes / us / 1e3:6.0f} GB/s")

# ablations of the wave kernel (x2g_tuning key 9; timing only, the output is wrong when set)
for dbg, what in ((1, "no MFMA"), (2, "no stores"), (3, "loads only")):
    lib.x2g_tuning(9, dbg)
    print(f"waves {what:10s}: {t(f):6.1f} us")
lib.x2g_tuning(9, 0)
