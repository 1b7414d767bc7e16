"""Featurisation kernels at config-2 size (E = 21,058 line nodes, 338 -> 256 -> 128): time per
launch of x2g_feat_fwd (with the x2g_tuning key-8 ablations), x2g_feat_bwd and the 8-job T-layout
weight gradient, HIP events on the launch stream."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "x2-gnn_amd"))
from x2gnn import _lib, ops  # noqa: E402
from x2gnn.layers import Linear  # noqa: E402

dev = torch.device("cuda")
lib = _lib.load()
R = int(os.environ.get("ROWS", "21058"))


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


x = 0.3 * torch.randn(R, 338, device=dev)
env = torch.rand(R, device=dev)
l1, l2 = Linear(338, 256).to(dev), Linear(256, 128).to(dev)
gy = torch.randn(R, 128, device=dev)
for dbg, what in ((0, "full"), (1, "no GEMM1"), (2, "no GEMM2"), (4, "no stores"), (8, "no staging"),
                  (3, "no GEMMs"), (15, "nothing")):
    lib.x2g_tuning(8, dbg)
    with torch.no_grad():
        us = t(lambda: ops._FeaturizeFn.apply(x, env, l1.weight, l1.bias, l2.weight, l2.bias))
    print(f"feat_fwd dbg={dbg:2d} ({what:10s}): {us:7.1f} us")
lib.x2g_tuning(8, 0)


def fb():
    y = ops._FeaturizeFn.apply(x, env, l1.weight, l1.bias, l2.weight, l2.bias)
    y.backward(gy)


print(f"fwd+bwd (incl. weight gradients, slab sums): {t(fb):7.1f} us")
