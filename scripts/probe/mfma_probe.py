"""Runs scripts/probe/libmfma_probe.so: sustained f32 MFMA rate of the chain product loop."""
import ctypes
import os

import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmfma_probe.so"))
src = torch.randn(4096, device="cuda")
out = torch.empty(256 * 512 * 4, device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
RB = {0: 6, 1: 6, 2: 8, 3: 4}
for v in (0, 1, 2, 3):
    for grid in (256, 512):
        iters = 200
        fn = lambda: lib.probe_run(v, ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(out.data_ptr()), iters, grid, st)
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            fn()
        b.record()
        b.synchronize()
        us = a.elapsed_time(b) / 10 * 1e3
        flops = grid * 8 * iters * 8 * 4 * RB[v] * 2 * 16 * 16 * 4
        print(f"variant {v} (RB={RB[v]}, {'LDS' if v != 1 else 'reg'} B) grid {grid}: {us:8.1f} us  {flops / us / 1e6:6.1f} TF/s",
              flush=True)
