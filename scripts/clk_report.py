"""SCLK a kernel ran at, from a trace build's x2g_clk_buf (core-clock and 100 MHz wall-clock stamps of
thread 0 of every workgroup at the kernel's start and end): median over workgroups of
delta(core) / delta(wall) x 100 MHz.  Imported by the trace scripts after their last launch."""
import ctypes

import numpy as np


def report(lib, label):
    lib.x2g_clk_fetch.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = np.zeros(1024 * 4, dtype=np.uint64)
    if lib.x2g_clk_fetch(buf.ctypes.data, buf.size) != 0:
        return
    t = buf.reshape(1024, 4).astype(np.float64)
    t = t[(t[:, 3] > t[:, 1]) & (t[:, 1] > 0)]
    if len(t) == 0:
        return
    ghz = (t[:, 2] - t[:, 0]) / (t[:, 3] - t[:, 1]) * 0.1
    span = (t[:, 3] - t[:, 1]) / 100.0
    print(f"{label}: SCLK median {np.median(ghz):.3f} GHz (min {ghz.min():.3f}, max {ghz.max():.3f}) over {len(t)} "
          f"workgroups; workgroup span median {np.median(span):.1f} us")
