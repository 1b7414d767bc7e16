"""Time the weight-gradient GEMM shapes of one training step under hipBLASLt and rocBLAS."""
import torch, time
dev = torch.device("cuda")
E, T, N = 21058, 194060, 2304
shapes = {"dW E-rows 128x128": (E, 128, 128), "dW sbf T-rows 128x42": (T, 128, 42),
          "dW mat_trans 256x338": (E, 256, 338), "fwd E x128x128": None}
def t(fn, reps=20):
    fn(); torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps): fn()
    b.record(); b.synchronize()
    return a.elapsed_time(b) / reps * 1e3
for lib in ("hipblaslt", "rocblas"):
    torch.backends.cuda.preferred_blas_library(lib)
    for name, shp in shapes.items():
        if shp is None:
            x = torch.randn(E, 128, device=dev); w = torch.randn(128, 128, device=dev); bb = torch.randn(128, device=dev)
            us = t(lambda: torch.nn.functional.linear(x, w, bb))
        else:
            R, O, I = shp
            dy = torch.randn(R, O, device=dev); x = torch.randn(R, I, device=dev)
            us = t(lambda: dy.t() @ x)
        print(f"{lib:10s} {name:24s} {us:9.1f} us", flush=True)
