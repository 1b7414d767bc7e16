"""Probe: do independent branches of a captured HIP graph run concurrently on this stack?  Two
spin kernels (torch.cuda._sleep, one thread each) on two streams forked / joined inside the capture;
the replay takes ~1x one kernel when the branches overlap, ~2x when the graph runs them one after
the other."""
import time
import torch

dev = torch.device("cuda")
cyc = 20_000_000
main = torch.cuda.current_stream()
side = torch.cuda.Stream()


def one():
    torch.cuda._sleep(cyc)


def two():
    side.wait_stream(torch.cuda.current_stream())
    torch.cuda._sleep(cyc)
    with torch.cuda.stream(side):
        torch.cuda._sleep(cyc)
    torch.cuda.current_stream().wait_stream(side)


for name, fn in (("one kernel", one), ("two branches", two)):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            fn()
    torch.cuda.synchronize()
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    print(f"{name}: graph replay {1e3 * (time.perf_counter() - t) / 10:.2f} ms")
    t = time.perf_counter()
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    print(f"{name}: eager {1e3 * (time.perf_counter() - t) / 10:.2f} ms")
