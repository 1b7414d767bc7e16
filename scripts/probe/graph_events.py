"""Probe: can timing events recorded inside a captured HIP graph time one kernel of each replay?  A
graph of [spin A, event a, spin B, event b, spin C]; after each replay a.elapsed_time(b) should read
spin B's duration."""
import torch

cyc = 2_000_000
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    torch.cuda._sleep(cyc)
    torch.cuda.synchronize()
    try:
        with torch.cuda.graph(g, stream=s):
            torch.cuda._sleep(cyc)
            a.record()
            torch.cuda._sleep(2 * cyc)
            b.record()
            torch.cuda._sleep(cyc)
        ok = True
    except Exception as e:  # noqa: BLE001
        print("capture failed:", repr(e)[:300])
        ok = False
torch.cuda.synchronize()
if ok:
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        try:
            print(f"replay {e0.elapsed_time(e1):.3f} ms; inner events {a.elapsed_time(b):.3f} ms (expect ~half)")
        except Exception as e:  # noqa: BLE001
            print("elapsed failed:", repr(e)[:300])
