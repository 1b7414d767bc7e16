"""Write-bandwidth ceiling probe for the S projection's output stream: time torch fill_ (pure
stores) and copy_ (read+write) on [rows, 128] f32 buffers at config-2 and config-5 triplet counts."""
import torch

for rows in (194060, 3490000):
    y = torch.empty(rows, 128, device="cuda")
    x = torch.empty(rows, 128, device="cuda").normal_()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name, fn, nbytes in (("fill", lambda: y.fill_(1.0), y.numel() * 4),
                             ("copy", lambda: y.copy_(x), 2 * y.numel() * 4)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s.record()
        for _ in range(20):
            fn()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 20
        print(f"rows={rows} {name}: {ms * 1e3:.1f} us  {nbytes / ms / 1e6:.0f} GB/s", flush=True)
