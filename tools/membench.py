"""HBM sanity check: torch device copy bandwidth at a few sizes."""
import torch

dev = torch.device("cuda")
for mb in (16, 64, 256, 1024):
    n = mb * 2 ** 20 // 4
    a = torch.randn(n, device=dev)
    b = torch.empty_like(a)
    for _ in range(3):
        b.copy_(a)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"copy {mb} MiB: {ms * 1000:.1f} us  {2 * mb * 2 ** 20 / ms / 1e6:.0f} GB/s", flush=True)
