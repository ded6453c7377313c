"""Per-kernel floor of a HIP-graph replay: N tiny kernels captured in one
graph, replayed; prints microseconds per kernel."""
import torch

x = torch.zeros(64, device="cuda")
for n in (10, 100):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            x.add_(1.0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            x.add_(1.0)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"graph of {n} tiny kernels: {e0.elapsed_time(e1) / 20 / n * 1000:.2f} us/kernel",
          flush=True)
