"""Lab probe (GPU): hipBLASLt (torch) bf16 GEMM times on the IMIM head's
shapes (B = 64: 12544 rows), as an achievable-time reference for the
hand-written kernels.  Not part of the product."""
import torch

M = 64 * 196


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


dev = torch.device("cuda")
for name, (k, n) in {"qkv": (256, 768), "tail1": (256, 128), "tail2": (128, 256),
                     "tail3": (256, 256)}.items():
    a = torch.randn(M, k, device=dev, dtype=torch.bfloat16)
    w = torch.randn(n, k, device=dev, dtype=torch.bfloat16)
    b = torch.randn(n, device=dev, dtype=torch.bfloat16)
    us = timeit(lambda: torch.nn.functional.linear(a, w, b))
    fl = 2 * M * k * n
    print(f"fwd {name}: M={M} K={k} N={n}: {us:.1f} us ({fl / us / 1e6:.0f} TFLOP/s)")
    g = torch.randn(M, n, device=dev, dtype=torch.bfloat16)
    us = timeit(lambda: g.t() @ a)
    print(f"dW  {name}: {n}x{k} over {M}: {us:.1f} us ({fl / us / 1e6:.0f} TFLOP/s)")
    us = timeit(lambda: g @ w)
    print(f"dX  {name}: {us:.1f} us ({fl / us / 1e6:.0f} TFLOP/s)")
x = torch.randn(M, 256, device=dev)
us = timeit(lambda: x.sum(0))
print(f"colsum fp32 12.8 MB: {us:.1f} us")
y = torch.empty(M, 256, device=dev, dtype=torch.bfloat16)
us = timeit(lambda: y.copy_(x))
print(f"fp32->bf16 copy 12.8+6.4 MB: {us:.1f} us")
