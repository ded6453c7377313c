"""Probe: hipBLASLt (torch.matmul) bf16 / fp32 times for the IMIM head GEMM
shapes of the stage-1 step (B = 64 images, HW = 196), to price a library
path against tgfr_bgemm."""
import torch

shapes = {"qkv": (12544, 256, 768), "conv1": (12544, 256, 128), "conv2": (12544, 128, 256),
          "lin": (12544, 256, 256), "dW_qkv": (256, 12544, 768), "arc": (64, 256, 4500),
          "attn_qk": (196, 256, 196)}
for dt in (torch.bfloat16, torch.float32):
    for name, (m, k, n) in shapes.items():
        bs = 64 if name == "attn_qk" else 1
        a = torch.randn(bs, m, k, device="cuda", dtype=dt)
        b = torch.randn(bs, k, n, device="cuda", dtype=dt)
        for _ in range(5):
            c = torch.bmm(a, b)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            c = torch.bmm(a, b)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 50 * 1000
        print(f"{str(dt):15s} {name:8s} {bs}x{m}x{k}x{n}: {us:7.1f} us "
              f"{2 * bs * m * k * n / us / 1e6:7.1f} TF", flush=True)
