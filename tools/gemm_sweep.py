"""K sweep of one GEMM family (run under rocprofv3 --kernel-trace): separates
a tile's fixed cost (prologue / epilogue) from its per-k-stage cost.

    python tools/gemm_sweep.py            # M=12544 N=128, K = 32 .. 1024
"""
import sys

import torch

sys.path.insert(0, ".")
from text_guided_face_recognition_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
for k in (32, 64, 128, 256, 512, 1024):
    a = torch.randn(1, 12544, k, device=dev)
    b = torch.randn(1, 128, k, device=dev).transpose(1, 2)
    for _ in range(5):
        K.bgemm(a, b, mode="bf16")
    torch.cuda.synchronize()
    print("k", k, flush=True)
