"""A/B of the weight-resident GEMM (TGFR_GEMM_WRES) against bgemm_glds on the
head's tall products; run under rocprofv3 --kernel-trace (each shape 5 times
per arm, wres arm first)."""
import os
import sys

import torch

sys.path.insert(0, ".")
from text_guided_face_recognition_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
for arm in ("1", "0"):
    os.environ["TGFR_GEMM_WRES"] = arm
    for (n, k) in [(768, 256), (256, 256), (128, 256), (256, 128)]:
        for lb in ("kmaj", "row"):
            a = torch.randn(1, 12544, k, device=dev)
            b = torch.randn(1, n, k, device=dev).transpose(1, 2) if lb == "kmaj" else \
                torch.randn(1, k, n, device=dev)
            bias = torch.randn(n, device=dev)
            for _ in range(5):
                K.bgemm(a, b, mode="bf16", bias=bias)
            torch.cuda.synchronize()
            print(arm, n, k, lb, flush=True)
