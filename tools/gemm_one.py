"""Run one bgemm shape repeatedly (for rocprofv3 PMC passes).

    python tools/gemm_one.py <shape-name> [iters]     (shapes: tools/gemm_bench.py)
"""
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tools")
from gemm_bench import SHAPES  # noqa: E402
from text_guided_face_recognition_amd import kernels as K  # noqa: E402

name = sys.argv[1]
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
nb, m, n, k, la, lb = SHAPES[name]
dev = torch.device("cuda")
a = torch.randn(nb, m, k, device=dev) if la == "row" else torch.randn(nb, k, m, device=dev).transpose(1, 2)
b = torch.randn(nb, k, n, device=dev) if lb == "row" else torch.randn(nb, n, k, device=dev).transpose(1, 2)
ks = K._ksplit(k, nb * -(-m // 64) * -(-n // 64)) if nb == 1 else 1
for _ in range(iters):
    K.bgemm(a, b, mode="bf16", ksplit=ks)
torch.cuda.synchronize()
