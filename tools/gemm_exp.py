"""Time tgfr_bgemm on a few (M, N, K) shapes with torch events (kernel
variants via TGFR_LIB / TGFR_GEMM_CFG in the environment)."""
import sys

import torch

sys.path.insert(0, ".")
from text_guided_face_recognition_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
res = []
for (m, n, k) in [(12544, 128, 32), (12544, 128, 256), (12544, 768, 32), (12544, 768, 256),
                  (12544, 256, 768)]:
    a = torch.randn(1, m, k, device=dev)
    b = torch.randn(1, n, k, device=dev).transpose(1, 2)
    out = torch.empty(1, m, n, device=dev)
    for _ in range(3):
        K.bgemm(a, b, out=out, mode="bf16")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        K.bgemm(a, b, out=out, mode="bf16")
    e1.record()
    torch.cuda.synchronize()
    res.append(f"{m}x{n}x{k}:{e0.elapsed_time(e1) / 20 * 1000:.1f}")
print(" ".join(res), flush=True)
