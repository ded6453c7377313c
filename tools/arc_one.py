"""Run the fused ArcFace head forward + backward a few times (for rocprofv3)."""
import sys

import torch

sys.path.insert(0, ".")
from text_guided_face_recognition_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
x = torch.randn(64, 256, device=dev, requires_grad=True)
w = torch.randn(4500, 256, device=dev, requires_grad=True)
lab = torch.randint(0, 4500, (64,), device=dev)
for _ in range(5):
    out = K.arc_head(x, w, lab, 30.0, 0.5, mode="bf16")
    out.sum().backward()
torch.cuda.synchronize()
