"""Time the fused ArcFace head forward / backward launches at a few shapes
(also usable under rocprofv3).

    python tools/arc_one.py [B D C ...]   (default: the stage-1 and stage-2 shapes)
"""
import sys

import torch

sys.path.insert(0, ".")
from text_guided_face_recognition_amd import _hip  # noqa: E402
from text_guided_face_recognition_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
shapes = [(64, 256, 4500), (256, 256, 4500), (64, 640, 4500), (256, 640, 4500)]
if len(sys.argv) > 3:
    v = [int(a) for a in sys.argv[1:]]
    shapes = [tuple(v[i:i + 3]) for i in range(0, len(v) - 2, 3)]
for b, d, c in shapes:
    x = torch.randn(b, d, device=dev, requires_grad=True)
    w = torch.randn(c, d, device=dev, requires_grad=True)
    lab = torch.randint(0, c, (b,), device=dev)
    for _ in range(3):
        K.arc_head(x, w, lab, 30.0, 0.5, mode="bf16").sum().backward()
    torch.cuda.synchronize()
    with _hip.KernelTimer(replay=("tgfr_arc_fwd", "tgfr_arc_bwd"), reps=20) as kt:
        K.arc_head(x, w, lab, 30.0, 0.5, mode="bf16").sum().backward()
    torch.cuda.synchronize()
    f, bw = kt.replayed["tgfr_arc_fwd"], kt.replayed["tgfr_arc_bwd"]
    flop = 2 * b * c * d
    print(f"B={b} D={d} C={c}: fwd {f * 1e3:.1f} us ({flop / f / 1e9:.1f} TFLOP/s), "
          f"bwd {bw * 1e3:.1f} us ({flop / bw / 1e9:.1f} TFLOP/s)", flush=True)
