"""Time TextHeading (tgfr_text_heading) on the GPU vs the CPU oracle.

    python tools/text_bench.py [--b 64] [--L 32]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from text_guided_face_recognition_amd import _hip  # noqa: E402
from text_guided_face_recognition_amd.config import make_args  # noqa: E402
from text_guided_face_recognition_amd.models.models import TextHeading  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--b", type=int, default=64)
ap.add_argument("--L", type=int, default=32)
ap.add_argument("--reps", type=int, default=50)
a = ap.parse_args()
for prec in ("bf16", "fp32"):
    net = TextHeading(make_args(bert_words_num=a.L, precision=prec)).cuda()
    x = torch.randn(a.b, a.L - 1, 768, device="cuda")
    with torch.no_grad():
        for _ in range(3):
            net(x)
        torch.cuda.synchronize()
        with _hip.KernelTimer(replay=("tgfr_text_heading",), reps=a.reps) as kt:
            net(x)
        ms = kt.replayed["tgfr_text_heading"]
    flop = sum(2 * a.b * (a.L - 1 - k + 1) * 256 * k * 768 for k in (2, 3, 4))
    byts = a.b * (a.L - 1) * 768 * 4 + 256 * 9 * 768 * 4 + a.b * (a.L - 1) * 256 * 4
    print(f"{prec} B={a.b} L={a.L}: {ms * 1e3:.1f} us/call, {flop / ms / 1e9:.1f} TFLOP/s, "
          f"{a.b / ms * 1e3:.0f} captions/s, alg bytes {byts / 1e6:.1f} MB")
