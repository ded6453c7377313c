"""Calibrate the CPU oracle against the reference's own CPU timings
(measured by importing the reference in the survey
container, 8 cores, torch 2.10 CPU fp32): words_loss fwd+bwd at B=64, T=30
(470 ms) and Working (FCFM) fwd+bwd at B=256 (124 ms); the restatement must land
within +-15 %.  Median of 3 after 1 warm-up, as BASELINE.md's protocol.

    python tools/calibrate_oracle.py [--threads 8]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import tgfr_oracle as O  # noqa: E402

REF_MS = {"words_loss_b64_t30": 470.0, "working_b256": 124.0}


def med(fn, reps=3):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2] * 1000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    torch.manual_seed(100)
    unit = lambda x: x / x.norm(dim=-1, keepdim=True)  # noqa: E731
    b, nw = 64, 30
    r = unit(torch.randn(b, 14, 14, 256)).permute(0, 3, 1, 2).contiguous().requires_grad_()
    w = unit(torch.randn(b, nw, 256)).transpose(1, 2)
    labels = torch.arange(b)

    def words():
        r.grad = None
        w0, w1, _, _ = O.words_loss(r, w, labels, None, nw, 4.0, 5.0, 10.0)
        (w0 + w1).backward()

    # Working (FCFM) at B = 256, its parameters as the drop-in module makes them
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "tests"))
    from test_gpu_step_parity import WORKING_KEYS, _cpu_params
    from text_guided_face_recognition_amd.models.fusion_nets import Working
    bw = 256
    p = _cpu_params(Working(256).train(), WORKING_KEYS)
    img = unit(torch.randn(bw, 14, 14, 256)).permute(0, 3, 1, 2).contiguous().requires_grad_()
    word = torch.randn(bw, 256, 22)
    gl, sent = torch.randn(bw, 256), torch.randn(bw, 256)

    def working():
        img.grad = None
        for v in p.values():
            v.grad = None
        O.working(img, word, gl, sent, p).sum().backward()

    res = {"threads": a.threads, "cpu": os.cpu_count(), "torch": torch.__version__}
    for name, fn in (("words_loss_b64_t30", words), ("working_b256", working)):
        ms = med(fn)
        res[name] = {"oracle_ms": round(ms, 1), "reference_ms": REF_MS[name],
                     "ratio": round(ms / REF_MS[name], 3),
                     "within_15pct": abs(ms / REF_MS[name] - 1) <= 0.15}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
