"""Time the stage-2 FCFM train step (BASELINE configs[3]: Working + ImageHeading
+ ArcMargin(640) + focal, B = 256 per GPU, L = 24 -> T = 22) on one GPU.

    python tools/fcfm_bench.py [--batch 256] [--words 24] [--steps 20] [--eager]

Prints one JSON line: samples/s of the graph-replayed step and the per-ABI-call
HIP-event timings of an eager pass (library kernels only; torch-native ops of
the step are the remainder of ms_per_step).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from text_guided_face_recognition_amd._hip import KernelTimer  # noqa: E402
from text_guided_face_recognition_amd.config import make_args  # noqa: E402
from text_guided_face_recognition_amd.train import Fusion, GraphedStep, synthetic_batch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--words", type=int, default=24)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
ap.add_argument("--eager", action="store_true")
a = ap.parse_args()

dev = torch.device("cuda", 0)
torch.manual_seed(100)
tr = Fusion(make_args(batch_size=a.batch, bert_words_num=a.words, num_classes=4500,
                      precision=a.precision), dev)
batch = synthetic_batch(a.batch, a.words - 2, dev, seed=100)
batch = batch[:4] + (batch[4] % 4500,)
with KernelTimer() as kt:
    for _ in range(3):
        tr.step(batch)
prof = kt.summary()
runner = tr if a.eager else GraphedStep(tr, batch)
for _ in range(a.warmup):
    runner.step(batch)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.steps):
    runner.step(batch)
torch.cuda.synchronize()
el = time.perf_counter() - t0
print(json.dumps({
    "workload": "FCFM stage-2 train step (BASELINE configs[3]) on one GPU",
    "batch": a.batch, "words_per_caption": a.words - 2, "precision": a.precision,
    "launch": "eager" if a.eager else "hip-graph",
    "value": round(a.batch * a.steps / el, 1), "unit": "samples/s",
    "ms_per_step": round(el / a.steps * 1e3, 4),
    "eager_entry_ms": {k: round(v[1], 4) for k, v in sorted(prof.items())}}), flush=True)
