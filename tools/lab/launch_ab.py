"""Launch schemes of the stage-1 step on one GPU (config 2 shape): graph
replay vs eager; wall time per step (host clock around N replays,
synchronised) and GPU time per step (HIP events around the same replays).
(Round 2 also timed the loss branches forked onto side streams inside the
graph: 0.694 ms/step against 0.665 for the linear graph.)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from text_guided_face_recognition_amd import train as T  # noqa: E402
from text_guided_face_recognition_amd.config import make_args  # noqa: E402

dev = torch.device("cuda", 0)
batch = T.synthetic_batch(64, 30, dev, seed=101)
batch = batch[:4] + (batch[4] % 4500,)


def build():
    torch.manual_seed(100)
    return T.Train(make_args(batch_size=64, bert_words_num=32, num_classes=4500,
                             precision="bf16"), dev)


def timeit(step, n=30):
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(n):
        step()
    e1.record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / n * 1e3
    return wall, e0.elapsed_time(e1) / n


for mode in ("graph", "eager"):
    tr = build()
    if mode == "eager":
        w, g = timeit(lambda: tr.step(batch))
    else:
        gs = T.GraphedStep(tr, batch)
        w, g = timeit(gs.step)
    print(f"{mode:9s} wall {w:.4f} ms/step  gpu {g:.4f} ms/step", flush=True)
