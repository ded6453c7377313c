"""How long the HOST takes to enqueue one replay of the config-2 step graph
(bench.py's GraphedStep, B = 64, T = 30, bf16), against the GPU time per
step: if the enqueue rate is close to the step rate, node submission -- not
the kernels -- paces the step (run on the GPU box):
    python tools/replay_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from text_guided_face_recognition_amd.config import make_args  # noqa: E402
from text_guided_face_recognition_amd.dist import init_from_env  # noqa: E402
from text_guided_face_recognition_amd.train import (GraphedStep, Train,  # noqa: E402
                                                    synthetic_batch)


def main():
    ctx = init_from_env()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(100)
    tr = Train(make_args(batch_size=64, bert_words_num=32, num_classes=4500,
                         precision=os.environ.get("PREC", "bf16")), dev, ctx)
    batch = synthetic_batch(64, 30, dev, seed=100, bert_hidden=True)
    batch = batch[:-1] + (batch[-1] % 4500,)
    gs = GraphedStep(tr, batch)
    for _ in range(10):
        gs.step()
    torch.cuda.synchronize()
    n = 50
    # host enqueue time per replay, the GPU far behind (the queue fills)
    t0 = time.perf_counter()
    for _ in range(n):
        gs.capture.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    # one replay at a time: enqueue, then wait
    lat = []
    for _ in range(20):
        a = time.perf_counter()
        gs.capture.replay()
        b = time.perf_counter()
        torch.cuda.synchronize()
        lat.append((b - a, time.perf_counter() - a))
    enq = sorted(x[0] for x in lat)[10] * 1e6
    tot = sorted(x[1] for x in lat)[10] * 1e6
    print(f"back-to-back: host enqueue {(t1 - t0) / n * 1e6:.1f} us/replay, "
          f"GPU-bound total {(t2 - t0) / n * 1e6:.1f} us/replay")
    print(f"isolated replay: enqueue {enq:.1f} us, enqueue -> done {tot:.1f} us (median)")


if __name__ == "__main__":
    main()
