"""Capture bench.py's config-2 train step (B = 64, T = 30, bf16, one GPU)
with graph debug mode and dump each captured HIP graph as DOT, then print
the cross-branch edges into the word<->region forward (run on the GPU box):
    python tools/graph_dot.py gpurun_out/graph/step"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["TGFR_GRAPH_DOT"] = "1"

from text_guided_face_recognition_amd.config import make_args  # noqa: E402
from text_guided_face_recognition_amd.dist import init_from_env  # noqa: E402
from text_guided_face_recognition_amd.train import (GraphedStep, Train,  # noqa: E402
                                                    synthetic_batch)


def main(prefix):
    os.makedirs(os.path.dirname(prefix), exist_ok=True)
    ctx = init_from_env()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(100)
    tr = Train(make_args(batch_size=64, bert_words_num=32, num_classes=4500,
                         precision="bf16"), dev, ctx)
    batch = synthetic_batch(64, 30, dev, seed=100, bert_hidden=True)
    batch = batch[:-1] + (batch[-1] % 4500,)
    gs = GraphedStep(tr, batch)
    gs.step()
    torch.cuda.synchronize()
    gs.capture.dump(prefix)
    print("dumped", len(gs.capture.graphs), "graph(s) to", prefix)


if __name__ == "__main__":
    main(sys.argv[1])
