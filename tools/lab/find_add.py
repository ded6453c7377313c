"""Lab (GPU): list the aten ops that torch itself launches inside one eager
bench step (config 2, bf16) -- shapes, and the autograd node they ran under --
to find framework-side kernels (gradient accumulation adds, fills) in the step."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from text_guided_face_recognition_amd import train as T  # noqa: E402
from text_guided_face_recognition_amd.config import make_args  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    args = make_args(batch_size=64, num_classes=4500, precision="bf16", bert_words_num=32)
    tr = T.Train(args, dev)
    batch = T.synthetic_batch(64, 30, dev, seed=1, n_ids=4500, bert_hidden=True)
    for _ in range(3):
        tr.step(batch)
    torch.cuda.synchronize()
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU], record_shapes=True) as prof:
        tr.step(batch)
        torch.cuda.synchronize()
    for e in prof.events():
        if e.name in ("aten::add", "aten::add_", "aten::fill_", "aten::zero_", "aten::copy_",
                      "aten::mul", "aten::sum", "aten::cat", "aten::zeros", "aten::clone"):
            print(e.name, e.input_shapes, "| seq", e.sequence_nr, "| fwd_thread", e.fwd_thread,
                  "| stack-parent", e.cpu_parent.name if e.cpu_parent else None, flush=True)


if __name__ == "__main__":
    main()
