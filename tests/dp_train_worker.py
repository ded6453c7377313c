"""Worker for tests/test_gpu_dp.py::test_dp_graphed_train_step (run under
torch.distributed.run, gloo transport so both ranks share one GPU).

Each rank builds the stage-1 trainer from a DIFFERENT seed (the trainer
broadcasts rank 0's parameters) and its own batch.  One copy steps eagerly,
one through GraphedStep (graphs cut at the collectives, dist.StepCapture);
after the same number of steps both copies must agree, and every rank must
hold the same parameters (the gradient all-reduce keeps the replicas equal).
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from text_guided_face_recognition_amd.config import make_args  # noqa: E402
from text_guided_face_recognition_amd.dist import all_gather_cat, init_from_env  # noqa: E402
from text_guided_face_recognition_amd.train import (GraphedStep, Train,  # noqa: E402
                                                    synthetic_batch)


def main():
    ctx = init_from_env()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    precision = os.environ.get("TGFR_DP_PRECISION", "fp32")

    def build():
        torch.manual_seed(7 + ctx.rank)
        args = make_args(batch_size=8, num_classes=200, precision=precision,
                         bert_words_num=24)
        return Train(args, dev, ctx)

    bert = os.environ.get("TGFR_DP_BERT", "0") == "1"
    batch = synthetic_batch(8, 22, dev, seed=40 + ctx.rank, n_ids=200, bert_hidden=bert)
    eager, graphed = build(), build()
    outs_e = [eager.step(batch) for _ in range(5)]
    gs = GraphedStep(graphed, tuple(t.clone() for t in batch), warmup=3)
    gs.step()
    out_g = {k: v.clone() for k, v in gs.step().items()}
    torch.cuda.synchronize()
    err_out = max((out_g[k] - outs_e[-1][k]).abs().max().item() for k in out_g)
    err_par = max((a - b).abs().max().item()
                  for a, b in zip(graphed.params, eager.params))
    # replicas identical across ranks
    flat = torch.cat([p.detach().reshape(-1) for p in graphed.params +
                      list(graphed.text_head.parameters())]).unsqueeze(0)
    allp = all_gather_cat(flat, ctx.group)
    err_rank = (allp[0] - allp[1]).abs().max().item()
    res = {"rank": ctx.rank, "segments": len(gs.capture.graphs), "err_out": err_out,
           "err_par": err_par, "err_rank": err_rank}
    out = os.environ.get("TGFR_DP_OUT")
    if out:
        with open(f"{out}.{ctx.rank}", "w") as f:
            json.dump(res, f)
    ok = err_out < 1e-4 and err_par < 1e-5 and err_rank == 0.0
    sys.exit(0 if ok else 3)


if __name__ == "__main__":
    main()
