"""Worker for tests/test_gpu_dp.py::test_dp_graphed_train_step (run under
torch.distributed.run, gloo transport so both ranks share one GPU).

Each rank builds the stage-1 trainer from a DIFFERENT seed (the trainer
broadcasts rank 0's parameters) and its own batch.  One copy steps eagerly,
one through GraphedStep (graphs cut at the collectives, dist.StepCapture);
after the same number of steps both copies must agree, and every rank must
hold the same parameters (the gradient all-reduce keeps the replicas equal).
With the forked DP step, one step of it is also held against the linear DP
step (TGFR_FORK=0 semantics) on the same seed and per-rank batch.
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


def oracle_dp_step(tr, parts, args, nw):
    """The reference's stage-1 step (src/train_encoders_bert.py:254-331) on the
    oracle as its nn.DataParallel runs it over the ranks' batches: the image
    head per replica (IMIM's BatchNorm takes each replica's batch statistics,
    models/models.py:394 -- DataParallel does not synchronise them), the
    losses over the gathered global batch (:146-169)."""
    from oracle import tgfr_oracle as O
    from test_gpu_step_parity import HEAD_KEYS, _cpu_params
    hp = _cpu_params(tr.image_head, HEAD_KEYS)
    arc_i = tr.image_cls.weight.detach().cpu().clone().requires_grad_()
    arc_t = tr.text_cls.weight.detach().cpu().clone().requires_grad_()
    heads = [O.image_heading(p[0].cpu(), p[1].cpu(), hp) for p in parts]
    gp = torch.cat([h[0] for h in heads])
    r = torch.cat([h[1] for h in heads])
    wc, sc, cc = (torch.cat([p[i].cpu() for p in parts]) for i in (2, 3, 4))
    b = gp.shape[0]
    labels = torch.arange(b)
    w0, w1, _, _ = O.words_loss(r, wc, labels, None, nw, 4.0, 5.0, 10.0)
    s0, s1, _ = O.sent_loss(gp, sc, labels, cc.numpy(), 10.0)
    tid = O.focal_loss(O.arc_margin(sc, arc_t, cc, s=35), cc)
    iid = O.focal_loss(O.arc_margin(gp, arc_i, cc, s=30), cc)
    cl, _ = O.global_loss(gp, sc)
    total = w0 + w1 + s0 + s1 + args.lambda_id * (tid + iid) + args.lambda_clip * cl
    total.backward()
    return ({k: v.grad.clone() for k, v in hp.items()},
            {"damsm": (w0 + w1 + s0 + s1).item(), "clip": cl.item(),
             "ident": args.lambda_id * (tid + iid).item()})


def oracle_check(ctx, build, dev, res):
    """One forked DP step against the oracle's DataParallel step over BOTH
    ranks' batches (oracle_dp_step), from the same weights: the contrastive
    losses summed over ranks (each rank holds its rows' share), the identity
    term (formed from the global mean CE on every rank) and every reduced head
    gradient."""
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
    from test_gpu_step_parity import HEAD_KEYS
    tr = build()
    parts = [synthetic_batch(8, 22, dev, seed=40 + r, n_ids=200) for r in range(ctx.world)]
    grads, groups = oracle_dp_step(tr, parts, tr.args, 22)
    out = tr.step(parts[ctx.rank])
    torch.cuda.synchronize()
    mine = torch.tensor([out[k].item() for k in ("damsm", "clip", "ident")])
    tot = mine.clone()
    dist.all_reduce(tot, group=ctx.group)
    res["oracle_groups"] = [tot[0].item(), tot[1].item(), mine[2].item()]
    res["oracle_groups_ref"] = [groups[k] for k in ("damsm", "clip", "ident")]
    res["oracle_err_loss"] = max(abs(a - b_) for a, b_ in zip(res["oracle_groups"],
                                                               res["oracle_groups_ref"]))
    named = dict(tr.image_head.named_parameters())
    g_all = max(x.abs().max().item() for x in grads.values())
    err = 0.0
    for k, v in HEAD_KEYS.items():
        if named[k].grad is None:     # (no path from the losses: the oracle's is 0)
            assert grads[v].abs().max().item() == 0.0, k
            continue
        e = (named[k].grad.detach().cpu() - grads[v]).abs().max().item()
        err = max(err, e / (grads[v].abs().max().item() + 1e-3 * g_all))
    res["oracle_err_grad"] = err
    return res["oracle_err_loss"] < 1e-3 * max(1.0, abs(res["oracle_groups_ref"][2])) \
        and err < 5e-3


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
    ok = err_out < 1e-4 and err_par < 1e-5 and err_rank == 0.0
    if graphed._side is not None:
        # the forked DP step (Train._step_forked_dp: gathered partials read per
        # rank at a row stride, row_offset > 0 on rank 1, each rank its own
        # batch) against the linear DP step on the same seed and batch: one
        # step each from the same parameters -- equal losses and reduced
        # gradients on every rank
        forked, linear = build(), build()
        linear._side = None
        o_f, o_l = forked.step(batch), linear.step(batch)
        torch.cuda.synchronize()
        res["lin_err_out"] = max(abs(o_f[k].item() - o_l[k].item()) for k in o_f)
        pairs = [(a.grad, b.grad) for a, b in zip(forked.params, linear.params)
                 if b.grad is not None]
        assert all(a is not None for a, _ in pairs)
        gscale = max(b.abs().max().item() for _, b in pairs)
        res["lin_err_grad"] = max((a - b).abs().max().item() for a, b in pairs) / gscale
        ok = ok and res["lin_err_out"] < 1e-4 and res["lin_err_grad"] < 2e-3
        if precision == "fp32" and not bert:
            ok = ok and oracle_check(ctx, build, dev, res)
    out = os.environ.get("TGFR_DP_OUT")
    if out:
        with open(f"{out}.{ctx.rank}", "w") as f:
            json.dump(res, f)
    sys.exit(0 if ok else 3)


if __name__ == "__main__":
    main()
