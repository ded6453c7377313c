"""Worker for tests/test_gpu_dp.py (run under torch.distributed.run).

Each rank owns B_l images, all-gathers nothing itself (the text side is given
globally, as Train.step gathers it), and runs words_loss / sent_loss /
global_loss with args.dist set.  The summed per-rank losses and each rank's
image gradients must equal the single-process global-batch losses and the
matching rows of the global gradient.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from text_guided_face_recognition_amd.config import make_args  # noqa: E402
from text_guided_face_recognition_amd.dist import DistContext, init_from_env  # noqa: E402
from text_guided_face_recognition_amd.models import losses as L  # noqa: E402


def unit(x):
    return x / x.norm(dim=-1, keepdim=True)


def losses(r, img, words, sent, cls, b, args):
    labels = torch.arange(words.shape[0], device=r.device)
    w0, w1, _ = L.words_loss(r, words, labels, None, cls, b, args)
    s0, s1 = L.sent_loss(img, sent, labels, cls, b, args)
    gl = L.global_loss(img, sent, args=args)
    return torch.stack([w0, w1, s0, s1, gl])


def main():
    ctx = init_from_env()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    b_l = 4
    n = b_l * ctx.world
    torch.manual_seed(11)
    r_all = unit(torch.randn(n, 14, 14, 256)).permute(0, 3, 1, 2).to(dev)
    words = unit(torch.randn(n, 22, 256)).to(dev).transpose(1, 2)
    sent = unit(torch.randn(n, 256)).to(dev)
    img_all = torch.randn(n, 256).to(dev)
    cls = torch.tensor([3, 1, 3, 7, 1, 9, 3, 0][:n], device=dev)
    args = make_args(bert_words_num=24, precision="fp32", return_att_maps=False)

    # single-process global reference on this rank
    rg = r_all.clone().requires_grad_()
    ig = img_all.clone().requires_grad_()
    ref = losses(rg, ig, words, sent, cls, n, args)
    ref.sum().backward()

    # this rank's share
    ctx.set_batch(b_l)
    args.dist = ctx
    rows = slice(ctx.row_offset, ctx.row_offset + b_l)
    rl = r_all[rows].clone().requires_grad_()
    il = img_all[rows].clone().requires_grad_()
    mine = losses(rl, il, words, sent, cls, b_l, args)
    mine.sum().backward()
    tot = ctx.sum(mine.detach())
    torch.cuda.synchronize()
    err_loss = (tot - ref.detach()).abs().max().item()
    err_r = ((rl.grad - rg.grad[rows]).abs().max() / rg.grad.abs().max()).item()
    err_i = ((il.grad - ig.grad[rows]).abs().max() / ig.grad.abs().max()).item()
    res = {"rank": ctx.rank, "err_loss": err_loss, "err_r": err_r, "err_i": err_i}
    out = os.environ.get("TGFR_DP_OUT")
    if out:
        with open(f"{out}.{ctx.rank}", "w") as f:
            json.dump(res, f)
    ok = err_loss < 1e-4 and err_r < 1e-4 and err_i < 1e-4
    sys.exit(0 if ok else 3)


if __name__ == "__main__":
    main()
