"""Worker for tests/test_gpu_dp.py (run under torch.distributed.run).

Each rank owns B_l images, all-gathers nothing itself (the text side is given
globally, as Train.step gathers it), and runs words_loss / sent_loss /
global_loss with args.dist set.  The summed per-rank losses and each rank's
image gradients must equal (1) the reference restatement's global-batch
losses and gradients (oracle/tgfr_oracle.py, CPU fp32: 1e-3 on losses, 2e-3
of scale on gradients) and (2) the single-process HIP global-batch result
(1e-4).
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from text_guided_face_recognition_amd.config import make_args  # noqa: E402
from text_guided_face_recognition_amd.dist import DistContext, init_from_env  # noqa: E402
from text_guided_face_recognition_amd.models import losses as L  # noqa: E402
from oracle import tgfr_oracle as O  # noqa: E402


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

    # the oracle's global batch (the reference's DataParallel losses, CPU)
    ro = r_all.cpu().clone().requires_grad_()
    io = img_all.cpu().clone().requires_grad_()
    lab = torch.arange(n)
    ow0, ow1, _, _ = O.words_loss(ro, words.cpu(), lab, None, 22, 4.0, 5.0, 10.0)
    os0, os1, _ = O.sent_loss(io, sent.cpu(), lab, cls.cpu().numpy(), 10.0)
    ogl, _ = O.global_loss(io, sent.cpu())
    oref = torch.stack([ow0, ow1, os0, os1, ogl])
    oref.sum().backward()

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
    orows = slice(ctx.row_offset, ctx.row_offset + b_l)
    # identity head under DP: the focal factor of the GLOBAL mean CE
    # (losses.py:313-325 on DataParallel's gathered batch), two heads, one
    # all-reduce; per-rank logit gradients are rows of the global gradient
    from text_guided_face_recognition_amd import kernels as K
    torch.manual_seed(12)
    lg = [torch.randn(n, 37) * 3, torch.randn(n, 37) * 5]
    tg = torch.tensor([5, 1, 36, 7, 1, 9, 3, 0][:n])
    lo = [x.clone().requires_grad_() for x in lg]
    fo = [O.focal_loss(x, tg) for x in lo]
    (fo[0] + 3 * fo[1]).backward()
    ll = [x[orows].to(dev).clone().requires_grad_() for x in lg]
    f0, f1 = K.focal_ce_multi([(ll[0], tg[orows].to(dev)), (ll[1], tg[orows].to(dev))], 2.0,
                              ctx.group, n)
    (f0 + 3 * f1).backward()
    ferr = max(abs(f0.item() - fo[0].item()), abs(f1.item() - fo[1].item()))
    fgerr = max(((a.grad.cpu() - b.grad[orows]).abs().max() / b.grad.abs().max()).item()
                for a, b in zip(ll, lo))
    oerr_loss = (tot.cpu() - oref.detach()).abs().max().item()
    oerr_r = ((rl.grad.cpu() - ro.grad[orows]).abs().max() / ro.grad.abs().max()).item()
    oerr_i = ((il.grad.cpu() - io.grad[orows]).abs().max() / io.grad.abs().max()).item()
    # bf16 with the text side gathered as the word<->region operand rows
    # (Train._gather_text: bf16 rows + norms, half the fp32 words' bytes):
    # each rank prepares its own captions' rows (as TextHeading attaches them),
    # one all-gather, rows-only words; the DP losses and this rank's region
    # gradient equal the single-process bf16 global batch on the same rows,
    # and the oracle within the bf16 mode's tolerance
    bargs = make_args(bert_words_num=24, precision="bf16", return_att_maps=False)
    wb = words.transpose(1, 2).contiguous()                       # [n, 22, 256]
    rows_all, _, norms_all = K.prep_rows(wb, 22, 32, want_norms=True, scale=K.LOG2E)
    K.attach_rows(wb, rows_all, norms_all, False, K.LOG2E)
    labels = torch.arange(n, device=dev)
    rgb = r_all.clone().requires_grad_()
    bref = torch.stack(L.words_loss(rgb, wb.transpose(1, 2), labels, None, cls, n, bargs)[:2])
    bref.sum().backward()
    rows_l, _, norms_l = K.prep_rows(wb[rows], 22, 32, want_norms=True, scale=K.LOG2E)
    rows_g, norms_g = ctx.gather_text(rows_l, norms_l)
    wro = K.rows_only_words(rows_g, norms_g, 22, False)
    bargs.dist = ctx
    rlb = r_all[rows].clone().requires_grad_()
    bmine = torch.stack(L.words_loss(rlb, wro, labels, None, cls, b_l, bargs)[:2])
    bmine.sum().backward()
    btot = ctx.sum(bmine.detach())
    torch.cuda.synchronize()
    rows_err_loss = (btot - bref.detach()).abs().max().item()
    rows_err_r = ((rlb.grad - rgb.grad[rows]).abs().max() / rgb.grad.abs().max()).item()
    rows_oerr_loss = (btot.cpu() - oref[:2].detach()).abs().max().item()
    rows_oerr_r = ((rlb.grad.cpu() - ro.grad[orows]).abs().max() / ro.grad.abs().max()).item()
    # (the oracle gradient above is of all five losses; compare the word terms' own)
    ro2 = r_all.cpu().clone().requires_grad_()
    w0o, w1o, _, _ = O.words_loss(ro2, words.cpu(), torch.arange(n), None, 22, 4.0, 5.0, 10.0)
    (w0o + w1o).backward()
    rows_oerr_r = ((rlb.grad.cpu() - ro2.grad[orows]).abs().max() / ro2.grad.abs().max()).item()
    res = {"rank": ctx.rank, "err_loss": err_loss, "err_r": err_r, "err_i": err_i,
           "oracle_err_loss": oerr_loss, "oracle_err_r": oerr_r, "oracle_err_i": oerr_i,
           "focal_err": ferr, "focal_grad_err": fgerr, "rows_err_loss": rows_err_loss,
           "rows_err_r": rows_err_r, "rows_oracle_err_loss": rows_oerr_loss,
           "rows_oracle_err_r": rows_oerr_r,
           "rows_bytes_per_caption": rows_l[0].numel() * 2 + norms_l[0].numel() * 4,
           "words_bytes_per_caption": 22 * 256 * 4}
    out = os.environ.get("TGFR_DP_OUT")
    if out:
        with open(f"{out}.{ctx.rank}", "w") as f:
            json.dump(res, f)
    ok = err_loss < 1e-4 and err_r < 1e-4 and err_i < 1e-4 and oerr_loss < 1e-3 and \
        oerr_r < 2e-3 and oerr_i < 2e-3 and ferr < 1e-5 and fgerr < 1e-5 and \
        rows_err_loss < 1e-4 and rows_err_r < 1e-4 and rows_oerr_loss < 5e-2 and \
        rows_oerr_r < 3e-2
    sys.exit(0 if ok else 3)


if __name__ == "__main__":
    main()
