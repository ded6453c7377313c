"""Whole-step parity: one train step of the drop-in trainers (fp32 parity mode)
against the CPU oracle's restatement of the reference's step on the SAME
weights and batch.

  Train      src/train_encoders_bert.py:254-331   (7 loss terms, Adam head + SGD classifiers)
  TrainLSTM  src/train_encoders_lstm.py:236-305   (w0 + w1 + 100 (tid + iid) + ClipLoss;
             text side from the reference's own words_loss_lstm_b5 fixture)
  Fusion     src/fusion_bert.py:205-243           (Working -> ArcMargin(640) -> focal)

Checked: every loss term within 1e-3 absolute; every head parameter's
gradient within 5e-3 of its largest reference gradient; the parameters after
the optimiser step.  SGD updates are linear in the gradient: relative 1e-4 of
the tensor's scale.  Adam's first update is lr * g / (|g| + eps), i.e. +-lr
for every element whose gradient is not ~0 -- a sign decision -- so it is
compared where the reference gradient exceeds 4x the measured gradient error
(the sign cannot flip) at 1e-4 relative, and everywhere within 2 lr.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden, t
from oracle import tgfr_oracle as O

pytestmark = pytest.mark.gpu

HEAD_KEYS = {
    "project_global.projection.weight": "pg_w", "project_global.projection.bias": "pg_b",
    "imim.project_local.projection.weight": "pl_w", "imim.project_local.projection.bias": "pl_b",
    "imim.bn_img.weight": "bn_w", "imim.bn_img.bias": "bn_b",
    "imim.sa.query_proj.weight": "sa_q_w", "imim.sa.query_proj.bias": "sa_q_b",
    "imim.sa.key_proj.weight": "sa_k_w", "imim.sa.key_proj.bias": "sa_k_b",
    "imim.sa.value_proj.weight": "sa_v_w", "imim.sa.value_proj.bias": "sa_v_b",
    "imim.conv1x1_1.weight": "c1_w", "imim.conv1x1_1.bias": "c1_b",
    "imim.conv1x1_2.weight": "c2_w", "imim.conv1x1_2.bias": "c2_b",
    "imim.ln.weight": "ln_w", "imim.ln.bias": "ln_b",
}
WORKING_KEYS = {
    "conv.weight": "conv_w", "conv.bias": "conv_b", "bn_img.weight": "bn_img_w",
    "bn_img.bias": "bn_img_b", "bn_word.weight": "bn_word_w", "bn_word.bias": "bn_word_b",
    "projection.weight": "proj_w", "projection.bias": "proj_b",
    "sa.query_proj.weight": "sa_q_w", "sa.query_proj.bias": "sa_q_b",
    "sa.key_proj.weight": "sa_k_w", "sa.key_proj.bias": "sa_k_b",
    "sa.value_proj.weight": "sa_v_w", "sa.value_proj.bias": "sa_v_b",
    "ln.weight": "ln_w", "ln.bias": "ln_b", "linear.weight": "lin_w", "linear.bias": "lin_b",
    "ln_gl_image.weight": "ln_g_w", "ln_gl_image.bias": "ln_g_b",
    "ln_sent.weight": "ln_s_w", "ln_sent.bias": "ln_s_b",
}


def _cpu_params(module, keys):
    named = dict(module.named_parameters())
    return {v: named[k].detach().cpu().clone().requires_grad_() for k, v in keys.items()}


def _check_adam(param, old, ref_new, grad, lr, name="", g_all=0.0, wd=0.0):
    """Gradient and first Adam update of one parameter against the oracle.

    The gradient (p.grad after the step) must be within 5e-3 of the tensor's
    largest reference gradient (the IMIM q/k projections reach ~4e-3: their
    gradient runs through the 196-wide attention softmax backward), plus
    1e-5 of the largest gradient of the whole head (g_all) -- a floor for
    tensors whose exact gradient is zero, such as the key-role bias, which
    the attention softmax cancels.  Adam's
    first update is lr * g / (|g| + 1e-8), i.e. +-lr: a sign decision, so it
    is compared (1e-4 of the tensor's scale) where |g_ref| exceeds 4x the
    measured gradient error and Adam's eps (with the weight decay term
    added: g + wd p), where the sign cannot flip; and
    everywhere it must stay within 2 lr."""
    new = param.detach().cpu()
    g_mine = param.grad.detach().cpu()
    g_err = (g_mine - grad).abs().max().item()
    g_scale = grad.abs().max().item()
    assert g_err <= 5e-3 * g_scale + 1e-5 * g_all + 1e-12, (
        f"{name}: gradient error {g_err:.3e} = {g_err / g_scale:.3e} of max {g_scale:.3e}")
    d_mine, d_ref = new - old, ref_new - old
    assert (d_mine - d_ref).abs().max().item() <= 2 * lr + 1e-7, name
    # the update's sign follows g + wd p (Adam's L2 weight decay)
    sure = (grad + wd * old).abs() > max(4 * g_err, 1e-6)
    scale = old.abs().max().clamp(min=1e-3)
    diff = (d_mine - d_ref).abs() * sure
    err = diff.max() / scale
    if err.item() >= 1e-4:
        i = int(diff.argmax())
        raise AssertionError(f"{name}: update error {err.item():.3e} of scale at element {i}: "
                             f"ref grad {grad.flatten()[i].item():.3e} (max {g_scale:.3e}), "
                             f"d_mine {d_mine.flatten()[i]:.3e}, d_ref {d_ref.flatten()[i]:.3e}")


def _check_sgd(new, ref_new):
    scale = ref_new.abs().max().clamp(min=1e-6)
    err = ((new - ref_new).abs().max() / scale).item()
    assert err < 1e-4, err


def _bert_trainer(dev, b, nw, seed, n_ids):
    from text_guided_face_recognition_amd.config import make_args
    from text_guided_face_recognition_amd.train import Train, synthetic_batch
    torch.manual_seed(seed)
    args = make_args(batch_size=b, bert_words_num=nw + 2, num_classes=n_ids, precision="fp32")
    tr = Train(args, dev)
    batch = synthetic_batch(b, nw, dev, seed=seed + 1, n_ids=n_ids)
    return tr, batch, args


@pytest.mark.parametrize("b,nw,n_ids", [(8, 22, 5), (16, 30, 200)])
def test_train_step_matches_oracle(gpu, b, nw, n_ids):
    """Stage-1 BERT step: duplicate class ids (n_ids = 5) exercise the
    sent_loss same-class mask."""
    tr, batch, args = _bert_trainer(gpu, b, nw, 31 + b, n_ids)
    g, local, words, sent, cls = batch
    hp = _cpu_params(tr.image_head, HEAD_KEYS)
    arc_i = tr.image_cls.weight.detach().cpu().clone().requires_grad_()
    arc_t = tr.text_cls.weight.detach().cpu().clone().requires_grad_()
    old = {k: v.detach().clone() for k, v in hp.items()}
    old_i, old_t = arc_i.detach().clone(), arc_t.detach().clone()

    # the oracle step (train_encoders_bert.py:254-331)
    gc, lc, wc, sc, cc = (x.cpu() for x in batch)
    labels = torch.arange(b)
    gp, r = O.image_heading(gc, lc, hp)
    w0, w1, _, _ = O.words_loss(r, wc, labels, None, nw, 4.0, 5.0, 10.0)
    s0, s1, _ = O.sent_loss(gp, sc, labels, cc.numpy(), 10.0)
    tid = O.focal_loss(O.arc_margin(sc, arc_t, cc, s=35), cc)
    iid = O.focal_loss(O.arc_margin(gp, arc_i, cc, s=30), cc)
    cl, _ = O.global_loss(gp, sc)
    total = w0 + w1 + s0 + s1 + args.lambda_id * (tid + iid) + args.lambda_clip * cl
    total.backward()
    grads = {k: v.grad.clone() for k, v in hp.items()}
    torch.optim.Adam(list(hp.values()), lr=args.lr_head, betas=(0.5, 0.999)).step()
    torch.optim.SGD([arc_i, arc_t], lr=0.1, momentum=0.9, weight_decay=5e-5).step()

    out = tr.step(batch)
    torch.cuda.synchronize()
    ref = {"damsm": (w0 + w1 + s0 + s1).item(), "clip": cl.item(),
           "ident": args.lambda_id * (tid + iid).item()}
    for k, v in ref.items():
        # ident is 100 x (two focal losses): 1e-3 on each focal term
        tol = 1e-3 * (2 * args.lambda_id if k == "ident" else 1)
        assert abs(out[k].item() - v) < tol, (k, out[k].item(), v)
    named = dict(tr.image_head.named_parameters())
    for k, v in HEAD_KEYS.items():
        _check_adam(named[k], old[v], hp[v].detach(), grads[v], args.lr_head, k,
                    max(x.abs().max().item() for x in grads.values()))
    _check_sgd(tr.image_cls.weight.detach().cpu(), arc_i.detach())
    _check_sgd(tr.text_cls.weight.detach().cpu(), arc_t.detach())
    assert not torch.equal(tr.image_cls.weight.detach().cpu(), old_i)
    assert not torch.equal(tr.text_cls.weight.detach().cpu(), old_t)


def test_train_step_each_loss_term(gpu):
    """The 7 loss terms of one stage-1 step individually (the trainer reports
    their weighted groups; this recomputes them through the drop-in API on
    the trainer's own head output)."""
    from text_guided_face_recognition_amd.models import losses as L
    b, nw = 12, 30
    tr, batch, args = _bert_trainer(gpu, b, nw, 77, 4)
    g, local, words, sent, cls = batch
    hp = _cpu_params(tr.image_head, HEAD_KEYS)
    arc_i = tr.image_cls.weight.detach().cpu()
    arc_t = tr.text_cls.weight.detach().cpu()
    labels = torch.arange(b)
    gc, lc, wc, sc, cc = (x.cpu() for x in batch)
    gp, r = O.image_heading(gc, lc, hp)
    ref = list(O.words_loss(r, wc, labels, None, nw, 4.0, 5.0, 10.0)[:2])
    ref += list(O.sent_loss(gp, sc, labels, cc.numpy(), 10.0)[:2])
    ref += [O.focal_loss(O.arc_margin(sc, arc_t, cc, s=35), cc),
            O.focal_loss(O.arc_margin(gp, arc_i, cc, s=30), cc), O.global_loss(gp, sc)[0]]
    args.return_att_maps = False
    with torch.no_grad():
        gi, ri = tr.image_head(g, local)
        lab = torch.arange(b, device=gpu)
        mine = list(L.words_loss(ri, words, lab, None, cls, b, args)[:2])
        mine += list(L.sent_loss(gi, sent, lab, cls, b, args))
        mine += [tr.ident_loss(tr.text_cls(sent, cls), cls),
                 tr.ident_loss(tr.image_cls(gi, cls), cls), L.global_loss(gi, sent, args=args)]
    for name, a, e in zip(("w0", "w1", "s0", "s1", "tid", "iid", "global"), mine, ref):
        assert abs(a.item() - e.item()) < 1e-3, (name, a.item(), e.item())


def test_lstm_step_matches_oracle(gpu):
    """Stage-1 LSTM step (config 1) on the reference fixture's BiLSTM words and
    caption lengths (tests/golden/words_loss_lstm_b5.npz)."""
    from text_guided_face_recognition_amd.config import make_args
    from text_guided_face_recognition_amd.train import TrainLSTM
    gw = load_golden("words_loss_lstm_b5")
    words = t(gw["words_emb"])                         # [5, 256, 18], unnormalised
    lens = t(gw["cap_lens"])
    b, lmax = words.shape[0], words.shape[2]
    torch.manual_seed(3)
    args = make_args(lstm=True, batch_size=b, num_classes=7, precision="fp32")
    tr = TrainLSTM(args, gpu)
    gen = torch.Generator().manual_seed(4)
    g = torch.randn(b, 512, generator=gen)
    local = torch.randn(b, 256, 14, 14, generator=gen)
    sent = torch.randn(b, 256, generator=gen)
    sent = sent / sent.norm(dim=1, keepdim=True)
    cls = torch.tensor([1, 4, 1, 0, 6])
    hp = _cpu_params(tr.image_head, HEAD_KEYS)
    arc_i = tr.image_cls.weight.detach().cpu().clone().requires_grad_()
    arc_t = tr.text_cls.weight.detach().cpu().clone().requires_grad_()
    old = {k: v.detach().clone() for k, v in hp.items()}

    labels = torch.arange(b)
    gp, r = O.image_heading(g, local, hp)
    w0, w1, _, _ = O.words_loss(r, words, labels, lens, None, 4.0, 5.0, 10.0)
    tid = O.focal_loss(O.arc_margin(sent, arc_t, cls, s=35), cls)
    iid = O.focal_loss(O.arc_margin(gp, arc_i, cls, s=30), cls)
    cl = O.clip_loss(sent, gp)
    total = w0 + w1 + args.lambda_id * (tid + iid) + args.lambda_clip * cl
    total.backward()
    grads = {k: v.grad.clone() for k, v in hp.items()}
    torch.optim.Adam(list(hp.values()), lr=args.lr_head, betas=(0.5, 0.999)).step()
    torch.optim.SGD([arc_i, arc_t], lr=0.1, momentum=0.9, weight_decay=5e-5).step()

    # device-resident caption lengths (graph-capturable; no host sync)
    batch = (g.to(gpu), local.to(gpu), words.to(gpu), sent.to(gpu), cls.to(gpu),
             lens.to(gpu, torch.int32))
    out = tr.step(batch)
    torch.cuda.synchronize()
    assert abs(out["damsm"].item() - (w0 + w1).item()) < 1e-3
    assert abs(out["clip"].item() - args.lambda_clip * cl.item()) < 1e-3
    assert abs(out["ident"].item() - args.lambda_id * (tid + iid).item()) < 2e-1
    named = dict(tr.image_head.named_parameters())
    for k, v in HEAD_KEYS.items():
        _check_adam(named[k], old[v], hp[v].detach(), grads[v], args.lr_head, k,
                    max(x.abs().max().item() for x in grads.values()))
    _check_sgd(tr.image_cls.weight.detach().cpu(), arc_i.detach())
    _check_sgd(tr.text_cls.weight.detach().cpu(), arc_t.detach())


def test_lstm_graphed_step(gpu):
    """The LSTM step (device cap_lens) replays from a HIP graph exactly as it
    runs eagerly."""
    from text_guided_face_recognition_amd.config import make_args
    from text_guided_face_recognition_amd.train import GraphedStep, TrainLSTM, \
        synthetic_batch_lstm

    def build():
        torch.manual_seed(9)
        return TrainLSTM(make_args(lstm=True, batch_size=16, num_classes=50, precision="fp32"),
                         gpu)
    batch = synthetic_batch_lstm(16, 18, gpu, seed=2, n_ids=50)
    eager, graphed = build(), build()
    outs = [eager.step(batch) for _ in range(4)]
    gs = GraphedStep(graphed, tuple(x.clone() for x in batch), warmup=3)
    out = gs.step()
    torch.cuda.synchronize()
    for k in out:
        torch.testing.assert_close(out[k], outs[-1][k], rtol=1e-5, atol=1e-5)


def test_fusion_step_matches_oracle(gpu):
    """Stage-2 FCFM step: image head -> Working -> ArcMargin(640) -> focal,
    SGD(lr 0.1, wd 5e-4) on the classifier, Adam(wd 5e-5) on head + fusion."""
    from text_guided_face_recognition_amd.config import make_args
    from text_guided_face_recognition_amd.train import Fusion, synthetic_batch
    b, nw = 6, 22
    torch.manual_seed(21)
    args = make_args(batch_size=b, bert_words_num=24, num_classes=11, precision="fp32")
    tr = Fusion(args, gpu)
    batch = synthetic_batch(b, nw, gpu, seed=22, n_ids=11)
    hp = _cpu_params(tr.image_head, HEAD_KEYS)
    wp = _cpu_params(tr.fusion_net, WORKING_KEYS)
    arc = tr.metric_fc.weight.detach().cpu().clone().requires_grad_()
    old = {**{("h", k): v.detach().clone() for k, v in hp.items()},
           **{("w", k): v.detach().clone() for k, v in wp.items()}}
    gc, lc, wc, sc, cc = (x.cpu() for x in batch)
    gp, r = O.image_heading(gc, lc, hp)
    out = O.working(r, wc, gp, sc, wp)
    loss = O.focal_loss(O.arc_margin(out, arc, cc, s=30), cc)
    loss.backward()
    grads = {**{("h", k): v.grad.clone() for k, v in hp.items()},
             **{("w", k): v.grad.clone() for k, v in wp.items()}}
    torch.optim.SGD([arc], lr=0.1, weight_decay=5e-4).step()
    torch.optim.Adam(list(hp.values()) + list(wp.values()), lr=args.lr_head,
                     weight_decay=5e-5).step()

    got = tr.step(batch)["loss"].item()
    torch.cuda.synchronize()
    assert abs(got - loss.item()) < 1e-3, (got, loss.item())
    _check_sgd(tr.metric_fc.weight.detach().cpu(), arc.detach())
    g_all = max(x.abs().max().item() for x in grads.values())
    named_h = dict(tr.image_head.named_parameters())
    for k, v in HEAD_KEYS.items():
        _check_adam(named_h[k], old[("h", v)], hp[v].detach(), grads[("h", v)], args.lr_head,
                    k, g_all, wd=5e-5)
    named_w = dict(tr.fusion_net.named_parameters())
    for k, v in WORKING_KEYS.items():
        _check_adam(named_w[k], old[("w", v)], wp[v].detach(), grads[("w", v)], args.lr_head,
                    k, g_all, wd=5e-5)
