"""Generate the golden fixtures in tests/golden/ by running the REFERENCE code.

Run in the build container only (the reference is not present on GPU boxes):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py /root/reference

The reference is imported read-only from the given path.  Modules it imports
but never uses on the hot path are stubbed (torchsummary at
models/fusion_nets.py:8; torchvision at models/models.py:5,13), as SURVEY.md
section 8(c) prescribes.  ``words_loss`` does not return its similarity
matrix, so CrossEntropyLoss inside models.losses is wrapped by a recorder to
capture the logits it is called with (models/losses.py:131-132).

Each fixture is an .npz with inputs, parameters, outputs and input gradients;
every case is seeded (manual_seed 100 per cfg/train_bert.yml:15, plus a case
offset) so the script is reproducible.
"""
from __future__ import annotations

import importlib.machinery
import os
import sys
import types

import numpy as np
import torch

OUT = os.path.dirname(os.path.abspath(__file__))


def _import_reference(root):
    sys.dont_write_bytecode = True          # the reference tree stays untouched
    sys.path.insert(0, root)
    sys.modules.setdefault("torchsummary", types.SimpleNamespace(summary=None))
    import transformers  # noqa: F401  (models.models imports these names first)
    from transformers import (AlignTextModel, BertModel, BlipTextModel,  # noqa
                              CLIPTextModel, FlavaTextModel, GroupViTTextModel)
    for name in ("torchvision", "torchvision.models"):
        mod = types.ModuleType(name)
        mod.__spec__ = importlib.machinery.ModuleSpec(name, None)
        sys.modules[name] = mod
    sys.modules["torchvision"].models = sys.modules["torchvision.models"]
    import models.attention as ref_att
    import models.fusion_nets as ref_fus
    import models.losses as ref_loss
    import models.metrics as ref_metrics
    import models.models as ref_models
    return ref_att, ref_loss, ref_fus, ref_models, ref_metrics


class _Args:
    """The attribute bag the reference losses read (cfg/train_bert.yml)."""

    def __init__(self, en_type="BERT", bert_words_num=32):
        self.en_type = en_type
        self.bert_words_num = bert_words_num
        self.CUDA = False
        self.device = torch.device("cpu")
        self.aux_feat_dim_per_granularity = 256
        smooth = types.SimpleNamespace(GAMMA1=4.0, GAMMA2=5.0, GAMMA3=10.0)
        self.TRAIN = types.SimpleNamespace(SMOOTH=smooth)


def _record_ce(ref_loss):
    """Wrap nn.CrossEntropyLoss inside models.losses to capture its inputs."""
    seen = []
    real = torch.nn.CrossEntropyLoss

    class Recorder(real):
        def forward(self, input, target):
            seen.append(input.detach().clone())
            return super().forward(input, target)

    proxy = types.ModuleType("nn_proxy")
    proxy.__dict__.update(torch.nn.__dict__)
    proxy.CrossEntropyLoss = Recorder
    ref_loss.nn = proxy
    return seen


def _unit_rows(x, dim):
    return x / x.norm(dim=dim, keepdim=True)


def _save(name, **arrays):
    clean = {}
    for k, v in arrays.items():
        if isinstance(v, torch.Tensor):
            v = v.detach().cpu().numpy()
        clean[k] = np.asarray(v)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **clean)
    size = sum(a.nbytes for a in clean.values())
    print(f"{name}: {len(clean)} arrays, {size / 1024:.0f} KiB")


def _params(module, prefix=""):
    return {prefix + k.replace(".", "_"): v.detach().clone()
            for k, v in module.state_dict().items()}


def gen_func_attention(ref_att):
    cases = {"small": (3, 16, 4, 5, 101), "t22": (2, 256, 14, 22, 102)}
    for tag, (b, d, hw, t, seed) in cases.items():
        torch.manual_seed(seed)
        q = torch.randn(b, d, t)
        ctx = torch.randn(b, d, hw, hw, requires_grad=True)
        wc, attn = ref_att.func_attention(q, ctx, 4.0)
        probe = torch.randn_like(wc)
        (wc * probe).sum().backward()
        _save(f"func_attention_{tag}", query=q, context=ctx, gamma1=4.0,
              weighted=wc, attn=attn, probe=probe, d_context=ctx.grad)


def gen_words_loss(ref_loss):
    seen = _record_ce(ref_loss)
    cases = {
        "bert_b4_t30": dict(b=4, words=32, lens=None),
        "bert_b6_t22": dict(b=6, words=24, lens=None),
        "lstm_b5": dict(b=5, words=None, lens=[18, 12, 7, 15, 3]),
    }
    for k, (tag, cfg) in enumerate(cases.items()):
        torch.manual_seed(200 + k)
        b = cfg["b"]
        # R: channels-last storage as IMIM produces it (models/models.py:401-404)
        r = _unit_rows(torch.randn(b, 14, 14, 256), -1).permute(0, 3, 1, 2)
        r = r.detach().requires_grad_()
        if cfg["lens"] is None:
            t = cfg["words"] - 2
            w = _unit_rows(torch.randn(b, t, 256), -1).transpose(1, 2)
            args = _Args("BERT", cfg["words"])
            cap_lens = None
        else:
            tmax = max(cfg["lens"])
            w = (torch.rand(b, tmax, 256) * 2 - 1).mul(0.6).transpose(1, 2)
            args = _Args("LSTM")
            cap_lens = torch.tensor(cfg["lens"])
        labels = torch.arange(b)
        seen.clear()
        l0, l1, att = ref_loss.words_loss(r, w, labels, cap_lens, None, b, args)
        (l0 + l1).backward()
        att_diag = np.zeros((b, w.shape[2], 14, 14), np.float32)
        for i, a in enumerate(att):
            att_diag[i, :a.shape[1]] = a[0].detach().numpy()
        _save(f"words_loss_{tag}", img_features=r, words_emb=w.contiguous(),
              cap_lens=(np.asarray(cfg["lens"]) if cap_lens is not None
                        else np.zeros(0, np.int64)),
              bert_words_num=(cfg["words"] or 0), logits=seen[0],
              loss0=l0, loss1=l1, att_diag=att_diag, d_img=r.grad)


def gen_sent_global_clip(ref_loss):
    torch.manual_seed(300)
    b = 8
    img = torch.randn(b, 256, requires_grad=True)
    sent = _unit_rows(torch.randn(b, 256), -1)
    class_ids = np.array([3, 7, 3, 1, 7, 7, 0, 5])
    labels = torch.arange(b)
    args = _Args()
    seen = _record_ce(ref_loss)
    seen.clear()
    s0, s1 = ref_loss.sent_loss(img, sent, labels, class_ids, b, args)
    (s0 + s1).backward()
    _save("sent_loss_b8", cnn_code=img, rnn_code=sent, class_ids=class_ids,
          loss0=s0, loss1=s1, logits=seen[0], d_cnn=img.grad)

    img2 = img.detach().clone().requires_grad_()
    gl = ref_loss.global_loss(img2, sent)
    gl.backward()
    _save("global_loss_b8", cnn_code=img2, rnn_code=sent, loss=gl,
          d_cnn=img2.grad)

    img3 = _unit_rows(img.detach(), -1).requires_grad_()
    text = _unit_rows(torch.randn(b, 256), -1)
    cl = ref_loss.ClipLoss()(text, img3, args)
    cl.backward()
    _save("clip_loss_b8", text=text, image=img3, loss=cl, d_image=img3.grad)

    logits = torch.randn(b, 50, requires_grad=True)
    tgt = torch.tensor([1, 4, 9, 0, 49, 3, 3, 7])
    fl = ref_loss.FocalLoss(gamma=2)(logits, tgt)
    fl.backward()
    _save("focal_loss_b8", logits=logits, target=tgt, loss=fl,
          d_logits=logits.grad)


def gen_self_attention(ref_fus):
    for tag, (b, c, hw, cross) in {"c256_hw196": (2, 256, 14, False),
                                   "c36_hw36": (3, 36, 6, True)}.items():
        torch.manual_seed(400 + c)
        m = ref_fus.SelfAttention(c, scale=1)
        x = torch.randn(b, c, hw, hw, requires_grad=True)
        y = torch.randn(b, c, hw, hw, requires_grad=True) if cross else x
        out = m(x, y)
        probe = torch.randn_like(out)
        (out * probe).sum().backward()
        p = {"q_w": m.query_proj.weight, "q_b": m.query_proj.bias,
             "k_w": m.key_proj.weight, "k_b": m.key_proj.bias,
             "v_w": m.value_proj.weight, "v_b": m.value_proj.bias}
        extra = {"d_" + k: v.grad for k, v in p.items()
                 if c < 64 or k in ("q_w", "v_w", "v_b")}
        _save(f"self_attention_{tag}", x=x, y=y, out=out, probe=probe,
              d_x=x.grad, d_y=(y.grad if cross else x.grad),
              **{k: v.detach() for k, v in p.items()}, **extra)


def gen_working(ref_fus):
    torch.manual_seed(500)
    b, t = 3, 22
    net = ref_fus.Working(256).train()
    img = _unit_rows(torch.randn(b, 14, 14, 256), -1).permute(0, 3, 1, 2)
    img = img.detach().requires_grad_()
    word = _unit_rows(torch.randn(b, t, 256), -1).transpose(1, 2).contiguous()
    gl = torch.randn(b, 256)
    sent = torch.randn(b, 256)
    out = net(img, word, gl, sent)
    probe = torch.randn_like(out)
    (out * probe).sum().backward()
    grads = {"d_" + k.replace(".", "_"): v.grad
             for k, v in net.named_parameters()}
    _save("working_b3", img=img, word=word, gl_img=gl, sent=sent, out=out,
          probe=probe, d_img=img.grad, **_params(net), **grads)


def gen_image_heading(ref_models):
    torch.manual_seed(600)
    b = 2
    args = _Args()
    net = ref_models.ImageHeading(args).train()
    g = torch.randn(b, 512, requires_grad=True)
    loc = torch.randn(b, 256, 14, 14, requires_grad=True)
    gp, r = net(g, loc)
    pg, pr = torch.randn_like(gp), torch.randn_like(r)
    ((gp * pg).sum() + (r * pr).sum()).backward()
    keep = ("imim.sa.value_proj.weight", "imim.sa.query_proj.bias",
            "imim.project_local.projection.weight", "imim.ln.weight",
            "project_global.projection.weight")
    grads = {"d_" + k.replace(".", "_"): v.grad
             for k, v in net.named_parameters() if k in keep}
    _save("image_heading_b2", global_image=g, local_image=loc, g_out=gp,
          r_out=r, probe_g=pg, probe_r=pr, d_global=g.grad, d_local=loc.grad,
          **_params(net), **grads)


def text_heading_inputs(seed, b, L):
    """Deterministic TextHeading inputs (numpy PCG64, stable across versions):
    BERT last hidden state without [CLS] [b, L-1, 768] and the three conv
    weights [256, 1, K, 768] / biases [256] for K = 2, 3, 4.  The test side
    regenerates the 7 MB of weights from the seed instead of storing them."""
    rng = np.random.default_rng(seed)
    words = rng.standard_normal((b, L - 1, 768), dtype=np.float32)
    ws, bs = [], []
    for k in (2, 3, 4):
        bound = 1.0 / np.sqrt(k * 768.0)
        ws.append((rng.uniform(-bound, bound, (256, 1, k, 768))).astype(np.float32))
        bs.append((rng.uniform(-bound, bound, (256,))).astype(np.float32))
    return words, ws, bs


def gen_text_heading(ref_models):
    """models/models.py:170-232, run as the trainer does (no_grad,
    utils/dataset_utils.py:42); torch.cuda.FloatTensor (:207) is the one
    CUDA-only call and is patched to a CPU float copy."""
    torch.cuda.FloatTensor = lambda t: t.float()
    for seed, b, L in ((700, 3, 32), (701, 2, 24)):
        args = _Args(bert_words_num=L)
        net = ref_models.TextHeading(args).eval()
        words, ws, bs = text_heading_inputs(seed, b, L)
        with torch.no_grad():
            for conv, w, bb in zip(net.bwm.convs1, ws, bs):
                conv.weight.copy_(torch.from_numpy(w))
                conv.bias.copy_(torch.from_numpy(bb))
            w_out, s_out = net(torch.from_numpy(words), torch.zeros(b, 768))
        _save(f"text_heading_b{b}_l{L}", seed=seed, bert_words_num=L,
              words_emb=words, words_out=w_out.contiguous(), sent_out=s_out)


def words_seeded_inputs(seed, b, t, noise=0.02):
    """Inputs of the full-shape words_loss fixtures, regenerated from the seed
    instead of stored (the B = 64 region map alone is 12.8 MB): unit regions
    R [B, 14, 14, 256] (returned as the channels-last [B, 256, 14, 14] view
    IMIM produces) and captions whose words are noisy copies of regions of
    their own image, W [B, 256, T] (a view of [B, T, 256] storage), so every
    matching pair leads its row and column by >= 1 logit -- a margin the
    reduced-precision kernels must resolve (argmax identity).  CPU generator:
    bit-identical on any host with this torch build."""
    gen = torch.Generator().manual_seed(seed)
    r = _unit_rows(torch.randn(b, 196, 256, generator=gen), -1)
    idx = torch.randint(0, 196, (b, t), generator=gen)
    w = _unit_rows(r[torch.arange(b)[:, None], idx] +
                   noise * torch.randn(b, t, 256, generator=gen), -1)
    return r.reshape(b, 14, 14, 256).permute(0, 3, 1, 2), w.transpose(1, 2)


SEEDED_WORDS = {"bert_b64_l32": (900, 64, 32), "bert_b16_l64": (901, 16, 64)}


def gen_words_loss_seeded(ref_loss):
    """words_loss at the headline batch (B = 64, bert_words_num = 32, T = 30)
    and at configs[4]'s caption length (bert_words_num = 64, T = 62,
    models/losses.py:83): the reference's logits and losses, and its region
    gradient sampled at 4096 seeded positions plus its max and norm (the
    inputs are regenerated from the seed, words_seeded_inputs)."""
    seen = _record_ce(ref_loss)
    for tag, (seed, b, L) in SEEDED_WORDS.items():
        r, w = words_seeded_inputs(seed, b, L - 2)
        r = r.detach().requires_grad_()
        args = _Args("BERT", L)
        labels = torch.arange(b)
        seen.clear()
        l0, l1, _ = ref_loss.words_loss(r, w, labels, None, None, b, args)
        (l0 + l1).backward()
        g = r.grad.detach()
        pick = torch.randperm(g.numel(), generator=torch.Generator().manual_seed(seed))[:4096]
        _save(f"words_loss_{tag}_seeded", seed=seed, batch=b, bert_words_num=L,
              r_sum=r.detach().double().sum(), w_sum=w.double().sum(),
              logits=seen[0], loss0=l0, loss1=l1, d_img_idx=pick,
              d_img_val=g.reshape(-1)[pick], d_img_absmax=g.abs().max(), d_img_norm=g.norm())


def _cpu_torch_proxy():
    """A ``torch`` module proxy whose ``zeros`` ignores ``device=``: the one
    CUDA-only call of ArcMarginProduct.forward is its one-hot buffer
    (models/metrics.py:53, ``torch.zeros(..., device='cuda')``); everything
    else is the real torch."""
    proxy = types.ModuleType("torch_proxy")
    proxy.__dict__.update(torch.__dict__)
    real = torch.zeros

    def zeros(*size, device=None, **kw):
        return real(*size, **kw)
    proxy.zeros = zeros
    return proxy


def gen_arc_margin(ref_metrics):
    """ArcMarginProduct (models/metrics.py:17-60) with s = 30 (image head) and
    35 (text head, src/train_encoders_bert.py:186-191), easy_margin False and
    True; some rows aligned and some anti-aligned with their class weight so
    both sides of every torch.where (:47-50) are taken.  Gradients to the input
    and to the weight through a random probe."""
    ref_metrics.torch = _cpu_torch_proxy()
    torch.manual_seed(800)
    b, d, n_cls = 8, 256, 50
    label = torch.tensor([3, 17, 3, 49, 0, 22, 8, 31])
    base = ref_metrics.ArcMarginProduct(d, n_cls, s=30.0, m=0.5)
    weight0 = base.weight.detach().clone()
    wn = weight0 / weight0.norm(dim=1, keepdim=True)
    sign = torch.tensor([1.0, -1.0, 0.3, -1.0, 1.0, 0.0, -0.2, 1.0]).view(-1, 1)
    x0 = 2.0 * (sign * wn[label] + 0.02 * torch.randn(b, d))
    probe = torch.randn(b, n_cls)
    arrays = dict(x=x0, weight=weight0, label=label, probe=probe, m=0.5)
    for s_ in (30.0, 35.0):
        for easy in (False, True):
            net = ref_metrics.ArcMarginProduct(d, n_cls, s=s_, m=0.5, easy_margin=easy)
            with torch.no_grad():
                net.weight.copy_(weight0)
            x = x0.clone().requires_grad_()
            out = net(x, label)
            (out * probe).sum().backward()
            tag = f"s{int(s_)}_{'easy' if easy else 'std'}"
            arrays[f"out_{tag}"] = out
            arrays[f"d_x_{tag}"] = x.grad
            arrays[f"d_w_{tag}"] = net.weight.grad
    _save("arc_margin_b8", **arrays)


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    torch.set_num_threads(8)
    ref_att, ref_loss, ref_fus, ref_models, ref_metrics = _import_reference(root)
    gen_func_attention(ref_att)
    gen_words_loss(ref_loss)
    gen_sent_global_clip(ref_loss)
    gen_self_attention(ref_fus)
    gen_working(ref_fus)
    gen_image_heading(ref_models)
    gen_text_heading(ref_models)
    gen_arc_margin(ref_metrics)
    gen_words_loss_seeded(ref_loss)


if __name__ == "__main__":
    main()
