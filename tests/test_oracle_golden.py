"""Pin the CPU oracle (oracle/tgfr_oracle.py) against fixtures produced by the
reference itself (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from conftest import load_golden, t, words_seeded_golden
from oracle import tgfr_oracle as O

torch.set_num_threads(4)


def close(a, b, atol=1e-5, rtol=1e-5):
    a = a.detach().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    np.testing.assert_allclose(a, b, atol=atol, rtol=rtol)


@pytest.mark.parametrize("tag", ["small", "t22"])
def test_func_attention(tag):
    g = load_golden(f"func_attention_{tag}")
    ctx = t(g["context"]).requires_grad_()
    wc, attn = O.func_attention(t(g["query"]), ctx, float(g["gamma1"]))
    close(wc, g["weighted"])
    close(attn, g["attn"])
    (wc * t(g["probe"])).sum().backward()
    close(ctx.grad, g["d_context"], atol=1e-4)


@pytest.mark.parametrize("tag", ["bert_b4_t30", "bert_b6_t22", "lstm_b5"])
def test_words_loss(tag):
    g = load_golden(f"words_loss_{tag}")
    r = t(g["img_features"]).requires_grad_()
    w = t(g["words_emb"])
    b = r.shape[0]
    lens = g["cap_lens"] if g["cap_lens"].size else None
    l0, l1, att, logits = O.words_loss(
        r, w, torch.arange(b), lens, int(g["bert_words_num"]) - 2,
        4.0, 5.0, 10.0)
    close(logits, g["logits"], atol=2e-4)
    # identical argmax identities, rows and columns
    assert (logits.argmax(1).numpy() == g["logits"].argmax(1)).all()
    assert (logits.argmax(0).numpy() == g["logits"].argmax(0)).all()
    close(l0, g["loss0"], atol=1e-5)
    close(l1, g["loss1"], atol=1e-5)
    for i, a in enumerate(att):
        close(a[0], g["att_diag"][i, :a.shape[1]], atol=1e-6)
    (l0 + l1).backward()
    close(r.grad, g["d_img"], atol=1e-6, rtol=1e-4)


@pytest.mark.parametrize("tag", ["bert_b64_l32", "bert_b16_l64"])
def test_words_loss_seeded_full_shape(tag):
    """The oracle at the headline batch (B = 64, T = 30) and at configs[4]'s
    caption length (T = 62) against the reference's own outputs there: logits,
    losses and the sampled region gradient (inputs regenerated from the seed)."""
    g, r, w = words_seeded_golden(f"words_loss_{tag}_seeded")
    r = r.contiguous().requires_grad_()
    b, nw = r.shape[0], int(g["bert_words_num"]) - 2
    l0, l1, _, logits = O.words_loss(r, w, torch.arange(b), None, nw, 4.0, 5.0, 10.0)
    close(logits, g["logits"], atol=2e-4)
    assert (logits.argmax(1).numpy() == g["logits"].argmax(1)).all()
    assert (logits.argmax(0).numpy() == g["logits"].argmax(0)).all()
    close(l0, g["loss0"], atol=1e-5)
    close(l1, g["loss1"], atol=1e-5)
    (l0 + l1).backward()
    got = r.grad.reshape(-1)[torch.from_numpy(g["d_img_idx"])]
    scale = float(g["d_img_absmax"])
    assert (got - t(g["d_img_val"])).abs().max().item() < 1e-4 * scale
    assert abs(r.grad.abs().max().item() - scale) < 1e-4 * scale
    assert abs(r.grad.norm().item() - float(g["d_img_norm"])) < 1e-4 * float(g["d_img_norm"])


def test_sent_global_clip_focal():
    g = load_golden("sent_loss_b8")
    x = t(g["cnn_code"]).requires_grad_()
    l0, l1, sc = O.sent_loss(x, t(g["rnn_code"]), torch.arange(8),
                             g["class_ids"], 10.0)
    close(sc, g["logits"])
    close(l0, g["loss0"])
    close(l1, g["loss1"])
    (l0 + l1).backward()
    close(x.grad, g["d_cnn"], atol=1e-6)

    g = load_golden("global_loss_b8")
    x = t(g["cnn_code"]).requires_grad_()
    loss, _ = O.global_loss(x, t(g["rnn_code"]))
    close(loss, g["loss"])
    loss.backward()
    close(x.grad, g["d_cnn"], atol=1e-6)

    g = load_golden("clip_loss_b8")
    x = t(g["image"]).requires_grad_()
    loss = O.clip_loss(t(g["text"]), x)
    close(loss, g["loss"])
    loss.backward()
    close(x.grad, g["d_image"], atol=1e-6)

    g = load_golden("focal_loss_b8")
    x = t(g["logits"]).requires_grad_()
    loss = O.focal_loss(x, t(g["target"]))
    close(loss, g["loss"])
    loss.backward()
    close(x.grad, g["d_logits"], atol=1e-6)


@pytest.mark.parametrize("tag", ["c256_hw196", "c36_hw36"])
def test_self_attention(tag):
    g = load_golden(f"self_attention_{tag}")
    cross = tag == "c36_hw36"
    x = t(g["x"]).requires_grad_()
    y = t(g["y"]).requires_grad_() if cross else x
    p = {k: t(g[k]) for k in ("q_w", "q_b", "k_w", "k_b", "v_w", "v_b")}
    out = O.self_attention(x, y, p, 1)
    close(out, g["out"], atol=1e-5)
    (out * t(g["probe"])).sum().backward()
    close(x.grad, g["d_x"], atol=1e-4, rtol=1e-4)
    if cross:
        close(y.grad, g["d_y"], atol=1e-4, rtol=1e-4)


def _working_params(g):
    names = {
        "conv_w": "conv_weight", "conv_b": "conv_bias",
        "bn_img_w": "bn_img_weight", "bn_img_b": "bn_img_bias",
        "bn_word_w": "bn_word_weight", "bn_word_b": "bn_word_bias",
        "proj_w": "projection_weight", "proj_b": "projection_bias",
        "sa_q_w": "sa_query_proj_weight", "sa_q_b": "sa_query_proj_bias",
        "sa_k_w": "sa_key_proj_weight", "sa_k_b": "sa_key_proj_bias",
        "sa_v_w": "sa_value_proj_weight", "sa_v_b": "sa_value_proj_bias",
        "ln_w": "ln_weight", "ln_b": "ln_bias",
        "lin_w": "linear_weight", "lin_b": "linear_bias",
        "ln_g_w": "ln_gl_image_weight", "ln_g_b": "ln_gl_image_bias",
        "ln_s_w": "ln_sent_weight", "ln_s_b": "ln_sent_bias",
    }
    return {k: t(g[v]) for k, v in names.items()}


def test_working():
    g = load_golden("working_b3")
    img = t(g["img"]).requires_grad_()
    out = O.working(img, t(g["word"]), t(g["gl_img"]), t(g["sent"]),
                    _working_params(g))
    close(out, g["out"], atol=1e-4, rtol=1e-4)
    (out * t(g["probe"])).sum().backward()
    close(img.grad, g["d_img"], atol=1e-4, rtol=1e-3)


def _heading_params(g):
    m = {"bn_w": "imim_bn_img_weight", "bn_b": "imim_bn_img_bias",
         "sa_q_w": "imim_sa_query_proj_weight", "sa_q_b": "imim_sa_query_proj_bias",
         "sa_k_w": "imim_sa_key_proj_weight", "sa_k_b": "imim_sa_key_proj_bias",
         "sa_v_w": "imim_sa_value_proj_weight", "sa_v_b": "imim_sa_value_proj_bias",
         "ln_w": "imim_ln_weight", "ln_b": "imim_ln_bias",
         "c1_w": "imim_conv1x1_1_weight", "c1_b": "imim_conv1x1_1_bias",
         "c2_w": "imim_conv1x1_2_weight", "c2_b": "imim_conv1x1_2_bias",
         "pl_w": "imim_project_local_projection_weight",
         "pl_b": "imim_project_local_projection_bias",
         "pg_w": "project_global_projection_weight",
         "pg_b": "project_global_projection_bias"}
    return {k: t(g[v]) for k, v in m.items()}


def test_image_heading():
    g = load_golden("image_heading_b2")
    gi = t(g["global_image"]).requires_grad_()
    li = t(g["local_image"]).requires_grad_()
    gp, r = O.image_heading(gi, li, _heading_params(g))
    close(gp, g["g_out"], atol=1e-5)
    close(r, g["r_out"], atol=1e-4, rtol=1e-4)
    ((gp * t(g["probe_g"])).sum() + (r * t(g["probe_r"])).sum()).backward()
    close(gi.grad, g["d_global"], atol=1e-5)
    close(li.grad, g["d_local"], atol=1e-4, rtol=1e-3)


@pytest.mark.parametrize("tag", ["b3_l32", "b2_l24"])
def test_text_heading(tag):
    from conftest import text_heading_golden
    g = text_heading_golden(f"text_heading_{tag}")
    words, sent = O.text_heading(t(g["words_emb"]), [t(w) for w in g["conv_w"]],
                                 [t(b) for b in g["conv_b"]], int(g["bert_words_num"]))
    close(words, g["words_out"])
    close(sent, g["sent_out"])


ARC_TAGS = ["s30_std", "s35_std", "s30_easy", "s35_easy"]


@pytest.mark.parametrize("tag", ARC_TAGS)
def test_arc_margin(tag):
    """oracle.arc_margin against the reference's ArcMarginProduct
    (models/metrics.py:17-60, run with its CUDA one-hot buffer on the CPU,
    make_golden.gen_arc_margin): logits and both gradients, both heads'
    scales, both margin variants, rows on both sides of each torch.where."""
    g = load_golden("arc_margin_b8")
    s_, kind = tag.split("_")
    x = t(g["x"]).requires_grad_()
    w = t(g["weight"]).requires_grad_()
    out = O.arc_margin(x, w, t(g["label"]), s=float(s_[1:]), m=float(g["m"]),
                       easy_margin=kind == "easy")
    close(out, g[f"out_{tag}"], atol=2e-5)
    (out * t(g["probe"])).sum().backward()
    close(x.grad, g[f"d_x_{tag}"], atol=1e-5, rtol=1e-4)
    close(w.grad, g[f"d_w_{tag}"], atol=1e-5, rtol=1e-4)


def test_arc_margin_fixture_covers_both_branches():
    g = load_golden("arc_margin_b8")
    wn = g["weight"] / np.linalg.norm(g["weight"], axis=1, keepdims=True)
    xn = g["x"] / np.linalg.norm(g["x"], axis=1, keepdims=True)
    cos_lab = (xn * wn[g["label"]]).sum(1)
    th = np.cos(np.pi - 0.5)
    assert (cos_lab > th).any() and (cos_lab <= th).any()      # standard margin branch
    assert (cos_lab > 0).any() and (cos_lab <= 0).any()        # easy margin branch
