"""CPU oracle for the TGFR FCAM/FCFM hot path -- TEST INFRASTRUCTURE ONLY.

This module is a plain PyTorch-CPU fp32 restatement of the reference's hot-path
arithmetic, written op for op so that rounding behaviour and the CPU cost
profile follow the reference's own Python.  It exists for three consumers
only: ``tests/`` (as the parity checker), ``__graft_entry__.smoke()`` (as the
checker of one small GPU invocation) and ``bench.py``'s ``cpu_baseline`` leg
(timed on the host cores).  The product path in
``text_guided_face_recognition_amd`` never imports it.

Parity pin: every function here is checked in ``tests/test_oracle_golden.py``
against fixtures in ``tests/golden/`` that were produced by importing the
reference implementation itself (``tests/golden/make_golden.py``).

Reference anchors (paths relative to the reference checkout):
  cosine_similarity   models/losses.py:12-16
  sent_loss           models/losses.py:19-57
  words_loss          models/losses.py:61-135
  func_attention      models/attention.py:10-43
  ClipLoss            models/losses.py:268-309
  FocalLoss           models/losses.py:313-325
  global_loss         models/losses.py:329-351
  SelfAttention       models/fusion_nets.py:82-118
  Working (FCFM)      models/fusion_nets.py:217-258
  ProjectionHead      models/models.py:98-120
  IMIM                models/models.py:380-405
  ImageHeading        models/models.py:328-338
  ArcMarginProduct    models/metrics.py:17-60
  TextHeading         models/models.py:170-232 (Bert_Word_Mapping + TextHeading)
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

__all__ = [
    "cosine_similarity", "func_attention", "words_loss", "sent_loss",
    "global_loss", "clip_loss", "focal_loss", "self_attention", "working",
    "projection_head", "imim", "image_heading", "arc_margin", "text_heading",
]


def cosine_similarity(x1, x2, dim=1, eps=1e-8):
    """losses.py:12-16 -- the clamp is on the PRODUCT of the two norms."""
    num = (x1 * x2).sum(dim)
    den = torch.norm(x1, 2, dim) * torch.norm(x2, 2, dim)
    return (num / den.clamp(min=eps)).squeeze()


def func_attention(query, context, gamma1):
    """attention.py:10-43.

    query [B, D, T]; context [B, D, ih, iw].  Returns (C [B, D, T],
    attn [B, T, ih, iw]).  Softmax over words per region (:28-29), x gamma1,
    softmax over regions per word (:33-36), weighted context (:41).
    """
    b, _, t = query.shape
    ih, iw = context.shape[2], context.shape[3]
    n_src = ih * iw
    ctx = context.reshape(b, -1, n_src)                       # [B, D, R]
    scores = torch.bmm(ctx.transpose(1, 2).contiguous(), query)   # [B, R, T]
    a1 = torch.softmax(scores.reshape(b * n_src, t), dim=-1)
    a1 = a1.reshape(b, n_src, t).transpose(1, 2).contiguous()     # [B, T, R]
    a2 = torch.softmax((a1 * gamma1).reshape(b * t, n_src), dim=-1)
    a2 = a2.reshape(b, t, n_src)
    weighted = torch.bmm(ctx, a2.transpose(1, 2).contiguous())    # [B, D, T]
    return weighted, a2.reshape(b, -1, ih, iw)


def words_loss(img_features, words_emb, labels, cap_lens, n_words, gamma1,
               gamma2, gamma3, batch_size=None):
    """losses.py:61-135, restated with an explicit per-caption loop.

    ``n_words`` is the BERT word count (bert_words_num - 2, :83) used when
    ``cap_lens`` is None; otherwise caption i uses cap_lens[i] words (:82).
    Returns (loss0, loss1, att_maps, logits) where ``logits`` is the
    gamma3-scaled similarity matrix [B_img, B_cap] that the reference feeds to
    CrossEntropyLoss (:122-132).
    """
    n_img = img_features.shape[0]
    n_cap = words_emb.shape[0] if batch_size is None else batch_size
    cols, att_maps = [], []
    for i in range(n_cap):
        nw = int(cap_lens[i]) if cap_lens is not None else int(n_words)
        word = words_emb[i, :, :nw].unsqueeze(0).contiguous().repeat(n_img, 1, 1)
        wctx, attn = func_attention(word, img_features, gamma1)
        if i < n_img:
            att_maps.append(attn[i].unsqueeze(0).contiguous())
        w_rows = word.transpose(1, 2).contiguous().reshape(n_img * nw, -1)
        c_rows = wctx.transpose(1, 2).contiguous().reshape(n_img * nw, -1)
        sim = cosine_similarity(w_rows, c_rows).reshape(n_img, nw)
        sim = torch.log(torch.exp(sim * gamma2).sum(dim=1, keepdim=True))
        cols.append(sim)
    logits = torch.cat(cols, 1) * gamma3
    if labels is None:
        return None, None, att_maps, logits
    loss0 = F.cross_entropy(logits, labels)
    loss1 = F.cross_entropy(logits.transpose(0, 1), labels)
    return loss0, loss1, att_maps, logits


def _class_mask(class_ids, n):
    ids = np.asarray(class_ids)
    m = ids.reshape(-1, 1) == ids.reshape(1, -1)
    m[np.arange(n), np.arange(n)] = False
    return torch.from_numpy(m)


def sent_loss(cnn_code, rnn_code, labels, class_ids, gamma3, eps=1e-8):
    """losses.py:19-57 -> (loss0, loss1, masked logits)."""
    n = cnn_code.shape[0]
    num = cnn_code @ rnn_code.t()
    den = torch.norm(cnn_code, 2, dim=1, keepdim=True) @ \
        torch.norm(rnn_code, 2, dim=1, keepdim=True).t()
    scores = num / den.clamp(min=eps) * gamma3
    if class_ids is not None:
        scores.data.masked_fill_(_class_mask(class_ids, n), -float("inf"))
    if labels is None:
        return None, None, scores
    return (F.cross_entropy(scores, labels),
            F.cross_entropy(scores.t(), labels), scores)


def global_loss(cnn_code, rnn_code, eps=1e-8, temp3=10.0):
    """losses.py:329-351 -> (loss0 + loss1, logits)."""
    n = cnn_code.shape[0]
    labels = torch.arange(n)
    num = cnn_code @ rnn_code.t()
    den = torch.norm(cnn_code, 2, dim=1, keepdim=True) @ \
        torch.norm(rnn_code, 2, dim=1, keepdim=True).t()
    scores = num / den.clamp(min=eps) * temp3
    return F.cross_entropy(scores, labels) + \
        F.cross_entropy(scores.t(), labels), scores


def clip_loss(text_features, image_features, logit_scale=1.0):
    """losses.py:298-309: un-normalised dot products, mean of both CEs."""
    per_image = logit_scale * image_features @ text_features.t()
    per_text = logit_scale * text_features @ image_features.t()
    labels = torch.arange(per_image.shape[0])
    return (F.cross_entropy(per_image, labels) +
            F.cross_entropy(per_text, labels)) / 2


def focal_loss(logits, target, gamma=2.0):
    """losses.py:313-325 (the CE is already a batch mean; .mean() is a no-op)."""
    logp = F.cross_entropy(logits, target)
    p = torch.exp(-logp)
    return ((1 - p) ** gamma * logp).mean()


def self_attention(x, y, p, scale):
    """fusion_nets.py:82-118 with explicit parameters.

    p: dict with q_w [C', C, 1, 1], q_b, k_w, k_b, v_w [C, C, 1, 1], v_b.
    The query role is key_proj(x), the key role query_proj(y) (:94-103).
    """
    c = x.shape[1]
    sqrt_dim = np.sqrt(c / scale)
    q = F.conv2d(y, p["q_w"], p["q_b"])
    n, cq, w, h = q.shape
    q = q.contiguous().view(n, cq, h * w)
    k = F.conv2d(x, p["k_w"], p["k_b"]).contiguous().view(n, cq, -1)
    k = k.transpose(2, 1)
    att = torch.softmax(torch.bmm(k, q) / sqrt_dim, dim=-1)
    v = F.conv2d(x, p["v_w"], p["v_b"])
    n, c2, w, h = y.shape
    v = v.contiguous().view(n, c2, -1).transpose(2, 1)
    out = torch.bmm(att, v).permute(0, 2, 1)
    return out.contiguous().view(n, c2, w, h)


def _bn_train(x, w, b, eps=1e-5):
    return F.batch_norm(x, None, None, w, b, training=True, eps=eps)


def working(img, word, gl_img, sent, p):
    """fusion_nets.py:217-258 (FCFM) in training mode (batch-stat BN)."""
    z = F.max_pool2d(F.relu(F.conv2d(img, p["conv_w"], p["conv_b"])), 2)
    z = _bn_train(z, p["bn_img_w"], p["bn_img_b"])
    wd = F.linear(word.transpose(1, 2), p["proj_w"], p["proj_b"])
    wd = torch.bmm(wd.transpose(1, 2), wd) / np.sqrt(36)
    wd = wd.unsqueeze(-1).view(wd.size(0), wd.size(1), 6, 6)
    wd = _bn_train(wd, p["bn_word_w"], p["bn_word_b"])
    sa = {k[3:]: v for k, v in p.items() if k.startswith("sa_")}
    iw = self_attention(z, wd, sa, 1)
    iw = F.layer_norm(iw, [36, 6, 6], p["ln_w"], p["ln_b"])
    iw = F.max_pool2d(iw, 2).reshape(iw.size(0), -1)
    iw = F.linear(iw, p["lin_w"], p["lin_b"])
    g = F.layer_norm(gl_img, [256], p["ln_g_w"], p["ln_g_b"])
    s = F.layer_norm(sent, [256], p["ln_s_w"], p["ln_s_b"])
    return torch.cat((iw, g, s), dim=1)


def projection_head(x, w, b):
    """models.py:98-120: Linear then L2-normalise the last dim."""
    return F.normalize(F.linear(x, w, b), p=2, dim=-1)


def imim(img, p):
    """models.py:380-405 in training mode; returns R [B, 256, 14, 14]."""
    z = _bn_train(img, p["bn_w"], p["bn_b"])
    sa = {k[3:]: v for k, v in p.items() if k.startswith("sa_")}
    z = self_attention(z, z, sa, 1)
    z = F.layer_norm(z, [256, 14, 14], p["ln_w"], p["ln_b"])
    z = F.relu(F.conv2d(z, p["c1_w"], p["c1_b"]))
    z = F.relu(F.conv2d(z, p["c2_w"], p["c2_b"]))
    z = projection_head(z.permute(0, 2, 3, 1), p["pl_w"], p["pl_b"])
    return z.permute(0, 3, 1, 2)


def image_heading(global_image, local_image, p):
    """models.py:328-338 -> (g' [B, 256], R [B, 256, 14, 14])."""
    r = imim(local_image, p)
    g = projection_head(global_image, p["pg_w"], p["pg_b"])
    return g, r


def arc_margin(x, weight, label, s=30.0, m=0.5, easy_margin=False):
    """metrics.py:17-60 without the CUDA-only one-hot (:53)."""
    cosine = F.linear(F.normalize(x), F.normalize(weight))
    sine = torch.sqrt((1.0 - cosine ** 2).clamp(0, 1))
    phi = cosine * math.cos(m) - sine * math.sin(m)
    if easy_margin:
        phi = torch.where(cosine > 0, phi, cosine)
    else:
        phi = torch.where(cosine > math.cos(math.pi - m), phi,
                          cosine - math.sin(math.pi - m) * m)
    one_hot = torch.zeros_like(cosine)
    one_hot.scatter_(1, label.view(-1, 1).long(), 1)
    return (one_hot * phi + (1.0 - one_hot) * cosine) * s


def text_heading(words_emb, conv_w, conv_b, bert_words_num=None):
    """models.py:170-232 (forward of TextHeading; run under no_grad in the
    reference, utils/dataset_utils.py:42).

    words_emb [B, L-1, 768] (BERT last hidden state without [CLS],
    models.py:166); conv_w[k] [256, 1, K, 768], conv_b[k] [256] for K = 2, 3, 4.
    Returns (words [B, 256, L-2] -- a transposed view of [B, L-2, 256] storage,
    as :231 -- and sent [B, 256]).
    """
    x = words_emb.unsqueeze(1)                                            # :182
    x = [F.relu(F.conv2d(x, w, b)).squeeze(3) for w, b in zip(conv_w, conv_b)]  # :183
    L = words_emb.shape[1] + 1 if bert_words_num is None else bert_words_num
    a, b_, c = (t.transpose(2, 1) for t in x)                             # :199-201
    code = []
    seq = L - 1 - 3                                                       # :204
    for i in range(a.shape[0]):
        t = [torch.amax(torch.stack((a[i, j], b_[i, j], c[i, j])), dim=0) for j in range(seq)]
        t += [torch.amax(torch.stack((a[i, seq], b_[i, seq])), dim=0)]   # :206
        t += [a[i, seq + 1].float()]                                      # :207
        code.append(torch.stack(t))
    words = F.normalize(torch.stack(code), p=2, dim=2)                    # :211-212
    pooled = [F.max_pool1d(t, t.size(2)).squeeze(2) for t in x]          # :217
    sent = F.normalize(torch.stack(pooled).mean(dim=0), p=2, dim=1)       # :218-219
    return words.transpose(1, 2), sent
