"""Drop-in for the reference's models/losses.py hot-path functions.

Same names, signatures and return values as the reference; the arithmetic
runs in the gfx950 kernels of libtgfr_hip.so (see kernels.py):

  words_loss   models/losses.py:61-135   fused word<->region kernel + CE kernel
  sent_loss    models/losses.py:19-57    cosine-logit kernel (class mask) + CE
  global_loss  models/losses.py:329-351  cosine-logit kernel + CE
  ClipLoss     models/losses.py:268-309  dot-product logits + CE
  FocalLoss    models/losses.py:313-325  fused focal-CE kernel (identity head)

Extra knobs ride on ``args`` so the call sites stay identical:
  args.precision   "fp32" (split-bf16 MFMA, parity mode; default) or "bf16"
  args.dist        a DistContext (see dist.py) when running one process per
                   GPU: inputs are this rank's images, text features are the
                   all-gathered global batch, and the returned losses are this
                   rank's contributions (sum over ranks = the global loss).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import kernels as K

__all__ = ["cosine_similarity", "sent_loss", "words_loss", "global_loss", "ClipLoss",
           "FocalLoss"]


def _precision(args):
    return getattr(args, "precision", "fp32")


def _dist(args):
    ctx = getattr(args, "dist", None)
    if ctx is None or not ctx.active:
        return 0, None, None
    return ctx.row_offset, ctx.n_global, ctx.group


def cosine_similarity(x1, x2, dim=1, eps=1e-8):
    """losses.py:12-16 (the clamp is on the product of the norms)."""
    w12 = torch.sum(x1 * x2, dim)
    w1 = torch.norm(x1, 2, dim)
    w2 = torch.norm(x2, 2, dim)
    return (w12 / (w1 * w2).clamp(min=eps)).squeeze()


def _class_tensor(class_ids, device):
    if class_ids is None:
        return None
    if isinstance(class_ids, np.ndarray):
        class_ids = torch.from_numpy(class_ids)
    return torch.as_tensor(class_ids).to(device=device, dtype=torch.int64)


def sent_loss(cnn_code, rnn_code, labels, class_ids, batch_size, args, eps=1e-8):
    """losses.py:19-57: gamma3-scaled cosine logits, same-class off-diagonal
    entries masked to -inf, CE over rows and over columns."""
    row_offset, n_global, group = _dist(args)
    cls = _class_tensor(class_ids, cnn_code.device)
    logits = K.cos_logits(cnn_code, rnn_code, args.TRAIN.SMOOTH.GAMMA3, True, cls,
                          row_offset, eps=eps)
    if labels is None:
        return None, None
    return K.contrastive_ce(logits, row_offset, n_global or logits.shape[0], group)


_LENS = {}


def _const_lens(n, n_words, device):
    """Device-resident per-caption word counts for the BERT path (cached, so a
    step issues no host->device copy and can be graph-captured)."""
    key = (n, n_words, str(device))
    if key not in _LENS:
        _LENS[key] = torch.full((n,), n_words, dtype=torch.int32, device=device)
    return _LENS[key]


def words_loss(img_features, words_emb, labels, cap_lens, class_ids, batch_size, args):
    """losses.py:61-135 -> (loss0, loss1, att_maps).

    img_features [B, 256, 14, 14] (any strides); words_emb [B_cap, 256, T'].
    BERT: every caption uses bert_words_num - 2 words (:83); LSTM: cap_lens[i]
    (:82) -- host data (a list, numpy array or CPU tensor, as the reference
    passes) or a device int tensor (then T' is taken as the longest caption,
    which keeps the call free of host synchronisation for graph capture).
    att_maps are the matching-pair maps [1, T, 14, 14] (:97), produced by the
    forward kernel.
    """
    b_img = img_features.shape[0]
    b_cap = words_emb.shape[0]
    lens_host = None
    if args.en_type == "BERT":
        n_words = args.bert_words_num - 2
        lens = _const_lens(b_cap, n_words, img_features.device)
    elif torch.is_tensor(cap_lens) and cap_lens.is_cuda:
        n_words = words_emb.shape[2]
        lens = cap_lens.to(torch.int32)
    else:
        lens_host = [int(x) for x in np.asarray(cap_lens).reshape(-1)]
        n_words = max(lens_host)
        lens = torch.tensor(lens_host, dtype=torch.int32).to(img_features.device,
                                                               non_blocking=True)
    words = K.words_view(words_emb, n_words)
    row_offset, n_global, group = _dist(args)
    smooth = args.TRAIN.SMOOTH
    want_maps = getattr(args, "return_att_maps", True)
    if labels is not None and not want_maps and group is None and row_offset == 0:
        # one process, every caption here: logits + both CEs as one node (the
        # CE gradient formed in the backward's token-table launch)
        loss0, loss1 = K.word_region_ce(img_features, words, lens, smooth.GAMMA1, smooth.GAMMA2,
                                        smooth.GAMMA3, mode=_precision(args),
                                        bounded=args.en_type == "BERT",
                                        uniform=args.en_type == "BERT",
                                        n_global=n_global or b_img)
        return loss0, loss1, []
    # BERT-path features are L2-normalised (TextHeading models/models.py:212,
    # IMIM :403), so the scores are bounded by 1 and the forward needs no
    # running max over the words
    out = K.word_region_logits(img_features, words, lens, smooth.GAMMA1, smooth.GAMMA2,
                               smooth.GAMMA3, mode=_precision(args), img_offset=row_offset,
                               att_T=n_words if want_maps else 0,
                               bounded=args.en_type == "BERT",
                               uniform=args.en_type == "BERT")
    logits, att = (out if want_maps else (out, None))
    att_maps = []
    if att is not None:
        if lens_host is None:
            # BERT: every caption has n_words; a device cap_lens tensor is read
            # back once here (the maps' shapes depend on it, as in :97)
            lens_host = [n_words] * b_cap if args.en_type == "BERT" else lens.tolist()
        for b in range(b_img):
            t = lens_host[row_offset + b] if row_offset + b < b_cap else n_words
            att_maps.append(att[b, :t].reshape(1, t, 14, 14))
    if labels is None:
        return None, None, att_maps
    loss0, loss1 = K.contrastive_ce(logits, row_offset, n_global or b_img, group)
    return loss0, loss1, att_maps


def words_logits_bert(img_features, words_emb, args):
    """words_loss's logit block for the BERT path with no attention maps (the
    data-parallel forked step computes its CE in stages around a merged
    exchange, train.Train._step_forked_dp): [B_img, B_cap] through
    kernels.word_region_logits, exactly as words_loss forms it."""
    b_cap = words_emb.shape[0]
    n_words = args.bert_words_num - 2
    lens = _const_lens(b_cap, n_words, img_features.device)
    row_offset, _, _ = _dist(args)
    smooth = args.TRAIN.SMOOTH
    return K.word_region_logits(img_features, K.words_view(words_emb, n_words), lens,
                                smooth.GAMMA1, smooth.GAMMA2, smooth.GAMMA3,
                                mode=_precision(args), img_offset=row_offset, att_T=0,
                                bounded=True, uniform=True)


def global_loss(cnn_code, rnn_code, eps=1e-8, temp3=10.0, args=None):
    """losses.py:329-351 -> loss0 + loss1 (labels are arange(batch))."""
    row_offset, n_global, group = _dist(args)
    logits = K.cos_logits(cnn_code, rnn_code, temp3, True, None, row_offset, eps=eps)
    l0, l1 = K.contrastive_ce(logits, row_offset, n_global or logits.shape[0], group)
    return l0 + l1


def sent_global_loss(cnn_code, rnn_code, labels, class_ids, batch_size, args, eps=1e-8,
                     temp3=10.0):
    """(sent loss0, sent loss1, global loss) = sent_loss(...) and
    global_loss(..., temp3) of the trainer (src/train_encoders_bert.py:276-277,
    :310) on the same features.  One process with the whole batch (n <= 64):
    one fused kernel each way (kernels.SentGlobal); this rank's <= 128 images
    against the gathered captions (one process per GPU, or n > 64 on one):
    kernels.SentGlobalDist, the same arithmetic over column tiles with ONE
    column-partial exchange for both losses; otherwise the two losses as
    above."""
    row_offset, n_global, group = _dist(args)
    n = cnn_code.shape[0]
    # the fused kernels return no gradient for the sentence codes (the
    # reference's text side is detached, utils/dataset_utils.py:42); a caller
    # whose codes require grad takes the per-loss path, which computes it
    if labels is not None and n <= 128 and not rnn_code.requires_grad:
        cls = _class_tensor(class_ids, cnn_code.device)
        if n <= 64 and group is None and n == rnn_code.shape[0]:
            return K.sent_global(cnn_code, rnn_code, cls, args.TRAIN.SMOOTH.GAMMA3, temp3, eps)
        if rnn_code.shape[0] <= 8192:
            return K.sent_global_dist(cnn_code, rnn_code, cls, args.TRAIN.SMOOTH.GAMMA3, temp3,
                                      eps, row_offset, n_global, group)
    s0, s1 = sent_loss(cnn_code, rnn_code, labels, class_ids, batch_size, args, eps)
    return s0, s1, global_loss(cnn_code, rnn_code, eps, temp3, args)


class ClipLoss(nn.Module):
    """losses.py:268-309: un-normalised logits, mean of the two CEs."""

    def __init__(self, cache_labels=False):
        super().__init__()
        self.cache_labels = cache_labels

    def forward(self, text_features, image_features, args, logit_scale=1):
        row_offset, n_global, group = _dist(args)
        logits = K.cos_logits(image_features, text_features, float(logit_scale), False,
                              None, row_offset)
        l0, l1 = K.contrastive_ce(logits, row_offset, n_global or logits.shape[0], group)
        return (l0 + l1) / 2


class FocalLoss(nn.Module):
    """losses.py:313-325: (1 - e^-logp)^gamma * logp of the batch-mean CE,
    one fused kernel each way (kernels.FocalCE)."""

    def __init__(self, gamma=0, eps=1e-7):
        super().__init__()
        self.gamma = gamma
        self.eps = eps

    def forward(self, input, target):
        return K.focal_ce(input, target, self.gamma)
