"""torch.autograd front-ends of the HIP kernels (device tensors only).

Each Function here calls the C ABI of libtgfr_hip.so on torch's current
stream, with no host synchronisation, so a whole train step can be captured
in a HIP graph.  There is no CPU fallback: CPU tensors raise.
"""
from __future__ import annotations

import torch

from . import _hip
from ._hip import call, ptr

D = 256
RPAD = 224
NREG = 196
TPAD = 32

MODES = {"bf16": 0, "fp32": 1}


def _mode(mode):
    try:
        return MODES[mode]
    except KeyError:
        raise ValueError(f"precision mode must be one of {sorted(MODES)}") from None


def prep_rows(x, n_rows, rows_pad, lens=None, want_norms=False):
    """fp32 [items, rows, 256] (any strides) -> bf16 hi/lo [items, rows_pad, 256].

    Rows >= n_rows (or >= lens[item]) are zero.  Optional fp32 row norms.
    """
    assert x.dtype == torch.float32 and x.dim() == 3 and x.shape[2] == D
    n_items = x.shape[0]
    hi = torch.empty(n_items, rows_pad, D, dtype=torch.int16, device=x.device)
    lo = torch.empty_like(hi)
    norms = torch.empty(n_items, rows_pad, dtype=torch.float32, device=x.device) \
        if want_norms else None
    s0, s1, s2 = x.stride()
    call("tgfr_prep_rows", ptr(x), s0, s1, s2, n_items, n_rows, D, rows_pad,
         ptr(lens), ptr(hi), ptr(lo), ptr(norms), _hip.stream())
    return hi, lo, norms


def regions_view(img_features):
    """[B, 256, 14, 14] (any strides) -> strided view [B, 196, 256]."""
    b, d, hh, ww = img_features.shape
    assert d == D and hh * ww == NREG
    return img_features.flatten(2).transpose(1, 2)


def words_view(words_emb, n_words):
    """[B, 256, T'] -> strided view [B, T, 256] of the first n_words words."""
    return words_emb[:, :, :n_words].transpose(1, 2)


def bwd_chunks(b_img, b_cap):
    """Caption chunks for the backward grid (>= ~512 workgroups)."""
    want = max(1, -(-512 // (2 * b_img)))
    return max(1, min(b_cap, want))


class WordRegionLogits(torch.autograd.Function):
    """gamma3 * log sum_t exp(gamma2 cos(W_t, C_t)) for all (image, caption).

    Replaces the per-caption loop of models/losses.py:73-122 (with
    func_attention, models/attention.py:10-43).  Gradients flow to the image
    regions only: the text side is detached in the reference
    (utils/dataset_utils.py:42).
    """

    @staticmethod
    def forward(ctx, img_features, words, lens, gamma1, gamma2, gamma3, mode,
                img_offset=0, att_T=0, eps=1e-8):
        dev = img_features.device
        regions = regions_view(img_features.float())
        b_img, b_cap = regions.shape[0], words.shape[0]
        t_words = words.shape[1]
        if t_words > TPAD:
            raise ValueError(f"at most {TPAD} words per caption (got {t_words})")
        lens = lens.to(device=dev, dtype=torch.int32).contiguous()
        r_hi, r_lo, _ = prep_rows(regions, NREG, RPAD)
        w_hi, w_lo, w_norm = prep_rows(words.float(), t_words, TPAD, lens=lens,
                                       want_norms=True)
        logits = torch.empty(b_img, b_cap, dtype=torch.float32, device=dev)
        stats = torch.empty(b_img, b_cap, TPAD, 4, dtype=torch.float32, device=dev)
        cbuf = torch.empty(b_img, b_cap, TPAD, D, dtype=torch.float32, device=dev)
        att = torch.zeros(b_img, att_T, NREG, dtype=torch.float32, device=dev) \
            if att_T else None
        m = _mode(mode)
        call("tgfr_wr_fwd", ptr(r_hi), ptr(r_lo), ptr(w_hi), ptr(w_lo), ptr(w_norm),
             ptr(lens), b_img, b_cap, img_offset, gamma1, gamma2, gamma3, eps,
             ptr(logits), b_cap, ptr(stats), ptr(cbuf), ptr(att), att_T, m,
             _hip.stream())
        ctx.save_for_backward(r_hi, r_lo, w_hi, w_lo, w_norm, lens, stats, cbuf)
        ctx.cfg = (gamma1, gamma2, gamma3, eps, m, img_features.shape)
        ctx.mark_non_differentiable(*([att] if att is not None else []))
        return (logits, att) if att is not None else logits

    @staticmethod
    def backward(ctx, dlogits, *unused):
        r_hi, r_lo, w_hi, w_lo, w_norm, lens, stats, cbuf = ctx.saved_tensors
        gamma1, gamma2, gamma3, eps, m, shape = ctx.cfg
        b_img, b_cap = stats.shape[0], stats.shape[1]
        dlogits = dlogits.float().contiguous()
        chunks = bwd_chunks(b_img, b_cap)
        slab = torch.empty(chunks, b_img, RPAD, D, dtype=torch.float32,
                           device=dlogits.device)
        call("tgfr_wr_bwd", ptr(r_hi), ptr(r_lo), ptr(w_hi), ptr(w_lo), ptr(w_norm),
             ptr(lens), b_img, b_cap, chunks, gamma1, gamma2, gamma3, eps,
             ptr(dlogits), b_cap, ptr(stats), ptr(cbuf), ptr(slab), m, _hip.stream())
        d_reg = torch.empty(b_img, NREG, D, dtype=torch.float32, device=dlogits.device)
        call("tgfr_wr_reduce", ptr(slab), chunks, b_img, ptr(d_reg), NREG * D, D, 1, 0,
             _hip.stream())
        # same logical shape as img_features, channels-last strides
        d_img = d_reg.transpose(1, 2).reshape(shape)
        return (d_img,) + (None,) * 9


def word_region_logits(img_features, words, lens, gamma1, gamma2, gamma3,
                       mode="fp32", img_offset=0, att_T=0):
    return WordRegionLogits.apply(img_features, words, lens, float(gamma1),
                                  float(gamma2), float(gamma3), mode, img_offset, att_T)
