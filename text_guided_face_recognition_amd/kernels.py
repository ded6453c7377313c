"""torch.autograd front-ends of the HIP kernels (device tensors only).

Each Function here calls the C ABI of libtgfr_hip.so on torch's current
stream, with no host synchronisation, so a whole train step can be captured
in a HIP graph.  There is no CPU fallback: CPU tensors raise.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _hip
from ._hip import call, ptr

D = 256
RPAD = 224
NREG = 196
TPAD = 32
NREG_TILES = RPAD // 32
SP_REC = 64 * 16 + 64   # stored scores per (pair, region tile), int16 units (csrc SP_REC)
N_WR_SAVED = 13         # tensors _wr_fwd saves for _wr_bwd

MODES = {"bf16": 0, "fp32": 1, "fp16": 2}


def _mode(mode):
    """C-ABI precision of the generic kernels: "fp16" (BASELINE config 5's
    "fp16 with fp32 contrastive accumulate": the word-region contraction on
    fp16 MFMAs) runs the generic GEMMs in the fp32 split mode; the fused IMIM
    and TextHeading kernels run bf16 (models/models.py)."""
    try:
        return min(MODES[mode], MODES["fp32"])
    except KeyError:
        raise ValueError(f"precision mode must be one of {sorted(MODES)}") from None


def _wr_mode(mode):
    """C-ABI precision of the word-region kernels (0 bf16, 1 fp32 split, 2 fp16)."""
    try:
        return MODES[mode]
    except KeyError:
        raise ValueError(f"precision mode must be one of {sorted(MODES)}") from None


LOG2E = 1.4426950408889634
# largest score bound max|W| max|R| the max-free word<->region kernels handle
# exactly (csrc/tgfr_wr.hip, bound_shift)
WR_BOUND_MAX = 85.9


def wr_fast(mode, t_words, bounded, att_T=0):
    """True when the word<->region forward / backward take the bounded
    (max-free) kernels, which read only the words' operand rows: bf16 / fp16
    with t_pad = 32 (the pipelined forward and the two-role backward, no
    attention maps) or t_pad = 64 (_wr_fwd)."""
    m = _wr_mode(mode)
    t_pad = TPAD if t_words <= TPAD else 2 * TPAD
    return bool(bounded) and m != MODES["fp32"] and (
        (not att_T and t_pad == TPAD) or t_pad == 2 * TPAD)


def wr_rows_path(mode, t_words, bounded):
    """Whether gathered words may travel as their operand rows alone
    (rows_only_words): only when every consumer takes the fast path."""
    return mode in ("bf16", "fp16") and wr_fast(mode, t_words, bounded)


def prep_rows(x, n_rows, rows_pad, lens=None, want_norms=False, scale=1.0, f16=False):
    """fp32 [items, rows, 256] (any strides) -> bf16 hi/lo of scale * x
    [items, rows_pad, 256] (f16: fp16 bits in hi, no lo).

    Rows >= n_rows (or >= lens[item]) are zero.  Optional fp32 norms of the
    unscaled rows.
    """
    assert x.dtype == torch.float32 and x.dim() == 3 and x.shape[2] == D
    n_items = x.shape[0]
    hi = torch.empty(n_items, rows_pad, D, dtype=torch.int16, device=x.device)
    norms = torch.empty(n_items, rows_pad, dtype=torch.float32, device=x.device) \
        if want_norms else None
    s0, s1, s2 = x.stride()
    if f16:
        call("tgfr_prep_rows_f16", ptr(x), s0, s1, s2, n_items, n_rows, D, rows_pad,
             ptr(lens), float(scale), ptr(hi), ptr(norms), _hip.stream())
        return hi, None, norms
    lo = torch.empty_like(hi)
    call("tgfr_prep_rows", ptr(x), s0, s1, s2, n_items, n_rows, D, rows_pad,
         ptr(lens), float(scale), ptr(hi), ptr(lo), ptr(norms), _hip.stream())
    return hi, lo, norms


def regions_view(img_features):
    """[B, 256, 14, 14] (any strides) -> strided view [B, 196, 256]."""
    b, d, hh, ww = img_features.shape
    assert d == D and hh * ww == NREG
    return img_features.flatten(2).transpose(1, 2)


def words_view(words_emb, n_words):
    """[B, 256, T'] -> strided view [B, T, 256] of the first n_words words."""
    return words_emb[:, :, :n_words].transpose(1, 2)


def wr_bwd_ws_floats(b_img, b_cap, bounded, t_pad, mode):
    out = (ctypes.c_longlong * 1)()
    rc = _hip.lib().tgfr_wr_bwd_ws(int(b_img), int(b_cap), int(bounded), int(t_pad), int(mode),
                                   ctypes.addressof(out))
    if rc != 0:
        raise RuntimeError(f"tgfr_wr_bwd_ws failed with code {rc}")
    return int(out[0])


def _wr_fwd(img_features, words, lens, gamma1, gamma2, gamma3, mode, img_offset=0, att_T=0,
            bounded=False, uniform=False, eps=1e-8):
    """WordRegionLogits' forward: (logits, att, tensors for the backward, cfg)."""
    dev = img_features.device
    guard = w_plain = None          # the 64-token device guard (tgfr_wr_guard)
    regions = regions_view(img_features.float())
    b_img, b_cap = regions.shape[0], words.shape[0]
    t_words = words.shape[1]
    if t_words > 2 * TPAD:
        raise ValueError(f"at most {2 * TPAD} words per caption (got {t_words})")
    # token stride: 32, or 64 for 64-token captions (general kernels only)
    t_pad = TPAD if t_words <= TPAD else 2 * TPAD
    lens = lens.to(device=dev, dtype=torch.int32).contiguous()
    m = _wr_mode(mode)
    f16 = m == MODES["fp16"]
    bf16 = m != MODES["fp32"]          # single-operand modes (bf16, fp16)
    # bounded scores: the bf16 path runs the pipelined kernels both ways;
    # 64-token captions (bf16 / fp16) the bounded backward (log2(e)-scaled
    # words, no running max)
    fast = wr_fast(mode, t_words, bounded, att_T)
    pre = attached_rows(img_features, f16) if bf16 else None
    own_rows = pre is not None
    if pre is not None:            # written by the IMIM tail kernel
        (r_hi, r_norm), r_lo = pre, None
    else:
        r_hi, r_lo, r_norm = prep_rows(regions, NREG, RPAD, want_norms=bf16, f16=f16)
    if bf16:
        # the bf16 / fp16 forward takes log2(e)-scaled words (tgfr.h,
        # tgfr_wr_fwd), and so does the pipelined backward; the other
        # backward the plain ones.  (Written by TextHeading when it made
        # the words; every caption then has t_words valid words.)
        pre = attached_rows(words, f16, scale=LOG2E) if uniform else None
        w_attached = pre is not None and pre[0].shape[1] == t_pad
        if w_attached:
            w_fwd, w_norm = pre
        else:
            if _rows_only(words):
                raise RuntimeError("words carry only their operand rows "
                                   "(rows_only_words), which this call cannot use")
            own_rows = False
            w_fwd, _, w_norm = prep_rows(words.float(), t_words, t_pad, lens=lens,
                                         want_norms=True, scale=LOG2E, f16=f16)
        # 32-token captions: the max-free kernels decide per caption on the
        # device (a caption whose score bound max|W| max|R| exceeds BIG_C = 10,
        # formed in the forward and again in the token-table kernel, takes
        # their running-max variant): overflow-free for any input, also under
        # graph capture (the bf16 / fp16 operands' rounding still moves each
        # score by ~c 2^-9 / c 2^-11).  64-token captions: exact while the bound is <=
        # WR_BOUND_MAX (csrc/tgfr_wr.hip, bound_shift).  Rows made by this
        # package's heads are L2-normalised (bound ~1); other inputs get a
        # device guard (tgfr_wr_guard): every launch of the path has its exact
        # running-max twin beside it and the guard picks one on the device --
        # overflow-free for any input, also under graph capture, with no host read --
        # as the reference's softmax never overflows (models/attention.py:28-36)
        if bounded and t_pad != TPAD and not own_rows:
            if not _rows_only(words):
                guard = torch.empty(1, dtype=torch.int32, device=dev)
                call("tgfr_wr_guard", ptr(w_norm), w_norm.numel(), ptr(r_norm), r_norm.numel(),
                     ptr(guard), _hip.stream())
                w_plain = prep_rows(words.float(), t_words, t_pad, lens=lens, f16=f16)[0]
            elif not torch.cuda.is_current_stream_capturing():
                # gathered operand rows of this package's TextHeading (unit
                # rows) beside foreign regions: checked on the host
                if not float((w_norm.max() * r_norm.max()).item()) <= WR_BOUND_MAX:
                    bounded = fast = False
        if _rows_only(words) and not fast:
            raise RuntimeError("words carry only their bounded-kernel operand rows "
                               "(rows_only_words): this path needs the feature values")
        w_hi = w_fwd if fast else prep_rows(words.float(), t_words, t_pad, lens=lens,
                                            f16=f16)[0]
        w_lo = None
    else:
        if _rows_only(words):
            raise RuntimeError("words carry only their bf16 / fp16 operand rows "
                               "(rows_only_words): fp32 mode needs the feature values")
        w_hi, w_lo, w_norm = prep_rows(words.float(), t_words, t_pad, lens=lens,
                                       want_norms=True)
        w_fwd = w_hi
    logits = torch.empty(b_img, b_cap, dtype=torch.float32, device=dev)
    stats = torch.empty(b_img, b_cap, t_pad, 4, dtype=torch.float32, device=dev)
    # C for the backward: bf16 hi (+lo in fp32 mode), chunk-major [pair][32][t_pad][8]
    c_hi = torch.empty(b_img, b_cap, 32, t_pad, 8, dtype=torch.int16, device=dev)
    c_lo = torch.empty_like(c_hi) if m == MODES["fp32"] else None
    att = torch.zeros(b_img, att_T, NREG, dtype=torch.float32, device=dev) \
        if att_T else None
    # the scores S' of every (pair, region tile) for the two-role backward,
    # written by the bounded bf16 forward (fp16 / bf16 bits, accumulator order)
    sp = torch.empty(b_img, b_cap, NREG_TILES, SP_REC, dtype=torch.int16, device=dev) \
        if fast and t_pad == TPAD else None
    call("tgfr_wr_fwd", ptr(r_hi), ptr(r_lo), ptr(w_fwd), ptr(w_lo), ptr(w_norm),
         ptr(r_norm), ptr(lens), b_img, b_cap, img_offset, gamma1, gamma2, gamma3, eps,
         ptr(logits), b_cap, ptr(stats), ptr(c_hi), ptr(c_lo), ptr(sp), ptr(att), att_T,
         int(bool(bounded) and (t_pad == TPAD or m != MODES["fp32"])), t_pad, m, ptr(guard),
         _hip.stream())
    saved = (r_hi, r_lo, r_norm, w_hi, w_lo, w_norm, lens, stats, c_hi, c_lo, sp, w_plain, guard)
    cfg = (gamma1, gamma2, gamma3, eps, m, img_features.shape, fast, t_pad)
    return logits, att, saved, cfg


def _wr_bwd(saved, cfg, tok_call):
    """WordRegionLogits' backward: d img_features, with the per-(pair, token)
    table made by tok_call(stats, w_norm, r_norm, lens, b_img, b_cap, fast,
    t_pad, tok) (tgfr_wr_bwd_tok from dlogits, or tgfr_wr_bwd_tok_ce)."""
    r_hi, r_lo, r_norm, w_hi, w_lo, w_norm, lens, stats, c_hi, c_lo, sp, w_plain, guard = saved
    gamma1, gamma2, gamma3, eps, m, shape, fast, t_pad = cfg
    b_img, b_cap = stats.shape[0], stats.shape[1]
    dev = stats.device
    ws = torch.empty(wr_bwd_ws_floats(b_img, b_cap, fast, t_pad, m), dtype=torch.float32,
                     device=dev)
    tok = torch.empty(b_img, b_cap, t_pad, 8, dtype=torch.float32, device=dev)
    split = m == MODES["fp32"]
    # the token table's `bounded` code: 2 = the fp16 two-role backward, whose
    # forward stored C-hat scaled by 2^-8 (tgfr.h, tgfr_wr_bwd_tok)
    tok_bounded = 2 if fast and m == MODES["fp16"] and t_pad == TPAD else int(fast)
    tok_call(stats, w_norm, r_norm, lens, b_img, b_cap, tok_bounded, t_pad, tok, guard)
    d_reg = torch.empty(b_img, NREG, D, dtype=torch.float32, device=dev)
    call("tgfr_wr_bwd", ptr(r_hi), ptr(r_lo) if split else None, ptr(w_hi),
         ptr(w_lo) if split else None, b_img, b_cap, gamma1, ptr(tok),
         ptr(c_hi), ptr(c_lo) if split else None, ptr(sp), ptr(d_reg), NREG * D, D, 1, ptr(ws),
         int(fast), t_pad, m, ptr(w_plain), ptr(guard), _hip.stream())
    # same logical shape as img_features, channels-last strides
    return d_reg.transpose(1, 2).reshape(shape)


class WordRegionLogits(torch.autograd.Function):
    """gamma3 * log sum_t exp(gamma2 cos(W_t, C_t)) for all (image, caption).

    Replaces the per-caption loop of models/losses.py:73-122 (with
    func_attention, models/attention.py:10-43).  Gradients flow to the image
    regions only: the text side is detached in the reference
    (utils/dataset_utils.py:42).
    """

    @staticmethod
    def forward(ctx, img_features, words, lens, gamma1, gamma2, gamma3, mode,
                img_offset=0, att_T=0, bounded=False, uniform=False, eps=1e-8):
        logits, att, saved, cfg = _wr_fwd(img_features, words, lens, gamma1, gamma2, gamma3,
                                          mode, img_offset, att_T, bounded, uniform, eps)
        ctx.save_for_backward(*saved)
        ctx.cfg = cfg
        ctx.mark_non_differentiable(*([att] if att is not None else []))
        return (logits, att) if att is not None else logits

    @staticmethod
    def backward(ctx, dlogits, *unused):
        gamma1, gamma2, gamma3, eps = ctx.cfg[:4]
        dlogits = dlogits.float().contiguous()

        def tok_call(stats, w_norm, r_norm, lens, b_img, b_cap, fast, t_pad, tok, guard):
            call("tgfr_wr_bwd_tok", ptr(stats), ptr(w_norm), ptr(r_norm), ptr(lens), b_img,
                 b_cap, gamma1, gamma2, gamma3, eps, ptr(dlogits), b_cap, int(fast), t_pad,
                 ptr(tok), ptr(guard), _hip.stream())
        return (_wr_bwd(ctx.saved_tensors, ctx.cfg, tok_call),) + (None,) * 11


class WordRegionCE(torch.autograd.Function):
    """words_loss's (loss0, loss1) as ONE node when one process holds every
    caption and no attention maps are asked for: WordRegionLogits then
    ContrastiveCE (its single-launch statistics), with the CE gradient formed
    inside the word<->region backward's token-table launch
    (tgfr_wr_bwd_tok_ce) -- one launch fewer per step than the two nodes."""

    @staticmethod
    def forward(ctx, img_features, words, lens, gamma1, gamma2, gamma3, mode, bounded, uniform,
                n_global):
        logits, _, saved, cfg = _wr_fwd(img_features, words, lens, gamma1, gamma2, gamma3,
                                        mode, 0, 0, bounded, uniform)
        n_r, n_c = logits.shape
        dev = logits.device
        row_lse = torch.empty(n_r, dtype=torch.float32, device=dev)
        part = torch.empty(2, n_c, dtype=torch.float32, device=dev)
        col_lse = torch.empty(n_c, dtype=torch.float32, device=dev)
        loss = torch.empty(2, dtype=torch.float32, device=dev)
        inv_n = 1.0 / float(n_global)
        call("tgfr_ce_stats", ptr(logits), n_c, n_r, n_c, ptr(row_lse), ptr(part[0]),
             ptr(part[1]), ptr(col_lse), 0, inv_n, ptr(loss), ptr(_hip.counters(dev)),
             _hip.stream())
        ctx.save_for_backward(*saved, logits, row_lse, col_lse)
        ctx.cfg = cfg
        ctx.inv_n = inv_n
        return loss[0], loss[1]

    @staticmethod
    def backward(ctx, g0, g1):
        saved = ctx.saved_tensors
        logits, row_lse, col_lse = saved[N_WR_SAVED:]
        gamma1, gamma2, gamma3, eps = ctx.cfg[:4]
        w0 = 0.0 if g0 is None else 1.0
        w1 = 0.0 if g1 is None else 1.0
        g0 = None if g0 is None else g0.float().contiguous()
        g1 = None if g1 is None else g1.float().contiguous()

        def tok_call(stats, w_norm, r_norm, lens, b_img, b_cap, fast, t_pad, tok, guard):
            call("tgfr_wr_bwd_tok_ce", ptr(stats), ptr(w_norm), ptr(r_norm), ptr(lens), b_img,
                 b_cap, gamma1, gamma2, gamma3, eps, ptr(logits), logits.shape[1], 0,
                 ctx.inv_n, ptr(row_lse), ptr(col_lse), ptr(g0), ptr(g1), w0, w1, int(fast),
                 t_pad, ptr(tok), ptr(guard), _hip.stream())
        return (_wr_bwd(saved[:N_WR_SAVED], ctx.cfg, tok_call),) + (None,) * 9


def word_region_logits(img_features, words, lens, gamma1, gamma2, gamma3,
                       mode="fp32", img_offset=0, att_T=0, bounded=False, uniform=False):
    """bounded: the features are (near) unit rows -- the BERT path -- so the
    bf16 / fp16 kernels run without a running max (scores shifted by the
    device-computed bound max|W| max|R| when it reaches 40).  uniform: every
    caption has all words.shape[1] words (lens is that constant), so operand
    rows attached to the words by TextHeading (attach_rows) may be used."""
    return WordRegionLogits.apply(img_features, words, lens, float(gamma1),
                                  float(gamma2), float(gamma3), mode, img_offset, att_T,
                                  bool(bounded), bool(uniform))


def word_region_ce(img_features, words, lens, gamma1, gamma2, gamma3, mode="fp32",
                   bounded=False, uniform=False, n_global=None):
    """(loss0, loss1) of words_loss for one process holding every caption
    (WordRegionCE): word_region_logits + contrastive_ce in one node."""
    n_global = img_features.shape[0] if n_global is None else n_global
    return WordRegionCE.apply(img_features, words, lens, float(gamma1), float(gamma2),
                              float(gamma3), mode, bool(bounded), bool(uniform), n_global)


# -------------------------------------------------------- func_attention ---
class FuncAttention(torch.autograd.Function):
    """models/attention.py:10-43 for matched query / context batches, exact
    fp32 (tgfr_func_attention_fwd / _bwd), differentiable in both inputs."""

    @staticmethod
    def forward(ctx, query, context, gamma1):
        b, d, t = query.shape
        ih, iw = context.shape[2], context.shape[3]
        r = ih * iw
        q = query.float()
        c = context.float().reshape(b, context.shape[1], r)
        dev = q.device
        out = torch.empty(b, d, t, dtype=torch.float32, device=dev)
        a1 = torch.empty(b, r, t, dtype=torch.float32, device=dev)
        attn = torch.empty(b, t, r, dtype=torch.float32, device=dev)
        call("tgfr_func_attention_fwd", ptr(q), q.stride(0), q.stride(1), q.stride(2), ptr(c),
             c.stride(0), c.stride(1), c.stride(2), b, d, t, r, float(gamma1), ptr(out),
             out.stride(0), out.stride(1), out.stride(2), ptr(a1), ptr(attn), _hip.stream())
        ctx.save_for_backward(q, c, a1, attn)
        ctx.cfg = (float(gamma1), context.shape)
        return out, attn.view(b, t, ih, iw)

    @staticmethod
    def backward(ctx, d_out, d_attn):
        q, c, a1, attn = ctx.saved_tensors
        gamma1, cshape = ctx.cfg
        b, d, t = q.shape
        r = c.shape[2]
        if d_out is None:
            d_out = torch.zeros_like(q)
        d_out = d_out.float()
        da = None if d_attn is None else d_attn.float().reshape(b, t, r).contiguous()
        dq = torch.empty(b, d, t, dtype=torch.float32, device=q.device)
        dc = torch.empty(b, d, r, dtype=torch.float32, device=q.device)
        call("tgfr_func_attention_bwd", ptr(q), q.stride(0), q.stride(1), q.stride(2), ptr(c),
             c.stride(0), c.stride(1), c.stride(2), ptr(d_out), d_out.stride(0),
             d_out.stride(1), d_out.stride(2), ptr(da), b, d, t, r, gamma1, ptr(a1), ptr(attn),
             ptr(dq), ptr(dc), _hip.stream())
        return dq, dc.view(cshape), None


def func_attention(query, context, gamma1):
    """(weightedContext [B, D, T], attn [B, T, ih, iw]); device tensors only."""
    return FuncAttention.apply(query, context, gamma1)


# ------------------------------------------------------------ cos logits ---
class CosLogits(torch.autograd.Function):
    """scale * cos(x_b, y_i) (or scale * x_b.y_i) for all pairs, optional
    same-class mask; gradient to x (and to y when it requires grad)."""

    @staticmethod
    def forward(ctx, x, y, scale, normalize, cls, row_offset, eps=1e-8):
        x = x.float().contiguous()
        y = y.float().contiguous()
        n_x, n_y = x.shape[0], y.shape[0]
        out = torch.empty(n_x, n_y, dtype=torch.float32, device=x.device)
        masked = cls is not None
        if masked:
            cls = cls.to(device=x.device, dtype=torch.int64).contiguous()
        call("tgfr_cos_logits", ptr(x), D, ptr(y), D, n_x, n_y, D, int(normalize),
             float(scale), float(eps), int(masked), ptr(cls), int(row_offset), ptr(out),
             n_y, _hip.stream())
        ctx.save_for_backward(x, y)
        ctx.cfg = (float(scale), int(normalize), float(eps))
        return out

    @staticmethod
    def backward(ctx, g):
        x, y = ctx.saved_tensors
        scale, normalize, eps = ctx.cfg
        g = g.float().contiguous()
        n_x, n_y = g.shape
        dx = dy = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            call("tgfr_cos_logits_bwd", ptr(g), n_y, 1, ptr(x), D, ptr(y), D, n_x, n_y,
                 D, normalize, scale, eps, ptr(dx), D, _hip.stream())
        if ctx.needs_input_grad[1]:
            dy = torch.empty_like(y)
            call("tgfr_cos_logits_bwd", ptr(g), 1, n_y, ptr(y), D, ptr(x), D, n_y, n_x,
                 D, normalize, scale, eps, ptr(dy), D, _hip.stream())
        return dx, dy, None, None, None, None, None


def cos_logits(x, y, scale, normalize=True, cls=None, row_offset=0, eps=1e-8):
    return CosLogits.apply(x, y, scale, normalize, cls, row_offset, float(eps))


# ---------------------------------------------------------- contrastive CE ---
def _focal_global(group, n_global, rows, gamma, wss, losses):
    """Focal losses of 1-2 heads on the global mean CE: pack the local NLL sums
    (tgfr_focal_global phase 0), ONE all-reduce, finish (phase 1) into the
    heads' workspaces and 1-element loss tensors."""
    from .dist import all_reduce_sum_
    dev = wss[0].device
    sums = torch.empty(len(wss), dtype=torch.float32, device=dev)
    a = [ptr(w) for w in wss] + [None] * (2 - len(wss))
    lo = [ptr(l) for l in losses] + [None] * (2 - len(losses))
    call("tgfr_focal_global", 0, ptr(sums), 1, 0, len(wss), rows, 1.0 / float(n_global),
         float(gamma), a[0], a[1], None, None, _hip.stream())
    all_reduce_sum_(sums, group)
    call("tgfr_focal_global", 1, ptr(sums), 1, 0, len(wss), rows, 1.0 / float(n_global),
         float(gamma), a[0], a[1], lo[0], lo[1], _hip.stream())


def combine_col_partials(parts):
    """[world, 2, n_c] per-rank (column max, sum exp(x - max)) -> global column
    log-sum-exp [n_c] (tgfr_col_lse_combine, one launch)."""
    if parts.dtype != torch.float32 or parts.stride(2) != 1 or parts.stride(1) != parts.shape[2]:
        parts = parts.float().contiguous()
    world, _, n_c = parts.shape
    out = torch.empty(n_c, dtype=torch.float32, device=parts.device)
    call("tgfr_col_lse_combine", ptr(parts), world, parts.stride(0), n_c, ptr(out),
         _hip.stream())
    return out


def gather_col_partials(part, group):
    """The one collective of the contrastive CE: all_gather of this rank's
    [2, n_c] column partials -> [world, 2, n_c] (rank-major)."""
    if group is None:
        return part.unsqueeze(0)
    from .dist import all_gather_cat
    return all_gather_cat(part.unsqueeze(0), group)


def exchange_col_partials(part, group):
    """Global column log-sum-exp from this rank's partials: gather + combine."""
    return combine_col_partials(gather_col_partials(part, group))


class ContrastiveCE(torch.autograd.Function):
    """(CE(rows), CE(columns)) of a [local rows x global columns] logit block.

    Row b of this rank is global row `row_offset + b`, labelled with the
    caption of the same index.  With a process group, the column partials are
    exchanged with one all_gather so loss1 sees every rank's rows, exactly as
    the reference's single-process DataParallel losses do on the gathered
    batch.  Returned losses are this rank's contributions; summing them over
    ranks gives the global-batch losses.
    """

    @staticmethod
    def forward(ctx, logits, row_offset, n_global, group, pre=None):
        logits = logits.float().contiguous()
        n_r, n_c = logits.shape
        dev = logits.device
        loss = torch.empty(2, dtype=torch.float32, device=dev)
        inv_n = 1.0 / float(n_global)
        if pre is not None:
            # ce_partials ran earlier and its column partials rode in a merged
            # exchange (train.Train._step_forked_dp): row LSE + gathered parts
            row_lse, parts = pre
            col_lse = combine_col_partials(parts)
            call("tgfr_ce_loss", ptr(logits), n_c, n_r, int(row_offset), inv_n, ptr(row_lse),
                 ptr(col_lse), ptr(loss), _hip.stream())
            ctx.save_for_backward(logits, row_lse, col_lse)
            ctx.cfg = (int(row_offset), inv_n)
            return loss[0], loss[1]
        row_lse = torch.empty(n_r, dtype=torch.float32, device=dev)
        part = torch.empty(2, n_c, dtype=torch.float32, device=dev)
        if group is None:
            # one launch: stats, final column LSE and both losses
            col_lse = torch.empty(n_c, dtype=torch.float32, device=dev)
            call("tgfr_ce_stats", ptr(logits), n_c, n_r, n_c, ptr(row_lse), ptr(part[0]),
                 ptr(part[1]), ptr(col_lse), int(row_offset), inv_n, ptr(loss),
                 ptr(_hip.counters(dev)), _hip.stream())
        else:
            call("tgfr_ce_stats", ptr(logits), n_c, n_r, n_c, ptr(row_lse), ptr(part[0]),
                 ptr(part[1]), None, 0, 0.0, None, None, _hip.stream())
            col_lse = exchange_col_partials(part, group)
            call("tgfr_ce_loss", ptr(logits), n_c, n_r, int(row_offset), inv_n, ptr(row_lse),
                 ptr(col_lse), ptr(loss), _hip.stream())
        ctx.save_for_backward(logits, row_lse, col_lse)
        ctx.cfg = (int(row_offset), inv_n)
        return loss[0], loss[1]

    @staticmethod
    def backward(ctx, g0, g1):
        logits, row_lse, col_lse = ctx.saved_tensors
        row_offset, inv_n = ctx.cfg
        n_r, n_c = logits.shape
        w0 = 0.0 if g0 is None else 1.0
        w1 = 0.0 if g1 is None else 1.0
        g0 = None if g0 is None else g0.float().contiguous()
        g1 = None if g1 is None else g1.float().contiguous()
        dl = torch.empty_like(logits)
        call("tgfr_ce_grad", ptr(logits), n_c, n_r, n_c, row_offset, inv_n, ptr(row_lse),
             ptr(col_lse), ptr(g0), ptr(g1), w0, w1, ptr(dl), n_c, _hip.stream())
        return dl, None, None, None, None


def contrastive_ce(logits, row_offset=0, n_global=None, group=None, pre=None):
    """(CE rows, CE columns) of a logit block; pre = (row_lse, gathered column
    partials [world, 2, n_c]) from ce_partials and a merged exchange."""
    n_global = logits.shape[0] if n_global is None else n_global
    return ContrastiveCE.apply(logits, row_offset, n_global, group, pre)


def ce_partials(logits, part):
    """Stage 1 of a data-parallel contrastive CE: the row LSE [n_r] and this
    rank's column partials (max, sum exp(x - max)) written into `part` [2, n_c]
    (a view of a merged exchange buffer) by tgfr_ce_stats; no loss."""
    logits = logits.detach().float().contiguous()
    n_r, n_c = logits.shape
    row_lse = torch.empty(n_r, dtype=torch.float32, device=logits.device)
    assert part.shape == (2, n_c) and part.stride(1) == 1 and part.stride(0) == n_c
    call("tgfr_ce_stats", ptr(logits), n_c, n_r, n_c, ptr(row_lse), ptr(part[0]), ptr(part[1]),
         None, 0, 0.0, None, None, _hip.stream())
    return row_lse


class SentGlobal(torch.autograd.Function):
    """(sent loss0, sent loss1, global loss) of one process holding the whole
    batch (n <= 64): sent_loss (models/losses.py:19-57, gamma3, same-class
    mask) and global_loss (:329-351, temp3) share one cosine matrix, one
    forward launch and one backward launch (tgfr_sent_global).  Gradient to
    the image side only (the text side is detached, utils/dataset_utils.py:42)."""

    @staticmethod
    def forward(ctx, x, y, cls, s_sent, s_glob, eps):
        x = _aligned(x)
        y = _aligned(y)
        n = x.shape[0]
        dev = x.device
        cls = cls.to(device=dev, dtype=torch.int64).contiguous()
        cosv = torch.empty(n, n, dtype=torch.float32, device=dev)
        stats = torch.empty(4, n, dtype=torch.float32, device=dev)
        nrm = torch.empty(2, n, dtype=torch.float32, device=dev)
        loss = torch.empty(3, dtype=torch.float32, device=dev)
        call("tgfr_sent_global", ptr(x), x.stride(0), ptr(y), y.stride(0), n, ptr(cls),
             float(s_sent), float(s_glob), float(eps), ptr(cosv), ptr(stats), ptr(nrm), ptr(loss),
             _hip.stream())
        ctx.save_for_backward(x, y, cls, cosv, stats, nrm)
        ctx.cfg = (float(s_sent), float(s_glob), float(eps))
        ctx.set_materialize_grads(False)
        return loss[0], loss[1], loss[2]

    @staticmethod
    def backward(ctx, gs0, gs1, ggl):
        x, y, cls, cosv, stats, nrm = ctx.saved_tensors
        s_sent, s_glob, eps = ctx.cfg
        n = x.shape[0]
        dx = torch.empty_like(x)
        g = [None if v is None else v.float().contiguous() for v in (gs0, gs1, ggl)]
        call("tgfr_sent_global_bwd", ptr(g[0]), ptr(g[1]), ptr(g[2]), ptr(x), x.stride(0),
             ptr(y), y.stride(0), n, ptr(cls), s_sent, s_glob, eps, ptr(cosv), ptr(stats),
             ptr(nrm), ptr(dx), dx.stride(0), _hip.stream())
        return dx, None, None, None, None, None


def sent_global(x, y, cls, s_sent, s_glob, eps=1e-8):
    return SentGlobal.apply(x, y, cls, s_sent, s_glob, eps)


def _sgd_ws(n_r, n_c):
    out = (ctypes.c_longlong * 3)()
    rc = _hip.lib().tgfr_sent_global_dist_ws(int(n_r), int(n_c), ctypes.addressof(out),
                                             ctypes.addressof(out) + 8,
                                             ctypes.addressof(out) + 16)
    if rc != 0:
        raise RuntimeError(f"tgfr_sent_global_dist_ws failed with code {rc}")
    return int(out[0]), int(out[1]), int(out[2])


class SentGlobalDist(torch.autograd.Function):
    """SentGlobal for this rank's n_r <= 128 images (global rows row_offset ..)
    against n_c gathered captions: cosines and both losses' row / column
    partials in one launch over column tiles, ONE all-gather of the column
    partials of both losses (with a process group), one loss launch; backward
    one launch (tgfr_sent_global_dist_*).  Returns this rank's contributions
    (sum over ranks = the global-batch losses), as ContrastiveCE does."""

    @staticmethod
    def forward(ctx, x, y, cls, s_sent, s_glob, eps, row_offset, n_global, group, pre=None):
        x = _aligned(x)
        y = _aligned(y)
        n_r, n_c = x.shape[0], y.shape[0]
        dev = x.device
        cls = cls.to(device=dev, dtype=torch.int64).contiguous()
        n_rp, n_cp, n_st = _sgd_ws(n_r, n_c)
        stats = torch.empty(n_st, dtype=torch.float32, device=dev)
        loss = torch.empty(3, dtype=torch.float32, device=dev)
        if pre is not None:
            # sent_global_dist_parts ran earlier; its column partials rode in a
            # merged exchange: [world, >= n_cp] rows (any row stride)
            cosv, rowpart, nrm, parts = pre
            world, ld = parts.shape[0], parts.stride(0)
        else:
            cosv = torch.empty(n_r, n_c, dtype=torch.float32, device=dev)
            rowpart = torch.empty(n_rp, dtype=torch.float32, device=dev)
            colpart = torch.empty(n_cp, dtype=torch.float32, device=dev)
            nrm = torch.empty(n_r + n_c, dtype=torch.float32, device=dev)
            call("tgfr_sent_global_dist_fwd", ptr(x), x.stride(0), n_r, ptr(y), y.stride(0), n_c,
                 ptr(cls), int(row_offset), float(s_sent), float(s_glob), float(eps), ptr(cosv),
                 ptr(rowpart), ptr(colpart), ptr(nrm), _hip.stream())
            world, ld = 1, 0
            parts = colpart
            if group is not None:
                from .dist import all_gather_cat
                parts = all_gather_cat(colpart.unsqueeze(0), group)
                world = parts.shape[0]
        inv_n = 1.0 / float(n_global)
        call("tgfr_sent_global_dist_loss", ptr(cosv), n_r, n_c, int(row_offset), float(s_sent),
             float(s_glob), ptr(rowpart), ptr(parts), world, ld, inv_n, ptr(stats), ptr(loss),
             _hip.stream())
        ctx.save_for_backward(x, y, cls, cosv, stats, nrm)
        ctx.cfg = (float(s_sent), float(s_glob), float(eps), int(row_offset), inv_n)
        ctx.set_materialize_grads(False)
        return loss[0], loss[1], loss[2]

    @staticmethod
    def backward(ctx, gs0, gs1, ggl):
        x, y, cls, cosv, stats, nrm = ctx.saved_tensors
        s_sent, s_glob, eps, row_offset, inv_n = ctx.cfg
        n_r, n_c = cosv.shape
        dx = torch.empty_like(x)
        g = [None if v is None else v.float().contiguous() for v in (gs0, gs1, ggl)]
        call("tgfr_sent_global_dist_bwd", ptr(g[0]), ptr(g[1]), ptr(g[2]), ptr(x), x.stride(0),
             n_r, ptr(y), y.stride(0), n_c, ptr(cls), row_offset, s_sent, s_glob, eps, inv_n,
             ptr(cosv), ptr(stats), ptr(nrm), ptr(dx), dx.stride(0), _hip.stream())
        return (dx,) + (None,) * 9


def sent_global_dist(x, y, cls, s_sent, s_glob, eps=1e-8, row_offset=0, n_global=None,
                     group=None, pre=None):
    """pre: sent_global_dist_parts' (cosv, rowpart, nrm) + the gathered column
    partials [world, >= n_cp] of a merged exchange."""
    return SentGlobalDist.apply(x, y, cls, s_sent, s_glob, eps, row_offset,
                                n_global or x.shape[0], group, pre)


def sent_global_dist_cols(n_r, n_c):
    """Floats of this rank's sent/global column partials (tgfr_sent_global_dist_ws)."""
    return _sgd_ws(n_r, n_c)[1]


def sent_global_dist_parts(x, y, cls, s_sent, s_glob, eps, row_offset, colpart):
    """Stage 1 of SentGlobalDist: cosines, row partials and norms, this rank's
    column partials written into `colpart` (a view of a merged exchange
    buffer, sent_global_dist_cols floats); returns (cosv, rowpart, nrm)."""
    x = _aligned(x.detach())
    y = _aligned(y)
    n_r, n_c = x.shape[0], y.shape[0]
    dev = x.device
    cls = cls.to(device=dev, dtype=torch.int64).contiguous()
    n_rp, n_cp, _ = _sgd_ws(n_r, n_c)
    assert colpart.numel() == n_cp and colpart.is_contiguous()
    cosv = torch.empty(n_r, n_c, dtype=torch.float32, device=dev)
    rowpart = torch.empty(n_rp, dtype=torch.float32, device=dev)
    nrm = torch.empty(n_r + n_c, dtype=torch.float32, device=dev)
    call("tgfr_sent_global_dist_fwd", ptr(x), x.stride(0), n_r, ptr(y), y.stride(0), n_c,
         ptr(cls), int(row_offset), float(s_sent), float(s_glob), float(eps), ptr(cosv),
         ptr(rowpart), ptr(colpart), ptr(nrm), _hip.stream())
    return cosv, rowpart, nrm


# ------------------------------------------------------------------ bgemm ---
def bgemm(a, b, out=None, alpha=1.0, accumulate=False, mode="fp32", bias=None,
          relu=False, ksplit=1):
    """out[n] = epi(alpha * a[n] @ b[n] (+ out[n]) + bias) for 3-D fp32 tensors of
    any strides (transposed views cost nothing: strides are passed through).
    ksplit > 1 splits K over blocks; the partial tiles are summed in-launch."""
    assert a.dim() == 3 and b.dim() == 3 and a.shape[0] == b.shape[0]
    assert a.shape[2] == b.shape[1] and a.dtype == b.dtype == torch.float32
    nb, m, k = a.shape
    n = b.shape[2]
    if out is None:
        out = torch.empty(nb, m, n, dtype=torch.float32, device=a.device)
    slab = cnt = None
    if ksplit > 1:
        assert nb * -(-m // 64) * -(-n // 64) <= _hip.N_COUNTERS
        padded = nb * (-(-m // 128) * 128) * (-(-n // 128) * 128)
        slab = torch.empty(ksplit * padded, dtype=torch.float32, device=a.device)
        cnt = _hip.counters(a.device)
    call("tgfr_bgemm", ptr(a), a.stride(0), a.stride(1), a.stride(2), ptr(b), b.stride(0),
         b.stride(1), b.stride(2), ptr(out), out.stride(0), out.stride(1), out.stride(2),
         nb, m, n, k, float(alpha), int(accumulate), ptr(bias), int(relu), int(ksplit),
         ptr(slab), ptr(cnt), _mode(mode), _hip.stream())
    return out


def _ksplit(k, mn_blocks):
    """Split-K factor giving ~512 blocks to a small-output GEMM, with K slices
    of at least 128 (K < 2048) or 256 elements."""
    if mn_blocks >= 256 or k < 256:
        return 1
    chunk = 128 if k < 2048 else 256
    return int(max(1, min(k // chunk, -(-512 // mn_blocks))))


class ConvReluPool(torch.autograd.Function):
    """MaxPool2d(2)(relu(Conv2d(256, 36, 3, padding=0)(x))) of the FCFM image
    branch (models/fusion_nets.py:236-237) in one launch each way
    (csrc/tgfr_fcfm.hip): x [B, 256, 14, 14] -> [B, 36, 6, 6].

    x is read as channels-last rows [B][196][256] (ImageHeading's physical
    layout, no copy); other layouts are made channels-last first.  The forward
    keeps the 2x2 argmax (with the ReLU folded in) for the backward, which
    returns dx (channels-last strides), dW and db."""

    @staticmethod
    def forward(ctx, x, weight, bias, mode):
        b, cin, h, w = x.shape
        if (cin, h, w) != (256, 14, 14) or tuple(weight.shape) != (36, 256, 3, 3):
            raise ValueError("FCFM conv: x [B, 256, 14, 14], weight [36, 256, 3, 3] "
                             f"(got {tuple(x.shape)}, {tuple(weight.shape)})")
        rows = x.float().permute(0, 2, 3, 1)                       # [B, 14, 14, 256]
        if not (rows.stride(3) == 1 and rows.stride(2) == 256 and rows.stride(1) == 14 * 256
                and rows.stride(0) % 4 == 0 and rows.data_ptr() % 16 == 0):
            rows = rows.contiguous()
        m = _mode(mode)
        pk = torch.empty(_hip.lib().tgfr_fcfm_pack_elems(), dtype=torch.int16, device=x.device)
        call("tgfr_fcfm_pack", ptr(weight.float().contiguous()), ptr(pk), _hip.stream())
        pooled = torch.empty(b, 36, 6, 6, dtype=torch.float32, device=x.device)
        code = torch.empty(b, 36, 6, 6, dtype=torch.int8, device=x.device)
        call("tgfr_fcfm_conv_fwd", ptr(rows), rows.stride(0), 256, b, ptr(pk),
             ptr(bias.float().contiguous()), ptr(pooled), ptr(code), m, _hip.stream())
        ctx.save_for_backward(rows, pk, code)
        ctx.cfg = (b, m, weight.dtype)
        ctx.mark_non_differentiable(code)
        return pooled

    @staticmethod
    def backward(ctx, gpool):
        rows, pk, code = ctx.saved_tensors
        b, m, wdtype = ctx.cfg
        gpool = gpool.float().contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dxr = torch.empty(b, 14, 14, 256, dtype=torch.float32, device=gpool.device)
            call("tgfr_fcfm_conv_dx", ptr(gpool), ptr(code), b, ptr(pk), ptr(dxr),
                 dxr.stride(0), 256, m, _hip.stream())
            dx = dxr.permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            n = (ctypes.c_longlong * 1)()
            rc = _hip.lib().tgfr_fcfm_conv_dw_ws(b, ctypes.addressof(n))
            if rc != 0:
                raise RuntimeError(f"tgfr_fcfm_conv_dw_ws failed with code {rc}")
            ws = torch.empty(int(n[0]), dtype=torch.float32, device=gpool.device)
            dwf = torch.empty(36, 256, 3, 3, dtype=torch.float32, device=gpool.device)
            dbf = torch.empty(36, dtype=torch.float32, device=gpool.device)
            call("tgfr_fcfm_conv_dw", ptr(rows), rows.stride(0), 256, ptr(gpool), ptr(code), b,
                 ptr(dwf), ptr(dbf), ptr(ws), m, _hip.stream())
            dw = dwf.to(wdtype) if ctx.needs_input_grad[1] else None
            db = dbf if ctx.needs_input_grad[2] else None
        return dx, dw, db, None


def conv_relu_pool(x, weight, bias, mode="fp32"):
    return ConvReluPool.apply(x, weight, bias, mode)


def conv_relu_pool_code(x, weight, bias, mode="fp32"):
    """The forward kernel alone (no autograd): (pooled, code), code the 2x2
    argmax 0..3 = dy*2+dx of each window, -1 where the ReLU blocks it."""
    with torch.no_grad():
        rows = x.float().permute(0, 2, 3, 1).contiguous()
        pk = torch.empty(_hip.lib().tgfr_fcfm_pack_elems(), dtype=torch.int16, device=x.device)
        call("tgfr_fcfm_pack", ptr(weight.float().contiguous()), ptr(pk), _hip.stream())
        pooled = torch.empty(x.shape[0], 36, 6, 6, dtype=torch.float32, device=x.device)
        code = torch.empty(x.shape[0], 36, 6, 6, dtype=torch.int8, device=x.device)
        call("tgfr_fcfm_conv_fwd", ptr(rows), rows.stride(0), 256, x.shape[0], ptr(pk),
             ptr(bias.float().contiguous()), ptr(pooled), ptr(code), _mode(mode), _hip.stream())
    return pooled, code


class MaxPool2CL(torch.autograd.Function):
    """MaxPool2d(2) of a channels-last map x [B, H*W, C] (Working's pool after
    its LayerNorm, fusion_nets.py:252) -> [B, C, H/2, W/2] (NCHW)."""

    @staticmethod
    def forward(ctx, x, h, w):
        b, hw, c = x.shape
        assert hw == h * w
        x = _aligned(x)
        y = torch.empty(b, c, h // 2, w // 2, dtype=torch.float32, device=x.device)
        idx = torch.empty(b, c, h // 2, w // 2, dtype=torch.uint8, device=x.device)
        call("tgfr_maxpool2_cl", ptr(x), b, h, w, c, ptr(y), ptr(idx), _hip.stream())
        ctx.save_for_backward(idx)
        ctx.cfg = (b, h, w, c)
        ctx.mark_non_differentiable(idx)
        return y

    @staticmethod
    def backward(ctx, dy):
        idx, = ctx.saved_tensors
        b, h, w, c = ctx.cfg
        dy = _aligned(dy)
        dx = torch.empty(b, h * w, c, dtype=torch.float32, device=dy.device)
        call("tgfr_maxpool2_cl_bwd", ptr(dy), ptr(idx), b, h, w, c, ptr(dx), _hip.stream())
        return dx, None, None


def maxpool2_cl(x, h, w):
    return MaxPool2CL.apply(x, h, w)


class Gram(torch.autograd.Function):
    """G = alpha * X^T X per sample for X [B, T, C] -> [B, C, C]: Working's
    word Gram matrix (fusion_nets.py:241), on the batched MFMA GEMM; the
    backward dX = alpha X (dG + dG^T) as two accumulating GEMMs."""

    @staticmethod
    def forward(ctx, x, alpha, mode):
        x = x.float()
        g = bgemm(x.transpose(1, 2), x, alpha=alpha, mode=mode)
        ctx.save_for_backward(x)
        ctx.cfg = (float(alpha), mode)
        return g

    @staticmethod
    def backward(ctx, dg):
        x, = ctx.saved_tensors
        alpha, mode = ctx.cfg
        dg = dg.float()
        dx = bgemm(x, dg, alpha=alpha, mode=mode)
        bgemm(x, dg.transpose(1, 2), out=dx, alpha=alpha, accumulate=True, mode=mode)
        return dx, None, None


def gram(x, alpha=1.0, mode="fp32"):
    return Gram.apply(x, alpha, mode)


class LinearRows(torch.autograd.Function):
    """y = x W^T + b (optionally ReLU) over the rows of x [..., K]: every
    nn.Linear / 1x1 conv of the head, on the split-bf16 MFMA GEMM."""

    @staticmethod
    def forward(ctx, x, weight, bias, relu, mode):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).float()
        w = weight.reshape(weight.shape[0], -1).float()
        mb = -(-x2.shape[0] // 64) * -(-w.shape[0] // 64)
        y = bgemm(x2.unsqueeze(0), w.t().unsqueeze(0), mode=mode,
                  bias=None if bias is None else bias.float().contiguous(), relu=relu,
                  ksplit=_ksplit(x2.shape[1], mb))[0]
        ctx.save_for_backward(x2, w, y if relu else None)
        ctx.cfg = (relu, mode, bias is not None, shape, weight.shape)
        return y.reshape(*shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w, y = ctx.saved_tensors
        relu, mode, has_bias, shape, wshape = ctx.cfg
        dy = dy.reshape(-1, w.shape[0]).float()
        if dy.stride(1) != 1:
            dy = dy.contiguous()
        dx = dw = db = None
        want_db = has_bias and ctx.needs_input_grad[2]
        if relu or want_db:
            rows, cols = dy.shape
            ws = torch.empty(-(-rows // 128) * cols, dtype=torch.float32, device=dy.device)
            db = torch.empty(cols, dtype=torch.float32, device=dy.device)
            dym = torch.empty_like(dy) if relu else None
            call("tgfr_bias_grad", ptr(dy), dy.stride(0), rows, cols, ptr(y),
                 y.stride(0) if relu else 0, ptr(dym), dym.stride(0) if relu else 0, ptr(db),
                 ptr(ws), ptr(_hip.counters(dy.device)), _hip.stream())
            if relu:
                dy = dym
            if not want_db:
                db = None
        if ctx.needs_input_grad[0]:
            mb = -(-dy.shape[0] // 64) * -(-w.shape[1] // 64)
            dx = bgemm(dy.unsqueeze(0), w.unsqueeze(0), mode=mode,
                       ksplit=_ksplit(w.shape[0], mb))[0].reshape(shape)
        if ctx.needs_input_grad[1]:
            mb = -(-w.shape[0] // 64) * -(-w.shape[1] // 64)
            dw = bgemm(dy.t().unsqueeze(0), x2.unsqueeze(0), mode=mode,
                       ksplit=_ksplit(x2.shape[0], mb))[0].reshape(wshape)
        return dx, dw, db, None, None


def linear_rows(x, weight, bias=None, relu=False, mode="fp32"):
    return LinearRows.apply(x, weight, bias, relu, mode)


class AttentionCore(torch.autograd.Function):
    """O = softmax(scale * Qr Kr^T) V per sample (fusion_nets.py:103-115) on
    packed projections, so the backward writes dQr/dKr/dV straight into the
    column slices of one packed gradient (no zero-fill + add per slice).

    px [N, HW, Cx] holds Qr in columns [0, cq) and V in [cv, Cx); Kr is
    columns [ck, ck + cq) of py [N, HW, Cy], or of px when py is None
    (self-attention).  Returns O [N, HW, Cx - cv].
    """

    @staticmethod
    def forward(ctx, px, py, cq, ck, cv, scale, mode):
        px = _rows(px.float())
        ky = px if py is None else _rows(py.float())
        qr, kr, v = px[..., :cq], ky[..., ck:ck + cq], px[..., cv:]
        nb, hw, _ = qr.shape
        c = v.shape[-1]
        ctx.small = _attn_small_fits(hw, cq, ck, cv, c, py is None)
        if ctx.small:
            # FCFM-sized: one fused launch (tgfr_attn_small_fwd), exact fp32
            o = torch.empty(nb, hw, c, dtype=torch.float32, device=px.device)
            p = torch.empty(nb, hw, hw, dtype=torch.float32, device=px.device)
            call("tgfr_attn_small_fwd", ptr(px), px.stride(0), px.stride(1),
                 None if py is None else ptr(ky), ky.stride(0), ky.stride(1), nb, hw, cq, ck,
                 cv, c, float(scale), ptr(o), o.stride(0), o.stride(1), ptr(p), _hip.stream())
            ctx.save_for_backward(px, None if py is None else ky, p)
            ctx.cfg = (float(scale), mode, cq, ck, cv)
            return o
        s = bgemm(qr, kr.transpose(1, 2), mode=mode)
        p = torch.empty_like(s)
        call("tgfr_attn_softmax", ptr(s), ptr(p), None, nb * hw, hw, hw, float(scale),
             _hip.stream())
        o = bgemm(p, v, mode=mode)
        ctx.save_for_backward(px, None if py is None else ky, p)
        ctx.cfg = (float(scale), mode, cq, ck, cv)
        return o

    @staticmethod
    def backward(ctx, do):
        px, py, p = ctx.saved_tensors
        scale, mode, cq, ck, cv = ctx.cfg
        ky = px if py is None else py
        qr, kr, v = px[..., :cq], ky[..., ck:ck + cq], px[..., cv:]
        do = _rows(do.float())
        nb, hw, _ = qr.shape
        if ctx.small:
            dpx = torch.empty_like(px)
            dky = None if py is None else torch.empty_like(py)
            if py is None:
                if ck != cq or cv != 2 * cq or px.shape[-1] != cv + v.shape[-1]:
                    dpx.zero_()
            else:
                if cv != cq:
                    dpx.zero_()
                if ck != 0 or cq != py.shape[-1]:
                    dky.zero_()
            g = dpx if dky is None else dky
            call("tgfr_attn_small_bwd", ptr(px), px.stride(0), px.stride(1),
                 None if py is None else ptr(ky), ky.stride(0), ky.stride(1), nb, hw, cq, ck,
                 cv, v.shape[-1], scale, ptr(p), ptr(do), do.stride(0), do.stride(1), ptr(dpx),
                 dpx.stride(0), dpx.stride(1), None if dky is None else ptr(dky), g.stride(0),
                 g.stride(1), _hip.stream())
            return dpx, dky, None, None, None, None, None
        dp = bgemm(do, v.transpose(1, 2), mode=mode)
        ds = torch.empty_like(dp)
        call("tgfr_attn_softmax_bwd", ptr(p), ptr(dp), ptr(ds), nb * hw, hw, hw, scale,
             _hip.stream())
        dpx = torch.empty_like(px)
        dky = dpx if py is None else torch.empty_like(py)
        if py is None:
            covered = ck == cq and cv == 2 * cq
        else:
            covered = cv == cq and ck == 0 and cq == py.shape[-1]
        if not covered:
            dpx.zero_()
            if py is not None:
                dky.zero_()
        bgemm(ds, kr, out=dpx[..., :cq], mode=mode)
        bgemm(ds.transpose(1, 2), qr, out=dky[..., ck:ck + cq], mode=mode)
        bgemm(p.transpose(1, 2), do, out=dpx[..., cv:], mode=mode)
        return dpx, (None if py is None else dky), None, None, None, None, None


def _rows(t):
    """t with unit element stride (a copy only when it has not)."""
    return t if t.stride(-1) == 1 else t.contiguous()


def _attn_small_fits(hw, cq, ck, cv, c, self_attn):
    """Whether tgfr_attn_small_fwd/_bwd take this shape: HW, C', C <= 64,
    and gradient column ranges that do not overlap (the kernel overwrites
    them)."""
    if max(hw, cq, c) > 64:
        return False
    if self_attn:
        return ck >= cq and cv >= cq and not (ck < cv + c and cv < ck + cq)
    return cv >= cq


def attention_core(px, py, cq, ck, cv, scale, mode="fp32"):
    return AttentionCore.apply(px, py, cq, ck, cv, scale, mode)


# ------------------------------------------------- batch norm -> linear ---
def _bn_linear_fwd(ctx, x, gamma, beta, weight, bias, bn, training, mode, out_bf16=False,
                   xhat_bf16=False, fold3=None, prep=None):
    """BatchNorm2d (batch or running statistics) folded into the following
    1x1 projection; returns y [N, HW, O] (fp32, or bf16 with out_bf16) and
    stores what _bn_linear_bwd needs on ctx.  xhat_bf16 (with out_bf16: the
    bf16 q/k/v path, no BN input gradient): the normalised map is written and
    kept in bf16 -- the values the bf16 GEMMs read from the fp32 map anyway.
    fold3 (three-part weight only): a callable (wp, bp, rows, c, g, beta, wf,
    bf) that launches the fold instead of tgfr_bn_fold3 (ImimFused folds it
    into IMIM's one weight-preparation launch; on an auxiliary stream beside
    the BN statistics it measured slower, 0.471 vs 0.457 ms per step)."""
    n, c, h, w_ = x.shape
    hw = h * w_
    o = sum(t.shape[0] for t in weight) if isinstance(weight, tuple) else weight.shape[0]
    x = x.float().contiguous()
    dev = x.device
    mean = torch.empty(c, dtype=torch.float32, device=dev)
    rstd = torch.empty_like(mean)
    xhat_bf16 = xhat_bf16 and out_bf16
    xhat = torch.empty(n, hw, c, dtype=torch.int16 if xhat_bf16 else torch.float32, device=dev)
    track = training and bn.track_running_stats and bn.running_mean is not None
    if training and track and bn.momentum is None:
        raise NotImplementedError("cumulative-average BatchNorm (momentum=None)")
    use_batch = training or bn.running_mean is None
    # the bf16 q/k/v path normalises inside the projection launch
    # (tgfr_bn_qkv_bf16): only the statistics here
    fused = (xhat_bf16 and isinstance(weight, tuple) and prep is not None and c == 256 and
             128 < hw <= 224 and hw % 4 == 0 and o % 256 == 0 and
             os.environ.get("TGFR_BN_QKV", "1") == "1")
    stats = (ptr(x), n, c, hw, float(bn.eps), float(bn.momentum or 0.0), int(use_batch),
             ptr(bn.running_mean) if (track or not use_batch) else None,
             ptr(bn.running_var) if (track or not use_batch) else None,
             ptr(bn.num_batches_tracked) if track else None, ptr(mean), ptr(rstd))
    # prep (ImimFused): the statistics launched together with the weight
    # preparation (tgfr_imim_prep), one launch for both
    prep = prep if fused else None
    if prep is None:
        call("tgfr_bn_stats" if fused else "tgfr_bn_fwd_cl_bf16" if xhat_bf16 else
             "tgfr_bn_fwd_cl", *stats, *(() if fused else (ptr(xhat),)), _hip.stream())
    g = gamma.float().contiguous()
    bf = torch.empty(o, dtype=torch.float32, device=dev)
    if isinstance(weight, tuple):
        # three projections read in place (tgfr_bn_fold3), no concatenated copy
        rows = weight[0].shape[0]
        w2 = tuple(w_.reshape(rows, c).float().contiguous() for w_ in weight)
        b2 = tuple(None if b_ is None else b_.float().contiguous() for b_ in bias)
        wf = torch.empty(o, c, dtype=torch.float32, device=dev)
        wfb = torch.empty(o, c, dtype=torch.int16, device=dev) if fused else None
        wp = (ctypes.c_void_p * 3)(*[ptr(t) for t in w2])
        bp = (ctypes.c_void_p * 3)(*[ptr(t) for t in b2])
        if prep is not None:
            prep(stats, wp, bp, rows, c, g, beta.float().contiguous(), wf, wfb, bf)
        elif fold3 is not None:
            fold3(wp, bp, rows, c, g, beta.float().contiguous(), wf, bf)
        else:
            call("tgfr_bn_fold3", ctypes.addressof(wp), ctypes.addressof(bp), rows, c, ptr(g),
                 ptr(beta.float().contiguous()), ptr(wf), ptr(bf), _hip.stream())
    else:
        w2 = weight.reshape(o, c).float().contiguous()
        wf = torch.empty_like(w2)
        call("tgfr_bn_fold", ptr(w2), ptr(None if bias is None else bias.float().contiguous()),
             o, c, ptr(g), ptr(beta.float().contiguous()), ptr(wf), ptr(bf), _hip.stream())
    rows = n * hw
    if fused:
        y = torch.empty(rows, o, dtype=torch.int16, device=dev)
        call("tgfr_bn_qkv_bf16", ptr(x), n, c, hw, ptr(mean), ptr(rstd), ptr(wfb), ptr(bf), o,
             ptr(y), ptr(xhat), _hip.stream())
    elif out_bf16:
        y = torch.empty(rows, o, dtype=torch.int16, device=dev)
        call("tgfr_linear_bf16io" if xhat_bf16 else "tgfr_linear_bf16out", ptr(xhat), c, rows, c,
             ptr(wf), c, ptr(bf), o, ptr(y), o, _hip.stream())
    else:
        mb = -(-rows // 64) * -(-o // 64)
        y = bgemm(xhat.view(1, rows, c), wf.t().unsqueeze(0), bias=bf, mode=mode,
                  ksplit=_ksplit(c, mb))[0]
    ctx.bn_saved = (xhat, w2, wf, g, beta.float().contiguous(), rstd)
    wshape = tuple(t.shape for t in weight) if isinstance(weight, tuple) else weight.shape
    ctx.bn_cfg = (mode, bias is not None, x.shape, wshape, use_batch)
    return y.view(n, hw, o)


def _bn_linear_bwd(ctx, dy, want_dx):
    """(dx, dgamma, dbeta, dweight, dbias) of _bn_linear_fwd given dy [N, HW, O]."""
    xhat, w2, wf, g, bt, rstd = ctx.bn_saved
    mode, has_bias, xshape, wshape, use_batch = ctx.bn_cfg
    n, hw, c = xhat.shape
    o = wf.shape[0]
    rows = n * hw
    dp = dy.reshape(rows, o).float()
    if dp.stride(1) != 1 or dp.stride(0) != o:
        dp = dp.contiguous()
    dev = dp.device
    s = torch.empty(o, dtype=torch.float32, device=dev)
    ws = torch.empty(-(-rows // 128) * o, dtype=torch.float32, device=dev)
    call("tgfr_bias_grad", ptr(dp), o, rows, o, None, 0, None, 0, ptr(s), ptr(ws),
         ptr(_hip.counters(dev)), _hip.stream())
    mb = -(-o // 64) * -(-c // 64)
    gm = bgemm(dp.t().unsqueeze(0), xhat.view(1, rows, c), mode=mode,
               ksplit=_ksplit(rows, mb))[0]
    _, dgamma, dbeta, dw, db = _bn_unfold(ctx, gm, s)
    dx = None
    if want_dx:
        # d xhat = dp W'; BN input gradient (only when the map itself is trained)
        dxh = bgemm(dp.unsqueeze(0), wf.unsqueeze(0), mode=mode)[0]
        dx = torch.empty(xshape, dtype=torch.float32, device=dev)
        call("tgfr_bn_bwd_cl", ptr(dxh), ptr(xhat), ptr(rstd), n, c, hw, int(use_batch),
             ptr(dx), _hip.stream())
    return dx, dgamma, dbeta, dw, db


def _bn_unfold(ctx, gm, s):
    """(None, dgamma, dbeta, dweight, dbias) from G = dy^T xhat [O, C] and
    s = colsum(dy) [O] (tgfr_bn_unfold); with the weight in 3 parts, dweight
    and dbias are tuples of the parts' slices of the packed gradients."""
    xhat, w2, wf, g, bt, rstd = ctx.bn_saved
    mode, has_bias, xshape, wshape, use_batch = ctx.bn_cfg
    o, c = wf.shape
    dev = gm.device
    dw = torch.empty(o, c, dtype=torch.float32, device=dev)
    dgamma = torch.empty(c, dtype=torch.float32, device=dev)
    dbeta = torch.empty_like(dgamma)
    uws = torch.empty(2 * -(-o // 16) * c, dtype=torch.float32, device=dev)
    if isinstance(w2, tuple):
        rows = w2[0].shape[0]
        wp = (ctypes.c_void_p * 3)(*[ptr(t) for t in w2])
        call("tgfr_bn_unfold3", ptr(gm), ptr(s), ctypes.addressof(wp), rows, c, ptr(g), ptr(bt),
             ptr(dw), ptr(dgamma), ptr(dbeta), ptr(uws), ptr(_hip.counters(dev)), _hip.stream())
        dws = tuple(dw[k * rows:(k + 1) * rows].view(wshape[k]) for k in range(3))
        dbs = tuple(s[k * rows:(k + 1) * rows] for k in range(3)) if has_bias else None
        return None, dgamma, dbeta, dws, dbs
    call("tgfr_bn_unfold", ptr(gm), ptr(s), ptr(w2), o, c, ptr(g), ptr(bt), ptr(dw),
         ptr(dgamma), ptr(dbeta), ptr(uws), ptr(_hip.counters(dev)), _hip.stream())
    return None, dgamma, dbeta, dw.reshape(wshape), (s if has_bias else None)


class BNLinear(torch.autograd.Function):
    """y[n, hw] = W bn(x)[n, :, hw] + b for x [N, C, H, W] (NCHW), returned
    channels-last [N, HW, O]: nn.BatchNorm2d followed by a 1x1 projection
    (IMIM bn_img -> SelfAttention q/k/v, models/models.py:397-398), with the BN
    affine folded into the projection (tgfr_bn.hip)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, weight, bias, bn, training, mode):
        return _bn_linear_fwd(ctx, x, gamma, beta, weight, bias, bn, training, mode)

    @staticmethod
    def backward(ctx, dy):
        return _bn_linear_bwd(ctx, dy, ctx.needs_input_grad[0]) + (None, None, None)


class ImimAttention(torch.autograd.Function):
    """IMIM's bn_img -> SelfAttention (models/models.py:397-398,
    fusion_nets.py:93-118) in bf16 mode as one autograd node: BN folded into
    the packed [Qr | Kr | V] projection, which is written in bf16 and read in
    place by the fused attention kernels (tgfr_attn_fwd / _bwd); the packed
    projection never exists in fp32.  Returns O [N, HW, 256] fp32."""

    @staticmethod
    def forward(ctx, x, gamma, beta, wk, wq, wv, bk, bq, bv, bn, training, scale):
        # without a BN input gradient (the frozen backbone's map) xhat stays bf16
        px = _bn_linear_fwd(ctx, x, gamma, beta, (wk, wq, wv), (bk, bq, bv), bn, training,
                            "bf16", out_bf16=True, xhat_bf16=not ctx.needs_input_grad[0])
        nb, hw, _ = px.shape
        o = torch.empty(nb, hw, 256, dtype=torch.float32, device=px.device)
        lse = torch.empty(nb * hw, dtype=torch.float32, device=px.device)
        call("tgfr_attn_fwd", ptr(px), ptr(px[..., 256:]), ptr(px[..., 512:]), px.stride(1),
             px.stride(0), nb, hw, float(scale), ptr(o), o.stride(1), o.stride(0), ptr(lse),
             _hip.stream())
        ctx.save_for_backward(px, o, lse)
        ctx.scale = float(scale)
        return o

    @staticmethod
    def backward(ctx, do):
        px, o, lse = ctx.saved_tensors
        nb, hw, _ = px.shape
        do = do.float().contiguous()
        out = (ctypes.c_longlong * 1)()
        rc = _hip.lib().tgfr_attn_bwd_ws(nb, hw, ctypes.addressof(out))
        if rc != 0:
            raise RuntimeError(f"tgfr_attn_bwd_ws failed with code {rc}")
        ws = torch.empty(int(out[0]), dtype=torch.uint8, device=px.device)
        dpx = torch.empty(nb, hw, 768, dtype=torch.int16, device=px.device)     # bf16
        call("tgfr_attn_bwd", ptr(px), ptr(px[..., 256:]), ptr(px[..., 512:]), px.stride(1),
             px.stride(0), nb, hw, ctx.scale, ptr(o), ptr(do), do.stride(1), do.stride(0),
             ptr(lse), ptr(dpx), ptr(dpx[..., 256:]), ptr(dpx[..., 512:]), dpx.stride(1),
             dpx.stride(0), ptr(ws), _hip.stream())
        if ctx.needs_input_grad[0]:
            # the BN input gradient needs dp W' (the reference's frozen-backbone
            # step never asks for it): the fp32 path
            dpf = (dpx.to(torch.int32) << 16).view(torch.float32)
            return _imim_grads(_bn_linear_bwd(ctx, dpf, True))
        # G = dp^T xhat and colsum(dp) in one bf16 weight-gradient launch
        xhat = ctx.bn_saved[0]
        rows, c = nb * hw, xhat.shape[2]
        n = dpx.shape[2]
        out = (ctypes.c_longlong * 1)()
        rc = _hip.lib().tgfr_dw_bf16_ws(rows, n, c, ctypes.addressof(out))
        if rc != 0:
            raise RuntimeError(f"tgfr_dw_bf16_ws failed with code {rc}")
        gws = torch.empty(int(out[0]), dtype=torch.float32, device=px.device)
        gm = torch.empty(n, c, dtype=torch.float32, device=px.device)
        s = torch.empty(n, dtype=torch.float32, device=px.device)
        call("tgfr_dw_bf16", ptr(dpx), ptr(xhat), int(xhat.dtype == torch.float32), rows, n, c,
             ptr(gm), ptr(s), ptr(gws), _hip.stream())
        return _imim_grads(_bn_unfold(ctx, gm, s))


def _imim_grads(g):
    """(dx, dgamma, dbeta, (dwk, dwq, dwv), (dbk, dbq, dbv) or None) ->
    ImimAttention.backward's flat tuple."""
    dx, dgamma, dbeta, dws, dbs = g
    return (dx, dgamma, dbeta) + tuple(dws) + (tuple(dbs) if dbs else (None,) * 3) + \
        (None, None, None)


def imim_attention(x, bn, sa, scale):
    """bf16 mode: bn -> q/k/v projections of SelfAttention `sa` (key role,
    query role, value; read in place) -> fused self-attention; returns
    O [N, HW, 256]."""
    return ImimAttention.apply(x, bn.weight, bn.bias, sa.key_proj.weight, sa.query_proj.weight,
                               sa.value_proj.weight, sa.key_proj.bias, sa.query_proj.bias,
                               sa.value_proj.bias, bn, bn.training, scale)


def bn_linear(x, bn, weight, bias, mode="fp32"):
    """BatchNorm2d `bn` (its training flag and running buffers) then the
    projection; returns [N, HW, O]."""
    return BNLinear.apply(x, bn.weight, bn.bias, weight, bias, bn, bn.training, mode)


# ------------------------------------------------------------ layer norm ---
def _aligned(t):
    t = t.float().contiguous()
    return t if t.data_ptr() % 16 == 0 else t.clone()


def ln_ws_floats(rows, e, ch=0, backward=True):
    out = (ctypes.c_longlong * 1)()
    rc = _hip.lib().tgfr_ln_ws_floats(int(rows), int(e), int(ch), int(backward),
                                      ctypes.addressof(out))
    if rc != 0:
        raise RuntimeError(f"tgfr_ln_ws_floats failed with code {rc}")
    return int(out[0])


class LayerNormRows(torch.autograd.Function):
    """Per-sample LayerNorm over all trailing elements with an elementwise
    affine of the same size (nn.LayerNorm([C, H, W]), models.py:388/:401).
    ch > 0: x rows are channels-last [HW, ch] while weight/bias keep the
    reference's [ch, H, W] layout (the forward makes channels-last copies in
    its workspace, which the backward reuses)."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps, ch):
        rows = x.shape[0]
        x2 = _aligned(x.reshape(rows, -1))
        e = x2.shape[1]
        assert weight.numel() == e and bias.numel() == e
        w, b = _aligned(weight.reshape(-1)), _aligned(bias.reshape(-1))
        ws = torch.empty(ln_ws_floats(rows, e, ch), dtype=torch.float32, device=x.device)
        y = torch.empty_like(x2)
        call("tgfr_ln_fwd", ptr(x2), rows, e, ptr(w), ptr(b), float(eps), int(ch), ptr(y),
             ptr(ws), _hip.stream())
        ctx.save_for_backward(x2, w, ws)
        ctx.shapes = (x.shape, weight.shape, int(ch))
        return y.reshape(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w, ws = ctx.saved_tensors
        xshape, wshape, ch = ctx.shapes
        rows, e = x2.shape
        dy = _aligned(dy.reshape(rows, e))
        dx = torch.empty_like(x2)
        dw = torch.empty(e, dtype=torch.float32, device=x2.device)
        db = torch.empty_like(dw)
        call("tgfr_ln_bwd", ptr(dy), ptr(x2), rows, e, ptr(w), ch, ptr(ws), ptr(dx), ptr(dw),
             ptr(db), _hip.stream())
        return dx.reshape(xshape), dw.reshape(wshape), db.reshape(wshape), None, None


def layer_norm_rows(x, weight, bias, eps=1e-5, ch=0):
    return LayerNormRows.apply(x, weight, bias, eps, ch)


# ------------------------------------------------------------- IMIM tail ---
_TAIL_C, _TAIL_H, _TAIL_D = 256, 128, 256


def tail_dw_ws_floats(rows):
    out = (ctypes.c_longlong * 1)()
    rc = _hip.lib().tgfr_tail_dw_ws(int(rows), ctypes.addressof(out))
    if rc != 0:
        raise RuntimeError(f"tgfr_tail_dw_ws failed with code {rc}")
    return int(out[0])


class ImimTail(torch.autograd.Function):
    """IMIM after its LayerNorm (models/models.py:399-405 with ProjectionHead
    :98-120): relu(conv1x1_1) -> relu(conv1x1_2) -> project_local -> L2 norm,
    over channels-last rows, as ONE fused bf16 kernel each way (tgfr_tail.hip)
    plus one weight-gradient launch.  Activations saved for the backward are
    bf16 (Z, H1, H2), the operands the bf16 GEMMs consume anyway."""

    @staticmethod
    def forward(ctx, z, w1, b1, w2, b2, wp, bp, eps, rows_spec=None):
        shape = z.shape
        assert shape[-1] == _TAIL_C and tuple(w1.shape[:2]) == (_TAIL_H, _TAIL_C)
        assert tuple(w2.shape[:2]) == (_TAIL_C, _TAIL_H) and tuple(wp.shape) == (_TAIL_D, _TAIL_C)
        z2 = _aligned(z.reshape(-1, _TAIL_C))
        rows, dev = z2.shape[0], z2.device
        pk = torch.empty(_hip.lib().tgfr_tail_pack_elems(), dtype=torch.int16, device=dev)
        call("tgfr_tail_pack", ptr(_aligned(w1.reshape(_TAIL_H, _TAIL_C))),
             ptr(_aligned(w2.reshape(_TAIL_C, _TAIL_H))), ptr(_aligned(wp)), ptr(pk),
             _hip.stream())
        r = torch.empty(rows, _TAIL_D, dtype=torch.float32, device=dev)
        zb = torch.empty(rows, _TAIL_C, dtype=torch.int16, device=dev)
        h1 = torch.empty(rows, _TAIL_H, dtype=torch.int16, device=dev)
        h2 = torch.empty(rows, _TAIL_C, dtype=torch.int16, device=dev)
        inv = torch.empty(rows, dtype=torch.float32, device=dev)
        # rows_spec = (rows per item, padded rows, fp16): R also in the
        # word<->region operand layout (prep_rows' hi plane and norms)
        rr = rn = None
        per, pad, f16 = rows_spec if rows_spec else (0, 0, False)
        if rows_spec:
            rr = torch.empty(rows // per, pad, _TAIL_D, dtype=torch.int16, device=dev)
            rn = torch.empty(rows // per, pad, dtype=torch.float32, device=dev)
        call("tgfr_tail_fwd", ptr(z2), _TAIL_C, rows, ptr(pk), ptr(_aligned(b1)),
             ptr(_aligned(b2)), ptr(_aligned(bp)), float(eps), ptr(r), _TAIL_D, ptr(zb), ptr(h1),
             ptr(h2), ptr(inv), ptr(rr), ptr(rn), per, pad, int(bool(f16)), _hip.stream())
        ctx.save_for_backward(r, inv, pk, zb, h1, h2)
        ctx.cfg = (float(eps), shape, w1.shape, w2.shape)
        out = r.reshape(*shape[:-1], _TAIL_D)
        if rows_spec:
            # (no zero-filled gradients for the operand rows: that was a 7 MB
            # fill kernel per step)
            ctx.mark_non_differentiable(rr, rn)
            ctx.set_materialize_grads(False)
            return out, rr, rn
        return out

    @staticmethod
    def backward(ctx, dr, *unused):
        if dr is None:                       # (grads not materialised: nothing flows)
            return (None,) * 9
        r, inv, pk, zb, h1, h2 = ctx.saved_tensors
        eps, shape, w1shape, w2shape = ctx.cfg
        rows, dev = r.shape[0], r.device
        dr2 = _aligned(dr.reshape(rows, _TAIL_D))
        dz = torch.empty(rows, _TAIL_C, dtype=torch.float32, device=dev)
        dp = torch.empty(rows, _TAIL_D, dtype=torch.int16, device=dev)
        dh2 = torch.empty(rows, _TAIL_C, dtype=torch.int16, device=dev)
        dh1 = torch.empty(rows, _TAIL_H, dtype=torch.int16, device=dev)
        call("tgfr_tail_bwd", ptr(dr2), _TAIL_D, ptr(r), _TAIL_D, ptr(inv), rows, eps, ptr(pk),
             ptr(h1), ptr(h2), ptr(dz), _TAIL_C, ptr(dp), ptr(dh2), ptr(dh1), _hip.stream())
        ws = torch.empty(tail_dw_ws_floats(rows), dtype=torch.float32, device=dev)
        dwp = torch.empty(_TAIL_D, _TAIL_C, dtype=torch.float32, device=dev)
        dbp = torch.empty(_TAIL_D, dtype=torch.float32, device=dev)
        dw2 = torch.empty(_TAIL_C, _TAIL_H, dtype=torch.float32, device=dev)
        db2 = torch.empty(_TAIL_C, dtype=torch.float32, device=dev)
        dw1 = torch.empty(_TAIL_H, _TAIL_C, dtype=torch.float32, device=dev)
        db1 = torch.empty(_TAIL_H, dtype=torch.float32, device=dev)
        call("tgfr_tail_dw", ptr(dp), ptr(h2), ptr(dh2), ptr(h1), ptr(dh1), ptr(zb), rows,
             ptr(dwp), ptr(dbp), ptr(dw2), ptr(db2), ptr(dw1), ptr(db1), ptr(ws), _hip.stream())
        return (dz.reshape(shape), dw1.reshape(w1shape), db1, dw2.reshape(w2shape), db2, dwp,
                dbp, None, None)


class ImimLnTail(torch.autograd.Function):
    """IMIM from the attention output on: LayerNorm([C, H, W]) (models/
    models.py:401) -> relu(conv1x1_1) -> relu(conv1x1_2) -> project_local ->
    L2 norm (:399-405, ProjectionHead :98-120) with the LayerNorm fused into
    the tail's kernels (tgfr_ln_tail_fwd / _bwd): the normalised map is never
    written, and the LayerNorm backward's first pass (per-sample sums of dZ w
    and dZ w xhat) runs in the tail backward's epilogue.  Forward: the weight
    pack (+ the affine maps as channels-last rows), the LayerNorm slice
    moments, the tail; backward: the tail (+ LN sums), the LN input gradient,
    its dw/db reduce, the tail weight gradients."""

    @staticmethod
    def forward(ctx, x, lnw, lnb, w1, b1, w2, b2, wp, bp, ln_eps, eps, rows_spec=None):
        n, hw, c = x.shape
        assert c == _TAIL_C and tuple(w1.shape[:2]) == (_TAIL_H, _TAIL_C)
        assert tuple(w2.shape[:2]) == (_TAIL_C, _TAIL_H) and tuple(wp.shape) == (_TAIL_D, _TAIL_C)
        assert lnw.numel() == hw * c and lnb.numel() == hw * c
        x2 = _aligned(x.reshape(-1, c))
        rows, dev = x2.shape[0], x2.device
        out = (ctypes.c_longlong * 1)()
        rc = _hip.lib().tgfr_ln_tail_ws(rows, hw, ctypes.addressof(out))
        if rc != 0:
            raise RuntimeError(f"tgfr_ln_tail_ws failed with code {rc}")
        ws = torch.empty(int(out[0]), dtype=torch.float32, device=dev)
        pk = torch.empty(_hip.lib().tgfr_tail_pack_elems(), dtype=torch.int16, device=dev)
        call("tgfr_tail_pack_ln", ptr(_aligned(w1.reshape(_TAIL_H, _TAIL_C))),
             ptr(_aligned(w2.reshape(_TAIL_C, _TAIL_H))), ptr(_aligned(wp)),
             ptr(_aligned(lnw.reshape(-1))), ptr(_aligned(lnb.reshape(-1))), rows, hw, ptr(pk),
             ptr(ws), _hip.stream())
        r = torch.empty(rows, _TAIL_D, dtype=torch.float32, device=dev)
        zb = torch.empty(rows, _TAIL_C, dtype=torch.int16, device=dev)
        h1 = torch.empty(rows, _TAIL_H, dtype=torch.int16, device=dev)
        h2 = torch.empty(rows, _TAIL_C, dtype=torch.int16, device=dev)
        inv = torch.empty(rows, dtype=torch.float32, device=dev)
        rr = rn = None
        per, pad, f16 = rows_spec if rows_spec else (0, 0, False)
        if rows_spec:
            rr = torch.empty(rows // per, pad, _TAIL_D, dtype=torch.int16, device=dev)
            rn = torch.empty(rows // per, pad, dtype=torch.float32, device=dev)
        call("tgfr_ln_tail_fwd", ptr(x2), rows, hw, float(ln_eps), ptr(ws), ptr(pk),
             ptr(_aligned(b1)), ptr(_aligned(b2)), ptr(_aligned(bp)), float(eps), ptr(r), _TAIL_D,
             ptr(zb), ptr(h1), ptr(h2), ptr(inv), ptr(rr), ptr(rn), per, pad, int(bool(f16)),
             _hip.stream())
        ctx.save_for_backward(x2, r, inv, pk, zb, h1, h2, ws)
        ctx.cfg = (float(eps), x.shape, hw, lnw.shape, w1.shape, w2.shape)
        out_r = r.reshape(n, hw, _TAIL_D)
        if rows_spec:
            ctx.mark_non_differentiable(rr, rn)
            ctx.set_materialize_grads(False)
            return out_r, rr, rn
        return out_r

    @staticmethod
    def backward(ctx, dr, *unused):
        if dr is None:
            return (None,) * 12
        x2, r, inv, pk, zb, h1, h2, ws = ctx.saved_tensors
        eps, xshape, hw, lnshape, w1shape, w2shape = ctx.cfg
        rows, dev = r.shape[0], r.device
        dr2 = _aligned(dr.reshape(rows, _TAIL_D))
        dz = torch.empty(rows, _TAIL_C, dtype=torch.float32, device=dev)
        dp = torch.empty(rows, _TAIL_D, dtype=torch.int16, device=dev)
        dh2 = torch.empty(rows, _TAIL_C, dtype=torch.int16, device=dev)
        dh1 = torch.empty(rows, _TAIL_H, dtype=torch.int16, device=dev)
        dx = torch.empty_like(x2)
        dlnw = torch.empty(hw * _TAIL_C, dtype=torch.float32, device=dev)
        dlnb = torch.empty_like(dlnw)
        call("tgfr_ln_tail_bwd", ptr(dr2), ptr(r), ptr(inv), rows, eps, ptr(pk), ptr(h1),
             ptr(h2), ptr(x2), hw, ptr(ws), ptr(dz), ptr(dp), ptr(dh2), ptr(dh1), ptr(dx),
             ptr(dlnw), ptr(dlnb), _hip.stream())
        wsd = torch.empty(tail_dw_ws_floats(rows), dtype=torch.float32, device=dev)
        dwp = torch.empty(_TAIL_D, _TAIL_C, dtype=torch.float32, device=dev)
        dbp = torch.empty(_TAIL_D, dtype=torch.float32, device=dev)
        dw2 = torch.empty(_TAIL_C, _TAIL_H, dtype=torch.float32, device=dev)
        db2 = torch.empty(_TAIL_C, dtype=torch.float32, device=dev)
        dw1 = torch.empty(_TAIL_H, _TAIL_C, dtype=torch.float32, device=dev)
        db1 = torch.empty(_TAIL_H, dtype=torch.float32, device=dev)
        call("tgfr_tail_dw", ptr(dp), ptr(h2), ptr(dh2), ptr(h1), ptr(dh1), ptr(zb), rows,
             ptr(dwp), ptr(dbp), ptr(dw2), ptr(db2), ptr(dw1), ptr(db1), ptr(wsd), _hip.stream())
        return (dx.reshape(xshape), dlnw.reshape(lnshape), dlnb.reshape(lnshape),
                dw1.reshape(w1shape), db1, dw2.reshape(w2shape), db2, dwp, dbp, None, None, None)


class ImimFused(torch.autograd.Function):
    """The whole IMIM head in bf16 / fp16 mode (models/models.py:397-405:
    bn_img -> SelfAttention -> LayerNorm -> conv1x1_1 -> ReLU -> conv1x1_2 ->
    ReLU -> project_local -> L2 norm) as ONE autograd node, for a frozen input
    map (no BN input gradient, the trainers' case).  Against ImimAttention ->
    ImimLnTail it saves two launches per step: the BN fold, the tail weight
    pack and the LayerNorm affine transposes are one launch (tgfr_imim_pack),
    and the LayerNorm backward writes the attention backward's operands
    (bf16 dO and D = rowsum(dO * O)) itself (tgfr_ln_tail_bwd_att ->
    tgfr_attn_bwd_prepped), so the fp32 dO never exists.
    The attention forward also writes the LayerNorm's per-tile moments
    (tgfr_attn_fwd_ln), so no statistics pass runs either.
    Forward: BN statistics + bf16 xhat, the pack, the q/k/v GEMM, attention
    (+ LN moments), the fused tail (6 launches).  Backward: tail + LN sums,
    LN input gradient (as attention operands), attention dK/dV, dQ, the
    tail's and the q/k/v projection's weight gradients in one launch (+ a
    reduce that also sums the LN dw/db partials, tgfr_imim_dw_ln), BN unfold
    (7 launches; TGFR_LN_DW_DEFER=0: the LN dw/db reduce as its own launch)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, wk, wq, wv, bk, bq, bv, lnw, lnb, w1, b1, w2, b2, wp, bp,
                bn, training, scale, ln_eps, eps, rows_spec=None):
        nb, c, h, w_ = x.shape
        hw = h * w_
        rows = nb * hw
        dev = x.device
        out = (ctypes.c_longlong * 1)()
        rc = _hip.lib().tgfr_ln_tail_ws(rows, hw, ctypes.addressof(out))
        if rc != 0:
            raise RuntimeError(f"tgfr_ln_tail_ws failed with code {rc}")
        ws = torch.empty(int(out[0]), dtype=torch.float32, device=dev)
        pk = torch.empty(_hip.lib().tgfr_tail_pack_elems(), dtype=torch.int16, device=dev)
        tw = (_aligned(w1.reshape(_TAIL_H, _TAIL_C)), _aligned(w2.reshape(_TAIL_C, _TAIL_H)),
              _aligned(wp), _aligned(lnw.reshape(-1)), _aligned(lnb.reshape(-1)))

        def fold3(wptr, bptr, qrows, cc, g, bt, wf, bf):
            call("tgfr_imim_pack", ctypes.addressof(wptr), ctypes.addressof(bptr), qrows, cc,
                 ptr(g), ptr(bt), ptr(wf), ptr(bf), *[ptr(t) for t in tw], rows, hw, ptr(pk),
                 ptr(ws), _hip.stream())

        def prep(stats, wptr, bptr, qrows, cc, g, bt, wf, wfb, bf):
            x_, n_, c_, hw_, *rest = stats
            call("tgfr_imim_prep", x_, n_, hw_, *rest, ctypes.addressof(wptr),
                 ctypes.addressof(bptr), qrows, cc, ptr(g), ptr(bt), ptr(wf), ptr(wfb), ptr(bf),
                 *[ptr(t) for t in tw], rows, hw, ptr(pk), ptr(ws), _hip.stream())

        px = _bn_linear_fwd(ctx, x, gamma, beta, (wk, wq, wv), (bk, bq, bv), bn, training,
                            "bf16", out_bf16=True, xhat_bf16=True, fold3=fold3,
                            prep=prep if os.environ.get("TGFR_IMIM_PREP", "1") == "1" else None)
        o = torch.empty(nb, hw, _TAIL_C, dtype=torch.float32, device=dev)
        lse = torch.empty(rows, dtype=torch.float32, device=dev)
        # (the attention forward also leaves the LayerNorm's tile moments in ws)
        call("tgfr_attn_fwd_ln", ptr(px), ptr(px[..., 256:]), ptr(px[..., 512:]), px.stride(1),
             px.stride(0), nb, hw, float(scale), ptr(o), ptr(lse), ptr(ws), _hip.stream())
        r = torch.empty(rows, _TAIL_D, dtype=torch.float32, device=dev)
        zb = torch.empty(rows, _TAIL_C, dtype=torch.int16, device=dev)
        h1 = torch.empty(rows, _TAIL_H, dtype=torch.int16, device=dev)
        h2 = torch.empty(rows, _TAIL_C, dtype=torch.int16, device=dev)
        inv = torch.empty(rows, dtype=torch.float32, device=dev)
        rr = rn = None
        per, pad, f16 = rows_spec if rows_spec else (0, 0, False)
        if rows_spec:
            rr = torch.empty(rows // per, pad, _TAIL_D, dtype=torch.int16, device=dev)
            rn = torch.empty(rows // per, pad, dtype=torch.float32, device=dev)
        call("tgfr_ln_tail_fwd_att", ptr(o), rows, hw, float(ln_eps), ptr(ws), ptr(pk),
             ptr(_aligned(b1)), ptr(_aligned(b2)), ptr(_aligned(bp)), float(eps), ptr(r), _TAIL_D,
             ptr(zb), ptr(h1), ptr(h2), ptr(inv), ptr(rr), ptr(rn), per, pad, int(bool(f16)),
             _hip.stream())
        ctx.save_for_backward(px, o, lse, r, inv, pk, zb, h1, h2, ws)
        ctx.cfg = (float(scale), float(eps), hw, lnw.shape, w1.shape, w2.shape)
        out_r = r.reshape(nb, hw, _TAIL_D)
        if rows_spec:
            ctx.mark_non_differentiable(rr, rn)
            ctx.set_materialize_grads(False)
            return out_r, rr, rn
        return out_r

    @staticmethod
    def backward(ctx, dr, *unused):
        if dr is None:
            return (None,) * 23
        px, o, lse, r, inv, pk, zb, h1, h2, ws = ctx.saved_tensors
        scale, eps, hw, lnshape, w1shape, w2shape = ctx.cfg
        nb = px.shape[0]
        rows, dev = r.shape[0], r.device
        dr2 = _aligned(dr.reshape(rows, _TAIL_D))
        out = (ctypes.c_longlong * 1)()
        rc = _hip.lib().tgfr_attn_bwd_ws(nb, hw, ctypes.addressof(out))
        if rc != 0:
            raise RuntimeError(f"tgfr_attn_bwd_ws failed with code {rc}")
        aws = torch.empty(int(out[0]), dtype=torch.uint8, device=dev)
        dz = torch.empty(rows, _TAIL_C, dtype=torch.int16, device=dev)   # bf16 dZ scratch
        dp = torch.empty(rows, _TAIL_D, dtype=torch.int16, device=dev)
        dh2 = torch.empty(rows, _TAIL_C, dtype=torch.int16, device=dev)
        dh1 = torch.empty(rows, _TAIL_H, dtype=torch.int16, device=dev)
        dlnw = torch.empty(hw * _TAIL_C, dtype=torch.float32, device=dev)
        dlnb = torch.empty_like(dlnw)
        # (deferred: the LayerNorm's dw / db partials are reduced by the weight
        # gradients' reduce launch below, tgfr_imim_dw_ln)
        defer = os.environ.get("TGFR_LN_DW_DEFER", "1") == "1"
        call("tgfr_ln_tail_bwd_att", ptr(dr2), ptr(r), ptr(inv), rows, eps, ptr(pk), ptr(h1),
             ptr(h2), ptr(o), hw, ptr(ws), ptr(dz), ptr(dp), ptr(dh2), ptr(dh1), ptr(aws),
             None if defer else ptr(dlnw), None if defer else ptr(dlnb), _hip.stream())
        dpx = torch.empty(nb, hw, 768, dtype=torch.int16, device=dev)
        call("tgfr_attn_bwd_prepped", ptr(px), ptr(px[..., 256:]), ptr(px[..., 512:]),
             px.stride(1), px.stride(0), nb, hw, scale, ptr(lse), ptr(dpx), ptr(dpx[..., 256:]),
             ptr(dpx[..., 512:]), dpx.stride(1), dpx.stride(0), ptr(aws), _hip.stream())
        # the tail's and the q/k/v projection's weight gradients in one launch
        xhat = ctx.bn_saved[0]
        c = xhat.shape[2]
        n = dpx.shape[2]
        rc = _hip.lib().tgfr_imim_dw_ws(rows, n, c, ctypes.addressof(out))
        if rc != 0:
            raise RuntimeError(f"tgfr_imim_dw_ws failed with code {rc}")
        wsd = torch.empty(int(out[0]), dtype=torch.float32, device=dev)
        dwp = torch.empty(_TAIL_D, _TAIL_C, dtype=torch.float32, device=dev)
        dbp = torch.empty(_TAIL_D, dtype=torch.float32, device=dev)
        dw2 = torch.empty(_TAIL_C, _TAIL_H, dtype=torch.float32, device=dev)
        db2 = torch.empty(_TAIL_C, dtype=torch.float32, device=dev)
        dw1 = torch.empty(_TAIL_H, _TAIL_C, dtype=torch.float32, device=dev)
        db1 = torch.empty(_TAIL_H, dtype=torch.float32, device=dev)
        gm = torch.empty(n, c, dtype=torch.float32, device=dev)
        s = torch.empty(n, dtype=torch.float32, device=dev)
        dw_args = (ptr(dp), ptr(h2), ptr(dh2), ptr(h1), ptr(dh1), ptr(zb), rows, ptr(dwp),
                   ptr(dbp), ptr(dw2), ptr(db2), ptr(dw1), ptr(db1), ptr(dpx), ptr(xhat), n, c,
                   ptr(gm), ptr(s))
        if defer:
            call("tgfr_imim_dw_ln", *dw_args, ptr(ws), hw, ptr(dlnw), ptr(dlnb), ptr(wsd),
                 _hip.stream())
        else:
            call("tgfr_imim_dw", *dw_args, ptr(wsd), _hip.stream())
        att = _imim_grads(_bn_unfold(ctx, gm, s))[:9]
        return att + (dlnw.reshape(lnshape), dlnb.reshape(lnshape), dw1.reshape(w1shape), db1,
                      dw2.reshape(w2shape), db2, dwp, dbp) + (None,) * 6


def imim_fused(x, bn, sa, scale, ln, conv1, conv2, proj, eps=1e-12, rows_spec=None):
    """The IMIM head from the input map on (ImimFused); x must not require a
    gradient.  Returns R [N, HW, 256] (+ the operand rows with rows_spec)."""
    out = ImimFused.apply(x, bn.weight, bn.bias, sa.key_proj.weight, sa.query_proj.weight,
                          sa.value_proj.weight, sa.key_proj.bias, sa.query_proj.bias,
                          sa.value_proj.bias, ln.weight, ln.bias, conv1.weight, conv1.bias,
                          conv2.weight, conv2.bias, proj.weight, proj.bias, bn, bn.training,
                          scale, ln.eps, eps, rows_spec)
    if rows_spec:
        return out[0], (out[1], out[2])
    return out


def imim_ln_tail(x, ln, conv1, conv2, proj, eps=1e-12, rows_spec=None):
    """normalize(proj(relu(conv2(relu(conv1(LayerNorm(x))))))) on the
    channels-last attention output x [N, HW, 256] (ImimLnTail); rows_spec as
    imim_tail."""
    out = ImimLnTail.apply(x, ln.weight, ln.bias, conv1.weight, conv1.bias, conv2.weight,
                           conv2.bias, proj.weight, proj.bias, ln.eps, eps, rows_spec)
    if rows_spec:
        return out[0], (out[1], out[2])
    return out


def imim_tail(z, conv1, conv2, proj, eps=1e-12, rows_spec=None):
    """R = normalize(proj(relu(conv2(relu(conv1(z)))))) on channels-last rows
    z [..., 256] (bf16 operands, fp32 accumulation).  With rows_spec =
    (rows per item, padded rows, fp16) also returns (R rows in the
    word<->region operand layout, their norms) -- see attach_rows."""
    out = ImimTail.apply(z, conv1.weight, conv1.bias, conv2.weight, conv2.bias, proj.weight,
                         proj.bias, eps, rows_spec)
    if rows_spec:
        return out[0], (out[1], out[2])
    return out


def attach_rows(x, rows, norms, f16, scale=1.0):
    """Tag a feature tensor with its rows in the word<->region kernels'
    operand layout (tgfr_prep_rows' hi plane of scale * x, and |x| per row),
    written by the kernel that produced x: the image regions R by the IMIM
    tail (tgfr_tail_fwd), the words W by TextHeading (tgfr_text_heading).
    WordRegionLogits then skips its tgfr_prep_rows pass over x.  The tag
    holds while x (or a view of it with the same layout) is the same storage
    at the same version: no in-place change since."""
    x._tgfr_rows = (rows, norms, bool(f16), float(scale), x._version, x.data_ptr(),
                    tuple(x.shape), tuple(x.stride()))
    return x


def rows_only_words(rows, norms, n_words, f16, scale=LOG2E):
    """A words tensor [B, 256, n_words] that carries ONLY its operand rows
    (rows [B, t_pad, 256], norms [B, t_pad], attach_rows) -- no feature
    values: the text side of a data-parallel step, all-gathered as the
    word<->region kernels' bf16 / fp16 rows (half the bytes of the fp32
    words).  Any path that would read its values raises
    (WordRegionLogits)."""
    b = rows.shape[0]
    base = torch.empty_strided((b, n_words, D), (0, 0, 0), dtype=torch.float32,
                               device=rows.device)
    base._tgfr_rows_only = True
    attach_rows(base, rows, norms, f16, scale)
    return base.transpose(1, 2)


def _rows_only(x):
    return any(getattr(t, "_tgfr_rows_only", False) for t in (x, getattr(x, "_base", None)))


def attached_rows(x, f16, scale=1.0):
    """(rows, norms) attached to x -- or to the tensor x views with x's own
    shape and strides -- by attach_rows, if still valid for this operand
    precision and scale; else None."""
    for t in (x, getattr(x, "_base", None)):
        tag = getattr(t, "_tgfr_rows", None) if t is not None else None
        if tag is None:
            continue
        rows, norms, tf16, tscale, version, addr, shape, stride = tag
        if (tf16 == bool(f16) and tscale == float(scale) and version == t._version and
                addr == x.data_ptr() and shape == tuple(x.shape) and
                stride == tuple(x.stride())):
            return rows, norms
    return None


# ---------------------------------------------------------------- heads ---
class L2NormRows(torch.autograd.Function):
    """F.normalize(x, p=2, dim=-1, eps) in one kernel each way."""

    @staticmethod
    def forward(ctx, x, eps):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).float().contiguous()
        rows, d = x2.shape
        y = torch.empty_like(x2)
        inv = torch.empty(rows, dtype=torch.float32, device=x2.device)
        call("tgfr_l2norm_rows", ptr(x2), d, rows, d, float(eps), ptr(y), d, ptr(inv),
             _hip.stream())
        ctx.save_for_backward(y, inv)
        ctx.cfg = (float(eps), shape)
        return y.reshape(shape)

    @staticmethod
    def backward(ctx, dy):
        y, inv = ctx.saved_tensors
        eps, shape = ctx.cfg
        rows, d = y.shape
        dy2 = dy.reshape(rows, d).float().contiguous()
        dx = torch.empty_like(y)
        call("tgfr_l2norm_rows_bwd", ptr(dy2), d, ptr(y), d, ptr(inv), rows, d, eps, ptr(dx),
             d, _hip.stream())
        return dx.reshape(shape), None


def l2norm_rows(x, eps=1e-12):
    return L2NormRows.apply(x, eps)


class ProjL2Norm(torch.autograd.Function):
    """F.normalize(x W^T + b, dim=1, eps) -- nn.Linear then the row l2-norm
    (ProjectionHead, models/models.py:112-120) -- for a small batch of rows in
    exact fp32: one launch forward (tgfr_proj_l2norm_fwd), two backward (the
    l2-norm backward, then dW and db in one launch, tgfr_proj_dw)."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        x2 = _aligned(x)
        w = _aligned(weight)
        b_ = None if bias is None else bias.float().contiguous()
        rows, k = x2.shape
        n = w.shape[0]
        dev = x2.device
        out = (ctypes.c_longlong * 1)()
        rc = _hip.lib().tgfr_proj_l2norm_ws(rows, n, ctypes.addressof(out))
        if rc != 0:
            raise RuntimeError(f"tgfr_proj_l2norm_ws failed with code {rc}")
        ws = torch.empty(int(out[0]), dtype=torch.float32, device=dev)
        g = torch.empty(rows, n, dtype=torch.float32, device=dev)
        inv = torch.empty(rows, dtype=torch.float32, device=dev)
        call("tgfr_proj_l2norm_fwd", ptr(x2), k, rows, k, ptr(w), k, ptr(b_), n, float(eps),
             ptr(ws), ptr(g), n, ptr(inv), ptr(_hip.counters(dev)), _hip.stream())
        ctx.save_for_backward(x2, w, g, inv)
        ctx.cfg = (float(eps), bias is not None)
        return g

    @staticmethod
    def backward(ctx, dg):
        x2, w, g, inv = ctx.saved_tensors
        eps, has_bias = ctx.cfg
        rows, k = x2.shape
        n = w.shape[0]
        dg = dg.float().contiguous()
        dy = torch.empty(rows, n, dtype=torch.float32, device=w.device)
        call("tgfr_l2norm_rows_bwd", ptr(dg), n, ptr(g), n, ptr(inv), rows, n, eps, ptr(dy), n,
             _hip.stream())
        db = torch.empty(n, dtype=torch.float32, device=w.device) \
            if has_bias and ctx.needs_input_grad[2] else None
        dw = None
        if ctx.needs_input_grad[1] or db is not None:
            dw = torch.empty_like(w)
            call("tgfr_proj_dw", ptr(dy), n, ptr(x2), k, rows, k, n, ptr(dw), k, ptr(db),
                 _hip.stream())
        dx = bgemm(dy.unsqueeze(0), w.unsqueeze(0), mode="fp32")[0] \
            if ctx.needs_input_grad[0] else None
        return dx, dw if ctx.needs_input_grad[1] else None, db, None


def proj_l2norm(x, weight, bias=None, eps=1e-12, mode="fp32"):
    """normalize(x W^T + b): the exact-fp32 kernels for the trainers' small
    batches (rows <= 64, N % 32 == 0, N <= 1024, K % 4 == 0, K <= 612), else
    the Linear GEMM (in `mode`) and the row l2-norm as two Functions."""
    w = weight.reshape(weight.shape[0], -1)
    if (x.dim() == 2 and x.shape[0] <= 64 and w.shape[0] % 32 == 0 and w.shape[0] <= 1024 and
            x.shape[1] % 4 == 0 and x.shape[1] <= 612 and x.shape[1] == w.shape[1]):
        return ProjL2Norm.apply(x, w, bias, eps)
    return l2norm_rows(linear_rows(x, weight, bias, mode=mode), eps)


class ArcMargin(torch.autograd.Function):
    """The margin part of ArcMarginProduct on a cosine matrix (metrics.py:45-57)."""

    @staticmethod
    def forward(ctx, cosine, label, s, m, easy):
        cosine = cosine.float().contiguous()
        label = label.to(torch.int64).contiguous()
        rows, cols = cosine.shape
        out = torch.empty_like(cosine)
        call("tgfr_arc_margin", ptr(cosine), ptr(label), rows, cols, float(s), float(m),
             int(easy), ptr(out), _hip.stream())
        ctx.save_for_backward(cosine, label)
        ctx.cfg = (float(s), float(m), int(easy))
        return out

    @staticmethod
    def backward(ctx, dout):
        cosine, label = ctx.saved_tensors
        s, m, easy = ctx.cfg
        rows, cols = cosine.shape
        dout = dout.float().contiguous()
        dcos = torch.empty_like(cosine)
        call("tgfr_arc_margin_bwd", ptr(cosine), ptr(label), ptr(dout), rows, cols, s, m,
             easy, ptr(dcos), _hip.stream())
        return dcos, None, None, None, None


def arc_margin(cosine, label, s, m, easy_margin=False):
    return ArcMargin.apply(cosine, label, s, m, easy_margin)


class ArcHead(torch.autograd.Function):
    """ArcMarginProduct.forward (metrics.py:43-57) in one launch each way:
    normalise x and W, cosine, margin (tgfr_arc_fwd); margin backward, dW with
    the l2-norm backward fused (tgfr_arc_bwd); dx = l2-norm backward of
    (dcos / |W|) W (one GEMM + one row kernel, only when x needs a gradient)."""

    @staticmethod
    def forward(ctx, x, weight, label, s, m, easy, eps, mode):
        x2 = _aligned(x)
        w = _aligned(weight)
        label = label.to(torch.int64).contiguous()
        b, d = x2.shape
        c = w.shape[0]
        dev = x2.device
        logits = torch.empty(b, c, dtype=torch.float32, device=dev)
        cosv = torch.empty_like(logits)
        xn = torch.empty_like(x2)
        inv_nx = torch.empty(b, dtype=torch.float32, device=dev)
        inv_nw = torch.empty(c, dtype=torch.float32, device=dev)
        call("tgfr_arc_fwd", ptr(x2), d, b, d, ptr(w), d, c, ptr(label), float(s), float(m),
             int(easy), float(eps), ptr(logits), ptr(cosv), ptr(xn), ptr(inv_nx), ptr(inv_nw),
             _hip.stream())
        ctx.save_for_backward(w, label, cosv, xn, inv_nx, inv_nw)
        ctx.cfg = (float(s), float(m), int(easy), float(eps), mode)
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        w, label, cosv, xn, inv_nx, inv_nw = ctx.saved_tensors
        s, m, easy, eps, mode = ctx.cfg
        b, d = xn.shape
        c = w.shape[0]
        dl = dlogits.float().contiguous()
        dw = torch.empty_like(w)
        want_dx = ctx.needs_input_grad[0]
        dcs = torch.empty(b, c, dtype=torch.float32, device=w.device) if want_dx else None
        nws = arc_bwd_ws_floats(b, d, c)
        ws = torch.empty(nws, dtype=torch.float32, device=w.device) if nws else None
        call("tgfr_arc_bwd", ptr(dl), ptr(cosv), ptr(label), ptr(xn), ptr(w), d, ptr(inv_nw),
             b, d, c, s, m, easy, eps, ptr(dw), d, ptr(dcs), ptr(ws), _hip.stream())
        dx = arc_dx(dcs, w, xn, inv_nx, eps) if want_dx else None
        return dx, dw, None, None, None, None, None, None


def arc_dx(dcs, w, xn, inv_nx, eps):
    """An ArcMargin head's input gradient from its backward's dcs [B][C]
    (= dcos / |W_c|): dxn = dcs W, then the F.normalize backward of x
    (models/metrics.py:43), exact fp32, in two launches (tgfr_arc_dx)."""
    b, d = xn.shape
    c = w.shape[0]
    out = (ctypes.c_longlong * 1)()
    rc = _hip.lib().tgfr_arc_dx_ws(int(b), int(c), int(d), ctypes.addressof(out))
    if rc != 0:
        raise RuntimeError(f"tgfr_arc_dx_ws failed with code {rc}")
    ws = torch.empty(int(out[0]), dtype=torch.float32, device=xn.device)
    dx = torch.empty_like(xn)
    call("tgfr_arc_dx", ptr(dcs), ptr(w), w.stride(0), b, c, d, ptr(xn), ptr(inv_nx),
         float(eps), ptr(ws), ptr(dx), _hip.stream())
    return dx


def arc_bwd_ws_floats(b, d, c):
    out = (ctypes.c_longlong * 1)()
    rc = _hip.lib().tgfr_arc_bwd_ws(int(b), int(d), int(c), ctypes.addressof(out))
    if rc != 0:
        raise RuntimeError(f"tgfr_arc_bwd_ws failed with code {rc}")
    return int(out[0])


def arc_head(x, weight, label, s, m, easy_margin=False, eps=1e-12, mode="fp32"):
    return ArcHead.apply(x, weight, label, s, m, easy_margin, eps, mode)


class _ArcHeadArgs(ctypes.Structure):
    """tgfr_arc_head (include/tgfr.h)."""
    _fields_ = [("x", ctypes.c_void_p), ("W", ctypes.c_void_p), ("label", ctypes.c_void_p),
                ("s", ctypes.c_float), ("logits", ctypes.c_void_p), ("cosv", ctypes.c_void_p),
                ("xn", ctypes.c_void_p), ("inv_nx", ctypes.c_void_p),
                ("inv_nw", ctypes.c_void_p), ("focal_ws", ctypes.c_void_p),
                ("g", ctypes.c_void_p), ("dW", ctypes.c_void_p), ("dcs", ctypes.c_void_p)]


def _heads_fwd(x_t, w_t, x_i, w_i, label, s_t, s_i, m, easy, eps, gamma):
    """Both identity heads' ArcMargin forward (one launch) and both focal CEs
    on the local rows (one launch): per head the tensors IdentityHeads saves."""
    xs = [_aligned(x_t), _aligned(x_i)]
    ws_ = [w_t, w_i]
    b, d = xs[0].shape
    c = ws_[0].shape[0]
    dev = xs[0].device
    out = []
    heads = (_ArcHeadArgs * 2)()
    for k, sc in enumerate((s_t, s_i)):
        t = {"logits": torch.empty(b, c, dtype=torch.float32, device=dev),
             "cosv": torch.empty(b, c, dtype=torch.float32, device=dev),
             "xn": torch.empty_like(xs[k]),
             "inv_nx": torch.empty(b, dtype=torch.float32, device=dev),
             "inv_nw": torch.empty(c, dtype=torch.float32, device=dev),
             "fws": torch.empty(2 * b + 1, dtype=torch.float32, device=dev),
             "loss": torch.empty(1, dtype=torch.float32, device=dev)}
        out.append(t)
        heads[k] = _ArcHeadArgs(ptr(xs[k]), ptr(ws_[k]), ptr(label), float(sc),
                                ptr(t["logits"]), ptr(t["cosv"]), ptr(t["xn"]),
                                ptr(t["inv_nx"]), ptr(t["inv_nw"]), None, None, None, None)
    call("tgfr_arc_fwd_heads", ctypes.addressof(heads), 2, b, d, c, float(m), int(easy),
         float(eps), _hip.stream())
    call("tgfr_focal_ce2", ptr(out[0]["logits"]), ptr(out[1]["logits"]), b, c, ptr(label),
         float(gamma), ptr(out[0]["fws"]), ptr(out[1]["fws"]), ptr(_hip.counters(dev)),
         ptr(out[0]["loss"]), ptr(out[1]["loss"]), _hip.stream())
    return out


class IdentityHeads(torch.autograd.Function):
    """The stage-1 step's two identity losses, focal(ArcMargin_text(sent)) and
    focal(ArcMargin_image(img)) (src/train_encoders_bert.py:293-306, one
    process, B <= 128, heads of one (D, C)): both heads' cosine + margin in one
    launch, both focal losses in one launch; backward: the focal logit
    gradient formed inside the ArcMargin backward of both heads (one launch),
    then dx of the heads whose input is trained (dcs W GEMM + l2-norm
    backward, as ArcHead).

    With a process group (one process per GPU, rows = this rank's batch) the
    focal factor is applied to the GLOBAL mean cross-entropy, as FocalCE does:
    both heads' local NLL sums go into ONE all-reduce of two floats between
    the forward launches and the loss formation, and the backward's logit
    gradient carries f'(CE_global) / N_global -- the same kernels as one
    process, plus that collective."""

    @staticmethod
    def forward(ctx, x_t, w_t, x_i, w_i, label, s_t, s_i, m, easy, eps, gamma, mode,
                group=None, n_global=None, pre=None):
        ws_ = [_aligned(w_t), _aligned(w_i)]
        label = label.to(torch.int64).contiguous()
        if pre is not None:
            # identity_heads_parts ran earlier; both heads' NLL sums rode in a
            # merged all-gather: gathered [world, >= 2] rows (any row stride)
            out, gsums = pre
            b = out[0]["xn"].shape[0]
            call("tgfr_focal_global", 1, ptr(gsums), gsums.shape[0], gsums.stride(0), 2, b,
                 1.0 / float(n_global), float(gamma), ptr(out[0]["fws"]), ptr(out[1]["fws"]),
                 ptr(out[0]["loss"]), ptr(out[1]["loss"]), _hip.stream())
            ctx.save_for_backward(ws_[0], ws_[1], label,
                                  *[out[k][n] for k in range(2)
                                    for n in ("logits", "cosv", "xn", "inv_nx", "inv_nw", "fws")])
            ctx.cfg = (float(s_t), float(s_i), float(m), int(easy), float(eps), float(gamma), mode,
                       b / float(n_global))
            return out[0]["loss"][0], out[1]["loss"][0]
        out = _heads_fwd(x_t, ws_[0], x_i, ws_[1], label, s_t, s_i, m, easy, eps, gamma)
        b = out[0]["xn"].shape[0]
        losses = [out[0]["loss"][0], out[1]["loss"][0]]
        if group is not None:
            # fws[b] holds the local mean CE (FocalCE's layout): both heads'
            # NLL sums in one collective, then the global mean goes back in
            _focal_global(group, n_global, b, gamma, [out[0]["fws"], out[1]["fws"]],
                          [out[0]["loss"], out[1]["loss"]])
        ctx.save_for_backward(ws_[0], ws_[1], label,
                              *[out[k][n] for k in range(2)
                                for n in ("logits", "cosv", "xn", "inv_nx", "inv_nw", "fws")])
        ctx.cfg = (float(s_t), float(s_i), float(m), int(easy), float(eps), float(gamma), mode,
                   b / float(n_global) if group is not None else 1.0)
        return losses[0], losses[1]

    @staticmethod
    def backward(ctx, g_t, g_i):
        w_t, w_i, label, *rest = ctx.saved_tensors
        s_t, s_i, m, easy, eps, gamma, mode, gscale = ctx.cfg
        per = [dict(zip(("logits", "cosv", "xn", "inv_nx", "inv_nw", "fws"), rest[6 * k:6 * k + 6]))
               for k in range(2)]
        ws_ = (w_t, w_i)
        b, d = per[0]["xn"].shape
        c = w_t.shape[0]
        dev = w_t.device
        want_dx = (ctx.needs_input_grad[0], ctx.needs_input_grad[2])
        # (the kernel divides by the local row count; under a process group the
        # global mean's gradient divides by the global one)
        gs = [(g.float().reshape(1) * gscale if gscale != 1.0 else g.float().reshape(1))
              .contiguous() for g in (g_t, g_i)]
        dws = [torch.empty_like(w) for w in ws_]
        dcs = [torch.empty(b, c, dtype=torch.float32, device=dev) if want_dx[k] else None
               for k in range(2)]
        heads = (_ArcHeadArgs * 2)()
        for k, sc in enumerate((s_t, s_i)):
            t = per[k]
            heads[k] = _ArcHeadArgs(None, ptr(ws_[k]), ptr(label), sc, ptr(t["logits"]),
                                    ptr(t["cosv"]), ptr(t["xn"]), ptr(t["inv_nx"]),
                                    ptr(t["inv_nw"]), ptr(t["fws"]), ptr(gs[k]), ptr(dws[k]),
                                    ptr(dcs[k]))
        call("tgfr_arc_focal_bwd_heads", ctypes.addressof(heads), 2, b, d, c, m, easy, eps, gamma,
             _hip.stream())
        dx = [arc_dx(dcs[k], ws_[k], per[k]["xn"], per[k]["inv_nx"], eps) if want_dx[k]
              else None for k in range(2)]
        return (dx[0], dws[0], dx[1], dws[1]) + (None,) * 11


def identity_heads(x_t, head_t, x_i, head_i, label, gamma, eps=1e-12, group=None,
                   n_global=None, pre=None):
    """(focal(head_t(x_t)), focal(head_i(x_i))) for two ArcMarginProduct
    modules of one (D, C) and margin: kernels.IdentityHeads (with a process
    group: this rank's rows, focal factor of the global-batch mean CE).
    pre: identity_heads_parts' state + the gathered NLL sums [world, >= 2] of
    a merged exchange."""
    return IdentityHeads.apply(x_t, head_t.weight, x_i, head_i.weight, label, head_t.s, head_i.s,
                               head_t.m, head_t.easy_margin, eps, gamma, head_t.precision,
                               group, n_global, pre)


def identity_heads_parts(x_t, head_t, x_i, head_i, label, gamma, sums, eps=1e-12):
    """Stage 1 of the data-parallel identity heads: both ArcMargin forwards and
    local focal CEs, and both heads' local NLL sums written into `sums` [2] (a
    view of a merged exchange buffer; tgfr_focal_global phase 0).  Returns the
    heads' state for identity_heads(..., pre=(state, gathered sums))."""
    label = label.to(torch.int64).contiguous()
    out = _heads_fwd(x_t.detach(), _aligned(head_t.weight.detach()), x_i.detach(),
                     _aligned(head_i.weight.detach()), label, head_t.s, head_i.s, head_t.m,
                     head_t.easy_margin, eps, gamma)
    b = out[0]["xn"].shape[0]
    call("tgfr_focal_global", 0, ptr(sums), 1, 0, 2, b, 1.0, float(gamma), ptr(out[0]["fws"]),
         ptr(out[1]["fws"]), None, None, _hip.stream())
    return out


class FocalCE(torch.autograd.Function):
    """FocalLoss(gamma)(logits, target) (losses.py:313-325) on one or more
    (logits, target) pairs.

    The reference applies the focal factor to the mean cross-entropy of the
    WHOLE batch it sees (DataParallel gathers every replica's logits on GPU 0).
    With a process group each rank holds its own rows: the per-rank NLL sums
    are summed over ranks by all-reduces -- one per group of at most two pairs
    with the same row count (tgfr_focal_global packs two heads), so the
    trainers' two identity heads of one batch cost ONE; more pairs or other
    row counts cost one more collective (and one more graph segment under
    dist.StepCapture) per group -- the focal loss is formed from the global
    mean on every rank, and each rank's logit gradient carries
    f'(CE_global) / N_global -- so the gradients summed over ranks are the
    reference's global-batch gradients."""

    @staticmethod
    def forward(ctx, gamma, group, n_global, *pairs):
        n = len(pairs) // 2
        dev = pairs[0].device
        outs, saved = [], []
        for k in range(n):
            logits = pairs[2 * k].float().contiguous()
            target = pairs[2 * k + 1].to(torch.int64).contiguous()
            rows, cols = logits.shape
            ws = torch.empty(2 * rows + 1, dtype=torch.float32, device=dev)
            loss = torch.empty(1, dtype=torch.float32, device=dev)
            call("tgfr_focal_ce", ptr(logits), rows, cols, ptr(target), float(gamma), ptr(ws),
                 ptr(_hip.counters(dev)), ptr(loss), _hip.stream())
            outs.append(loss)
            saved += [logits, target, ws]
        rows_l = [saved[3 * k].shape[0] for k in range(n)]
        if group is not None:
            # every pair's local NLL sum in one collective (heads with one
            # batch size: tgfr_focal_global; otherwise the same per row count)
            for r in sorted(set(rows_l)):
                ks = [k for k in range(n) if rows_l[k] == r]
                for i in range(0, len(ks), 2):
                    kk = ks[i:i + 2]
                    _focal_global(group, n_global, r, gamma, [saved[3 * k + 2] for k in kk],
                                  [outs[k] for k in kk])
        ctx.save_for_backward(*saved)
        ctx.cfg = (float(gamma), n, rows_l, n_global if group is not None else None)
        return tuple(o[0] for o in outs)

    @staticmethod
    def backward(ctx, *gs):
        gamma, n, rows_l, n_global = ctx.cfg
        saved = ctx.saved_tensors
        grads = []
        for k in range(n):
            logits, target, ws = saved[3 * k:3 * k + 3]
            rows, cols = logits.shape
            g = gs[k]
            if g is None:
                grads += [None, None]
                continue
            g = g.float().reshape(1)
            if n_global is not None:
                # the kernel divides by the local row count; the global mean's
                # gradient divides by the global one
                g = g * (rows / float(n_global))
            g = g.contiguous()
            dl = torch.empty_like(logits)
            call("tgfr_focal_ce_bwd", ptr(logits), rows, cols, ptr(target), gamma, ptr(ws),
                 ptr(g), ptr(dl), _hip.stream())
            grads += [dl, None]
        return (None, None, None) + tuple(grads)


def focal_ce(logits, target, gamma, group=None, n_global=None):
    return FocalCE.apply(gamma, group, n_global, logits, target)[0]


def focal_ce_multi(pairs, gamma, group=None, n_global=None):
    """Focal losses of several (logits, target) pairs; under a process group
    their global means cost one all-reduce together."""
    flat = [x for p in pairs for x in p]
    return FocalCE.apply(gamma, group, n_global, *flat)


# ------------------------------------------------------------- loss mix ---
class LossMix(torch.autograd.Function):
    """(total, report) = (W[0] . losses, W[1:] . losses) in one launch; only
    total carries a gradient (dloss_i = g W[0][i], one launch)."""

    @staticmethod
    def forward(ctx, weights, *losses):
        n, m = len(losses), len(weights)
        dev = losses[0].device
        ptrs = (ctypes.c_void_p * n)(*[ptr(l.float()) for l in losses])
        w = (ctypes.c_float * (n * m))(*[float(x) for row in weights for x in row])
        out = torch.empty(m, dtype=torch.float32, device=dev)
        call("tgfr_loss_mix", n, ctypes.addressof(ptrs), m, ctypes.addressof(w), ptr(out),
             _hip.stream())
        ctx.w0 = [float(x) for x in weights[0]]
        ctx.set_materialize_grads(False)
        total, report = out[0], out[1:]
        ctx.mark_non_differentiable(report)
        return total, report

    @staticmethod
    def backward(ctx, g, _unused):
        n = len(ctx.w0)
        if g is None:
            return (None,) * (n + 1)
        g = g.float().contiguous()
        w = (ctypes.c_float * n)(*ctx.w0)
        d = torch.empty(n, dtype=torch.float32, device=g.device)
        call("tgfr_loss_mix_bwd", ptr(g), n, ctypes.addressof(w), ptr(d), _hip.stream())
        return (None,) + tuple(d[i] for i in range(n))


def loss_mix(losses, weights):
    """weights: m rows of len(losses) floats; returns (total [], report [m-1])."""
    return LossMix.apply(tuple(tuple(r) for r in weights), *losses)



# ---------------------------------------------------------------------------
# TextHeading (models/models.py:170-232)

def text_heading_ws_floats(b, l1):
    out = (ctypes.c_longlong * 1)()
    rc = _hip.lib().tgfr_text_heading_ws(int(b), int(l1), ctypes.addressof(out))
    if rc != 0:
        raise RuntimeError(f"tgfr_text_heading_ws failed with code {rc}")
    return int(out[0])


def text_pack(conv_w, mode="fp32"):
    """conv_w[k] [256, 1, k+2, 768] fp32 -> tap-major bf16 planes (uint16) for
    tgfr_text_heading (hi, plus lo in the fp32 mode)."""
    ws_ = [w.contiguous() for w in conv_w]
    for k, w in enumerate(ws_):
        assert tuple(w.shape) == (D, 1, k + 2, 768) and w.dtype == torch.float32
    out = (ctypes.c_longlong * 1)()
    rc = _hip.lib().tgfr_text_pack_bytes(_mode(mode), ctypes.addressof(out))
    if rc != 0:
        raise RuntimeError(f"tgfr_text_pack_bytes failed with code {rc}")
    taps = torch.empty(int(out[0]) // 2, dtype=torch.int16, device=ws_[0].device)
    wp = (ctypes.c_void_p * 3)(*[ptr(w) for w in ws_])
    call("tgfr_text_pack", ctypes.addressof(wp), ptr(taps), _mode(mode), _hip.stream())
    return taps


def text_heading(words_emb, taps, conv_b, mode="fp32", words=None, sent=None, rows_spec=None):
    """Bert_Word_Mapping + TextHeading forward: words_emb [B, L1, 768] fp32 (BERT
    last hidden state without [CLS]), taps = text_pack(conv weights, mode),
    conv_b[k] [256] -> (words [B, L1-1, 256] unit rows, sent [B, 256] unit
    rows).  One launch for the three convs + one pooling launch (tgfr_text.hip).
    rows_spec = (t_pad, scale, fp16): the pooling launch also writes the words
    as word<->region operand rows, attached to `words` (attach_rows)."""
    assert words_emb.dim() == 3 and words_emb.shape[2] == 768
    assert words_emb.dtype == torch.float32
    b, l1, _ = words_emb.shape
    if l1 < 4:
        raise ValueError("TextHeading needs bert_words_num >= 5 (three conv widths up to 4)")
    x = words_emb.contiguous()
    bs_ = [v.contiguous() for v in conv_b]
    for v in bs_:
        assert tuple(v.shape) == (D,) and v.dtype == torch.float32
    dev = x.device
    if words is None:
        words = torch.empty(b, l1 - 1, D, dtype=torch.float32, device=dev)
    if sent is None:
        sent = torch.empty(b, D, dtype=torch.float32, device=dev)
    ws = torch.empty(text_heading_ws_floats(b, l1), dtype=torch.float32, device=dev)
    bp = (ctypes.c_void_p * 3)(*[ptr(v) for v in bs_])
    t_pad, scale, f16 = rows_spec if rows_spec else (0, 1.0, False)
    w_rows = torch.empty(b, t_pad, D, dtype=torch.int16, device=dev) if rows_spec else None
    w_norm = torch.empty(b, t_pad, dtype=torch.float32, device=dev) if rows_spec else None
    call("tgfr_text_heading", ptr(x), b, l1, ptr(taps), ctypes.addressof(bp),
         ptr(ws), ptr(words), words.stride(0), words.stride(1),
         ptr(sent), sent.stride(0), ptr(w_rows), ptr(w_norm), t_pad, float(scale),
         int(bool(f16)), _mode(mode), _hip.stream())
    if rows_spec:
        attach_rows(words, w_rows, w_norm, f16, scale=scale)
    return words, sent
