"""Drop-in for the reference's image head (models/models.py:98-120, 328-338,
380-405) and text head (models/models.py:170-232).  Parameter names match the reference for checkpoint interop.

IMIM runs channels-last from the attention onwards: the SelfAttention core
is the gfx950 kernel, LayerNorm([256,14,14]) normalises each sample over all
of its elements (layout-agnostic) with the affine maps permuted to [HW, C],
the 1x1 convs and the projection are GEMMs on [B, 196, 256] rows, and the
result R is returned as a [B, 256, 14, 14] view with channels-last strides --
exactly the physical layout the reference produces (:401-404) and the layout
the word<->region kernel reads.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import kernels as K
from .fusion_nets import SelfAttention, _cl, set_precision

__all__ = ["ProjectionHead", "IMIM", "ImageHeading", "Bert_Word_Mapping", "TextHeading"]


class ProjectionHead(nn.Module):
    """models.py:98-120: Linear then L2-normalise (the GELU/fc/dropout members
    exist but are unused in the reference forward)."""

    def __init__(self, input_dim, projection_dim, dropout=0.4):
        super().__init__()
        self.projection = nn.Linear(input_dim, projection_dim)
        self.gelu = nn.GELU()
        self.fc = nn.Linear(projection_dim, projection_dim)
        self.dropout = nn.Dropout(dropout)
        self.precision = "fp32"

    def forward(self, x):
        return K.proj_l2norm(x, self.projection.weight, self.projection.bias,
                             mode=self.precision)


class IMIM(nn.Module):
    """models.py:380-405."""

    def __init__(self, args, channel_dim):
        super().__init__()
        self.channel_dim = channel_dim
        self.project_local = ProjectionHead(input_dim=256,
                                            projection_dim=args.aux_feat_dim_per_granularity)
        self.bn_img = nn.BatchNorm2d(self.channel_dim)
        self.sa = SelfAttention(channel_dim=self.channel_dim, scale=1)
        self.conv1x1_1 = nn.Conv2d(self.channel_dim, self.channel_dim // 2, kernel_size=(1, 1))
        self.relu = nn.ReLU()
        self.conv1x1_2 = nn.Conv2d(self.channel_dim // 2, self.channel_dim, kernel_size=(1, 1))
        self.ln = nn.LayerNorm([self.channel_dim, 14, 14])
        self.precision = getattr(args, "precision", "fp32")
        set_precision(self, self.precision)

    def forward(self, img):
        n, c, h, w = img.shape
        # bn_img folded into the packed q/k/v projection of the self-attention
        lowp = self.precision in ("bf16", "fp16")
        if lowp and c == 256 and 32 <= h * w <= 224 and not (
                torch.is_grad_enabled() and img.requires_grad):
            # the whole head as one node (the frozen backbone's map: no BN
            # input gradient); the kernel also writes R as the word<->region
            # operand rows (:403 -> losses.py:96), attached to the returned R
            f16 = self.precision == "fp16"
            spec = (h * w, K.RPAD, f16) if h * w == K.NREG else None
            z = K.imim_fused(img, self.bn_img, self.sa, 1.0 / float(self.sa.sqrt_dim), self.ln,
                             self.conv1x1_1, self.conv1x1_2, self.project_local.projection,
                             rows_spec=spec)
            if spec:
                z, (r_rows, r_norm) = z
            out = z.reshape(n, h, w, -1).permute(0, 3, 1, 2)
            return K.attach_rows(out, r_rows, r_norm, f16) if spec else out
        if lowp and c == 256 and h * w <= 224:
            # packed projection in bf16 straight into the fused attention kernels
            z = K.imim_attention(img, self.bn_img, self.sa, 1.0 / float(self.sa.sqrt_dim))
        else:
            wq, bq = self.sa.packed_self()
            px = K.bn_linear(img, self.bn_img, wq, bq, mode=self.precision)   # [B, HW, 3C]
            z = self.sa.core_self(px)
        if self.precision in ("bf16", "fp16"):
            # LayerNorm -> conv1x1_1 -> ReLU -> conv1x1_2 -> ReLU ->
            # project_local, fused (the LayerNorm applied on the tail's load,
            # its backward's sums in the tail backward); the kernel also writes
            # R as the word<->region operand rows (:403 -> losses.py:96),
            # attached to the returned R
            f16 = self.precision == "fp16"
            spec = (h * w, K.RPAD, f16) if h * w == K.NREG else None
            if h * w >= 32:
                z = K.imim_ln_tail(z.reshape(n, h * w, c), self.ln, self.conv1x1_1,
                                   self.conv1x1_2, self.project_local.projection,
                                   rows_spec=spec)
            else:
                z = K.layer_norm_rows(z, self.ln.weight, self.ln.bias, self.ln.eps, ch=c)
                z = K.imim_tail(z, self.conv1x1_1, self.conv1x1_2,
                                self.project_local.projection, rows_spec=spec)
            if spec:
                z, (r_rows, r_norm) = z
            out = z.reshape(n, h, w, -1).permute(0, 3, 1, 2)
            return K.attach_rows(out, r_rows, r_norm, f16) if spec else out
        # LayerNorm over (C, H, W) of each sample == over the channels-last
        # [HW, C] rows; the [C, H, W] affine maps are read channel-major in place
        z = K.layer_norm_rows(z, self.ln.weight, self.ln.bias, self.ln.eps, ch=c)
        z = K.linear_rows(z, self.conv1x1_1.weight, self.conv1x1_1.bias, relu=True,
                          mode=self.precision)
        z = K.linear_rows(z, self.conv1x1_2.weight, self.conv1x1_2.bias, relu=True,
                          mode=self.precision)
        z = self.project_local(z)                       # [B, HW, 256], unit rows
        return z.reshape(n, h, w, -1).permute(0, 3, 1, 2)


class ImageHeading(nn.Module):
    """models.py:328-338 -> (global [B, 256], local R [B, 256, 14, 14])."""

    def __init__(self, args):
        super().__init__()
        self.project_global = ProjectionHead(input_dim=512,
                                             projection_dim=args.aux_feat_dim_per_granularity)
        self.imim = IMIM(args, channel_dim=256)
        set_precision(self, getattr(args, "precision", "fp32"))

    def global_features(self, global_image):
        """g' = normalize(project_global(global_image)) (models.py:336)."""
        p = self.project_global
        return K.proj_l2norm(global_image, p.projection.weight, p.projection.bias, mode="fp32")

    def forward(self, global_image, local_image):
        local_image = self.imim(local_image)
        # g' feeds only fp32 consumers (the sentence / global cosine logits and
        # the fp32-MFMA identity head, whose loss is scaled by s * lambda_id =
        # 3000): its B x 512 x 256 projection runs in exact fp32 in every
        # precision (one launch each way at the trainers' batch sizes), so the
        # reduced-precision modes leave those terms at fp32 accuracy
        p = self.project_global
        return K.proj_l2norm(global_image, p.projection.weight, p.projection.bias,
                             mode="fp32"), local_image


class Bert_Word_Mapping(nn.Module):  # noqa: N801  (reference class name)
    """models.py:170-184: Conv2d(1, feat_dim, (K, 768)) for K = 2, 3, 4 (+ an
    unused Dropout).  The forward is fused into TextHeading's kernels."""

    def __init__(self, feat_dim):
        super().__init__()
        self.convs1 = nn.ModuleList([nn.Conv2d(1, feat_dim, (k, 768)) for k in (2, 3, 4)])
        self.dropout = nn.Dropout(0.1)


class TextHeading(nn.Module):
    """models.py:187-232 -> (words [B, 256, L-2] -- a transposed view of
    [B, L-2, 256] unit rows, as :231 -- and sent [B, 256] unit rows).

    Forward only: the reference runs it under no_grad
    (utils/dataset_utils.py:42-45), so no gradient reaches it; asking for one
    raises instead of returning a silently detached result."""

    def __init__(self, args):
        super().__init__()
        self.feat_dim = args.aux_feat_dim_per_granularity
        if self.feat_dim != K.D:
            raise ValueError(f"TextHeading kernels are built for feat_dim {K.D}")
        self.bwm = Bert_Word_Mapping(self.feat_dim)
        self.args = args
        self.precision = getattr(args, "precision", "fp32")
        self._taps = None          # (key, packed tap planes)

    def _conv_mode(self):
        # fp16 mode: bf16 convs (the words are normalised, then rounded to fp16)
        return "bf16" if self.precision == "fp16" else self.precision

    def packed_taps(self):
        """The conv weights as tap-major bf16 planes, re-packed only when a
        weight tensor is replaced or modified in place (its version moves)."""
        ws = [c.weight for c in self.bwm.convs1]
        key = (self._conv_mode(),) + tuple((w.data_ptr(), w._version) for w in ws)
        if self._taps is None or self._taps[0] != key:
            self._taps = (key, K.text_pack(ws, mode=self._conv_mode()))
        return self._taps[1]

    def forward(self, words_emb, sent_emb=None):
        # seq = bert_words_num - 1 - 3 (:204) fixes the token count
        if words_emb.shape[1] != self.args.bert_words_num - 1:
            raise ValueError(f"words_emb has {words_emb.shape[1]} tokens, expected "
                             f"bert_words_num - 1 = {self.args.bert_words_num - 1}")
        if torch.is_grad_enabled() and (words_emb.requires_grad or any(
                p.requires_grad for p in self.parameters())):
            raise RuntimeError("TextHeading is forward-only (the reference calls it under "
                               "torch.no_grad(), utils/dataset_utils.py:42); wrap the call "
                               "in torch.no_grad()")
        # bf16 / fp16: the pooling launch also writes the words as the
        # word<->region kernels' log2(e)-scaled operand rows (losses.py:96)
        # (captions past 64 words have no operand layout: the word<->region
        # kernels then prepare their rows themselves)
        spec = None
        n = words_emb.shape[1] - 1
        if self.precision in ("bf16", "fp16") and n <= 2 * K.TPAD:
            spec = (K.TPAD if n <= K.TPAD else 2 * K.TPAD, K.LOG2E, self.precision == "fp16")
        words, sent = K.text_heading(words_emb, self.packed_taps(),
                                     [c.bias for c in self.bwm.convs1], mode=self._conv_mode(),
                                     rows_spec=spec)
        return words.transpose(1, 2), sent
