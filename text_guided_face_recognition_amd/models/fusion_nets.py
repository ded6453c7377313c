"""Drop-in for the reference's models/fusion_nets.py SelfAttention and
Working (FCFM).  Parameter names match the reference (query_proj, key_proj,
value_proj, conv, bn_img, ...), so reference state dicts load unchanged.

The attention core (QK^T, softmax, PV and their backward) runs in the gfx950
kernels (kernels.AttentionCore); the 1x1 projections are plain GEMMs on a
channels-last view of the maps, so no NCHW<->NHWC copies are made.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import kernels as K

__all__ = ["SelfAttention", "Working", "conv1x1"]


def conv1x1(in_planes, out_planes):
    return nn.Conv2d(in_planes, out_planes, kernel_size=1, stride=1, padding=0, bias=False)


def _cl(x):
    """[N, C, H, W] (any strides) -> [N, H*W, C] view/copy, channels last."""
    n, c, h, w = x.shape
    return x.permute(0, 2, 3, 1).reshape(n, h * w, c)


class SelfAttention(nn.Module):
    """fusion_nets.py:82-118.

    forward(x, y): query role = key_proj(x), key role = query_proj(y),
    value = value_proj(x); softmax over y's positions; output [N, C, H, W]
    (returned as a channels-last strided view).
    """

    def __init__(self, channel_dim, scale=2):
        super().__init__()
        self.inplanes = channel_dim
        self.query_proj = nn.Conv2d(self.inplanes, self.inplanes // scale, 1)
        self.key_proj = nn.Conv2d(self.inplanes, self.inplanes // scale, 1)
        self.value_proj = nn.Conv2d(self.inplanes, self.inplanes, 1)
        self.sqrt_dim = np.sqrt(channel_dim / scale)
        self.precision = "fp32"

    def _w(self, conv):
        return conv.weight.reshape(conv.weight.shape[0], -1)

    def packed_self(self):
        """[key_proj; query_proj; value_proj] as one [2 C' + C, C] weight and
        bias: the query role, key role and value of self-attention."""
        w = torch.cat([self._w(self.key_proj), self._w(self.query_proj),
                       self._w(self.value_proj)], 0)
        b = torch.cat([self.key_proj.bias, self.query_proj.bias, self.value_proj.bias])
        return w, b

    def core_self(self, px):
        """Attention on packed [Qr | Kr | V] rows [N, HW, 2 C' + C]."""
        cq = self.key_proj.weight.shape[0]
        return K.attention_core(px, None, cq, cq, 2 * cq, 1.0 / float(self.sqrt_dim),
                                self.precision)

    def forward_cl(self, x_cl, y_cl):
        """Channels-last core: x_cl, y_cl [N, HW, C] -> [N, HW, C]."""
        mode = self.precision
        cq = self.key_proj.weight.shape[0]
        if y_cl is x_cl:
            w, b = self.packed_self()
            return self.core_self(K.linear_rows(x_cl, w, b, mode=mode))
        w = torch.cat([self._w(self.key_proj), self._w(self.value_proj)], 0)
        b = torch.cat([self.key_proj.bias, self.value_proj.bias])
        px = K.linear_rows(x_cl, w, b, mode=mode)                     # [Qr | V]
        py = K.linear_rows(y_cl, self._w(self.query_proj), self.query_proj.bias, mode=mode)
        return K.attention_core(px, py, cq, 0, cq, 1.0 / float(self.sqrt_dim), mode)

    def forward(self, x, y):
        n, c, h, w = y.shape
        assert x.shape[2] * x.shape[3] == h * w, "x and y need the same H*W (:105)"
        x_cl = _cl(x)
        y_cl = x_cl if y is x else _cl(y)
        o = self.forward_cl(x_cl, y_cl)
        return o.reshape(n, h, w, c).permute(0, 3, 1, 2)


class Working(nn.Module):
    """fusion_nets.py:217-258 (FCFM).  The channel_dim argument is ignored
    exactly as in the reference (:220)."""

    def __init__(self, channel_dim):
        super().__init__()
        channel_dim = 36
        self.bn_img = nn.BatchNorm2d(channel_dim)
        self.bn_word = nn.BatchNorm2d(channel_dim)
        self.projection = nn.Linear(256, channel_dim)
        self.sa = SelfAttention(channel_dim, scale=1)
        self.maxpool = nn.MaxPool2d(kernel_size=2)
        self.conv = nn.Conv2d(256, channel_dim, kernel_size=(3, 3), padding=0)
        self.relu = nn.ReLU()
        self.ln = nn.LayerNorm([channel_dim, 6, 6])
        self.ln_gl_image = nn.LayerNorm([256])
        self.ln_sent = nn.LayerNorm([256])
        self.linear = nn.Linear(324, 128)

    def forward(self, img, word, gl_img, sent):
        mode = self.sa.precision
        sa = self.sa
        # conv3x3 + ReLU + maxpool (:236-237): one fused kernel each way
        img = K.conv_relu_pool(img, self.conv.weight, self.conv.bias, mode=mode)   # [B,36,6,6]
        # word projection and its Gram matrix / 6 (:240-242)
        wd = K.linear_rows(word.transpose(1, 2), self.projection.weight, self.projection.bias,
                           mode=mode)                                    # [B, T, 36]
        wd = K.gram(wd, 1.0 / np.sqrt(36), mode=mode)                    # [B, 36, 36]
        wd = wd.view(wd.size(0), wd.size(1), 6, 6)
        # bn_img / bn_word (:237, :243) folded into the attention's 1x1
        # projections (query role = key_proj(img), value = value_proj(img),
        # key role = query_proj(word), :248 -> :97-99)
        wx = torch.cat([sa._w(sa.key_proj), sa._w(sa.value_proj)], 0)
        bx = torch.cat([sa.key_proj.bias, sa.value_proj.bias])
        px = K.bn_linear(img, self.bn_img, wx, bx, mode=mode)                # [B, 36, Qr | V]
        py = K.bn_linear(wd, self.bn_word, sa._w(sa.query_proj), sa.query_proj.bias,
                         mode=mode)                                        # [B, 36, Kr]
        cq = sa.key_proj.weight.shape[0]
        iw = K.attention_core(px, py, cq, 0, cq, 1.0 / float(sa.sqrt_dim), mode)   # [B, HW, C]
        # LayerNorm [36, 6, 6] on the channels-last rows, maxpool, flatten (:249-253)
        iw = K.layer_norm_rows(iw, self.ln.weight, self.ln.bias, self.ln.eps, ch=iw.shape[2])
        iw = K.maxpool2_cl(iw, 6, 6).reshape(iw.size(0), -1)             # [B, 324]
        iw = K.linear_rows(iw, self.linear.weight, self.linear.bias, mode=mode)
        gl_img = K.layer_norm_rows(gl_img, self.ln_gl_image.weight, self.ln_gl_image.bias,
                                   self.ln_gl_image.eps)
        sent = K.layer_norm_rows(sent, self.ln_sent.weight, self.ln_sent.bias, self.ln_sent.eps)
        return torch.concat((iw, gl_img, sent), dim=1)


def set_precision(module, mode):
    """Set the MFMA precision mode ("fp32" split or "bf16") of every drop-in
    module under ``module``."""
    for m in module.modules():
        if hasattr(m, "precision"):
            m.precision = mode
    return module
