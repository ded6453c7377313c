"""Drop-in for the reference's image head (models/models.py:98-120, 328-338,
380-405).  Parameter names match the reference for checkpoint interop.

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

__all__ = ["ProjectionHead", "IMIM", "ImageHeading"]


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
        y = K.linear_rows(x, self.projection.weight, self.projection.bias, mode=self.precision)
        return K.l2norm_rows(y)


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
        wq, bq = self.sa.packed_self()
        px = K.bn_linear(img, self.bn_img, wq, bq, mode=self.precision)   # [B, HW, 3C]
        z = self.sa.core_self(px)
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

    def forward(self, global_image, local_image):
        local_image = self.imim(local_image)
        global_image = self.project_global(global_image)
        return global_image, local_image
