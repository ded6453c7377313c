"""ArcMarginProduct (models/metrics.py:17-60): the identity head that runs
after the hot path every step.  Row normalisation,
the cosine product and the margin (with the one-hot that is CUDA-only in the
reference, :53) run as one gfx950 launch each way (csrc/tgfr_arc.hip)."""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn.parameter import Parameter

from .. import kernels as K

__all__ = ["ArcMarginProduct"]


class ArcMarginProduct(nn.Module):
    def __init__(self, in_features, out_features, s=30.0, m=0.50, easy_margin=False):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.s = s
        self.m = m
        self.weight = Parameter(torch.empty(out_features, in_features))
        nn.init.xavier_uniform_(self.weight)
        self.easy_margin = easy_margin
        self.cos_m = math.cos(m)
        self.sin_m = math.sin(m)
        self.th = math.cos(math.pi - m)
        self.mm = math.sin(math.pi - m) * m
        self.precision = "fp32"

    def forward(self, input, label):
        # normalize(x) normalize(W)^T and the margin (the reference's two
        # F.normalize, F.linear and 15 elementwise ops, :43-57) in one fp32
        # launch each way (kernels.ArcHead)
        return K.arc_head(input, self.weight, label, self.s, self.m, self.easy_margin,
                          mode=self.precision)
