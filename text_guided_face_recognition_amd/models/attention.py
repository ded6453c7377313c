"""Drop-in for models/attention.py:10-43 ``func_attention``.

The trainers never call func_attention directly: words_loss reaches it only
through the fused word<->region kernel (kernels.WordRegionLogits), which
implements this exact arithmetic for every (image, caption) pair at once.
This standalone entry point keeps the reference's per-call contract
(matched query/context batches, differentiable in both inputs) for API users
and runs the same math as device-side PyTorch ops; it is not on the measured
path.
"""
from __future__ import annotations

import torch

__all__ = ["func_attention"]


def func_attention(query, context, gamma1):
    """query [B, D, T], context [B, D, ih, iw] -> (C [B, D, T], attn [B, T, ih, iw])."""
    if not query.is_cuda:
        raise RuntimeError("func_attention takes device tensors (no CPU path)")
    b, _, t = query.shape
    ih, iw = context.shape[2], context.shape[3]
    ctx = context.reshape(b, context.shape[1], ih * iw)
    s = torch.bmm(ctx.transpose(1, 2), query)                  # [B, R, T]
    a1 = torch.softmax(s, dim=-1).transpose(1, 2)              # [B, T, R]
    a2 = torch.softmax(a1 * gamma1, dim=-1)
    weighted = torch.bmm(ctx, a2.transpose(1, 2))              # [B, D, T]
    return weighted, a2.reshape(b, t, ih, iw)
