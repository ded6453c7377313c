"""Drop-in for models/attention.py:10-43 ``func_attention``.

The trainers never call func_attention directly: words_loss reaches it only
through the fused word<->region kernel (kernels.WordRegionLogits), which
implements this exact arithmetic for every (image, caption) pair at once.
This standalone entry point keeps the reference's per-call contract (matched
query / context batches, differentiable in both inputs, attn returned as
[B, T, ih, iw]) on its own gfx950 kernels (csrc/tgfr_fa.hip, exact fp32).
"""
from __future__ import annotations

from .. import kernels as K

__all__ = ["func_attention"]


def func_attention(query, context, gamma1):
    """query [B, D, T], context [B, D, ih, iw] -> (C [B, D, T], attn [B, T, ih, iw])."""
    return K.func_attention(query, context, gamma1)
