"""Fused IMIM self-attention (csrc/tgfr_attn.hip attn_fwd / attn_bwd_*;
reference models/fusion_nets.py:93-118 with C' = C = 256) through the C ABI,
on a packed bf16 projection, against plain PyTorch fp32 on the GPU (inputs =
the same bf16 values):
  forward: lse to 1e-3; O against the same math with P rounded to bf16:
    1e-2 of max|O|;
  forward and backward against fp32 autograd of softmax(scale Qr Kr^T) V:
    relative Frobenius 2e-2 on O, dQr, dKr, dV."""
import pytest
import torch

from text_guided_face_recognition_amd import kernels as K

pytestmark = pytest.mark.gpu


def _bf(t):
    return t.to(torch.bfloat16).float()


def _frob(a, b):
    return float((a - b).norm() / b.norm())


def _attn(pxb, do, scale):
    """tgfr_attn_fwd / _bwd on a packed bf16 projection [nb, hw, 768]."""
    import ctypes
    from text_guided_face_recognition_amd import _hip
    from text_guided_face_recognition_amd._hip import call, ptr
    nb, hw, _ = pxb.shape
    bits = pxb.view(torch.int16)
    o = torch.empty(nb, hw, 256, device="cuda")
    lse = torch.empty(nb * hw, device="cuda")
    call("tgfr_attn_fwd", ptr(bits), ptr(bits[..., 256:]), ptr(bits[..., 512:]), 768, hw * 768,
         nb, hw, scale, ptr(o), 256, hw * 256, ptr(lse), _hip.stream())
    out = (ctypes.c_longlong * 1)()
    assert _hip.lib().tgfr_attn_bwd_ws(nb, hw, ctypes.addressof(out)) == 0
    ws = torch.empty(int(out[0]), dtype=torch.uint8, device="cuda")
    g = torch.empty(nb, hw, 768, dtype=torch.int16, device="cuda")      # bf16 gradients
    call("tgfr_attn_bwd", ptr(bits), ptr(bits[..., 256:]), ptr(bits[..., 512:]), 768, hw * 768,
         nb, hw, scale, ptr(o), ptr(do), 256, hw * 256, ptr(lse), ptr(g), ptr(g[..., 256:]),
         ptr(g[..., 512:]), 768, hw * 768, ptr(ws), _hip.stream())
    return o, lse, (g.to(torch.int32) << 16).view(torch.float32)


@pytest.mark.parametrize("nb,hw", [(64, 196), (3, 196), (2, 37), (1, 224), (4, 5), (5, 161)])
def test_fused_attention(nb, hw):
    torch.backends.cuda.matmul.allow_tf32 = False
    g = torch.Generator(device="cuda").manual_seed(nb * 1000 + hw)
    pxb = torch.randn(nb, hw, 768, generator=g, device="cuda").to(torch.bfloat16)
    do = torch.randn(nb, hw, 256, generator=g, device="cuda")
    scale = 1.0 / 16.0
    o, lse, dx = _attn(pxb, do, scale)

    px = pxb.float()
    q, k, v = px[..., :256], px[..., 256:512], px[..., 512:]
    s = scale * q @ k.transpose(1, 2)
    assert float((lse.view(nb, hw) - torch.logsumexp(s, -1)).abs().max()) < 1e-3
    o_em = _bf(torch.softmax(s, dim=-1)) @ v          # P rounded to bf16 as in the kernel
    assert float((o - o_em).abs().max() / o_em.abs().max()) < 1e-2

    xr = px.clone().requires_grad_()
    qr, kr, vr = xr[..., :256], xr[..., 256:512], xr[..., 512:]
    o_ref = torch.softmax(scale * qr @ kr.transpose(1, 2), dim=-1) @ vr
    (dx_ref,) = torch.autograd.grad(o_ref, xr, do)
    assert _frob(o, o_ref.detach()) < 2e-2
    for name, sl in (("dQr", slice(0, 256)), ("dKr", slice(256, 512)), ("dV", slice(512, 768))):
        e = _frob(dx[..., sl], dx_ref[..., sl])
        assert e < 2e-2, (name, e)


def test_self_attention_golden_bf16(gpu):
    """SelfAttention module in bf16 mode (the composed bgemm path, used for
    cross attention and outside IMIM) on the reference golden (C=256,
    HW=196): relative Frobenius 2e-2 on the output and gradients."""
    from conftest import load_golden, t
    from text_guided_face_recognition_amd.models.fusion_nets import SelfAttention
    g = load_golden("self_attention_c256_hw196")
    m = SelfAttention(256, scale=1).to(gpu)
    m.precision = "bf16"
    for name, key in (("query_proj", "q"), ("key_proj", "k"), ("value_proj", "v")):
        getattr(m, name).weight.data = t(g[f"{key}_w"]).to(gpu)
        getattr(m, name).bias.data = t(g[f"{key}_b"]).to(gpu)
    x = t(g["x"]).to(gpu).requires_grad_()
    out = m(x, x)
    ref = t(g["out"]).to(gpu)
    assert _frob(out.detach(), ref) < 2e-2
    (out * t(g["probe"]).to(gpu)).sum().backward()
    assert _frob(x.grad, t(g["d_x"]).to(gpu)) < 2e-2
    assert _frob(m.value_proj.weight.grad, t(g["d_v_w"]).to(gpu)) < 2e-2
    assert _frob(m.query_proj.weight.grad, t(g["d_q_w"]).to(gpu)) < 2e-2


@pytest.mark.parametrize("tag", ["small", "t22"])
def test_func_attention_golden(gpu, tag):
    """Standalone func_attention (csrc/tgfr_fa.hip, exact fp32) against the
    reference's fixtures (weighted context, attn, d_context through the
    probe) and the oracle's query gradient: 1e-5 / 1e-5 / 1e-4 absolute."""
    import numpy as np
    from conftest import load_golden, t
    from text_guided_face_recognition_amd.models.attention import func_attention
    import oracle.tgfr_oracle as O
    g = load_golden(f"func_attention_{tag}")
    q = t(g["query"]).to(gpu).requires_grad_()
    ctx = t(g["context"]).to(gpu).requires_grad_()
    wc, attn = func_attention(q, ctx, float(g["gamma1"]))
    assert np.abs(wc.detach().cpu().numpy() - g["weighted"]).max() < 1e-5
    assert np.abs(attn.detach().cpu().numpy() - g["attn"]).max() < 1e-5
    (wc * t(g["probe"]).to(gpu)).sum().backward()
    assert np.abs(ctx.grad.cpu().numpy() - g["d_context"]).max() < 1e-4
    qo = t(g["query"]).requires_grad_()
    wo, _ = O.func_attention(qo, t(g["context"]), float(g["gamma1"]))
    (wo * t(g["probe"])).sum().backward()
    assert np.abs(q.grad.cpu().numpy() - qo.grad.numpy()).max() < 1e-4


def test_func_attention_attn_grad(gpu):
    """Gradient through the returned attention map as well (dattn path):
    against torch fp32 autograd of the oracle on the GPU, 1e-4 relative."""
    import oracle.tgfr_oracle as O
    from text_guided_face_recognition_amd.models.attention import func_attention
    g = torch.Generator(device="cuda").manual_seed(3)
    q = torch.randn(3, 64, 17, generator=g, device="cuda")
    c = torch.randn(3, 64, 7, 9, generator=g, device="cuda")
    pw = torch.randn(3, 64, 17, generator=g, device="cuda")
    pa = torch.randn(3, 17, 7, 9, generator=g, device="cuda")
    outs = []
    for fn in (func_attention, O.func_attention):
        qq, cc = q.clone().requires_grad_(), c.clone().requires_grad_()
        w, a = fn(qq, cc, 4.0)
        ((w * pw).sum() + (a * pa).sum()).backward()
        outs.append((w.detach(), a.detach(), qq.grad, cc.grad))
    for x, y in zip(*outs):
        assert float((x - y).abs().max() / y.abs().max()) < 1e-4


@pytest.mark.parametrize("nb,hw,cq,c,cross", [
    (256, 36, 36, 36, True), (3, 36, 36, 36, False), (2, 49, 8, 20, True), (5, 64, 64, 64, False),
    (4, 5, 3, 7, True), (1, 1, 1, 1, False), (2, 65, 16, 16, True)])
def test_small_attention(nb, hw, cq, c, cross):
    """kernels.attention_core at FCFM sizes (HW <= 64: the fused
    tgfr_attn_small_fwd / _bwd, exact fp32; HW = 65 takes the composed path)
    against fp32 autograd on the GPU: 1e-5 of max on O and on each gradient
    slice; packed gradients must leave no column unwritten."""
    torch.backends.cuda.matmul.allow_tf32 = False
    g = torch.Generator(device="cuda").manual_seed(hw * 100 + cq)
    if cross:
        px = torch.randn(nb, hw, cq + c, generator=g, device="cuda")
        py = torch.randn(nb, hw, cq, generator=g, device="cuda")
        ck, cv = 0, cq
    else:
        px = torch.randn(nb, hw, 2 * cq + c, generator=g, device="cuda")
        py = None
        ck, cv = cq, 2 * cq
    do = torch.randn(nb, hw, c, generator=g, device="cuda")
    scale = 1.0 / float(cq) ** 0.5
    xr = px.clone().requires_grad_()
    yr = py.clone().requires_grad_() if cross else None
    mode = "fp32" if hw > 64 else "bf16"       # the fused path is fp32 in every mode
    o = K.attention_core(xr, yr, cq, ck, cv, scale, mode)
    dx, *dy = torch.autograd.grad(o, [xr] + ([yr] if cross else []), do)

    xe = px.clone().requires_grad_()
    ye = py.clone().requires_grad_() if cross else None
    ky = ye if cross else xe
    ref = torch.softmax(scale * xe[..., :cq] @ ky[..., ck:ck + cq].transpose(1, 2), -1) @ \
        xe[..., cv:]
    dxe, *dye = torch.autograd.grad(ref, [xe] + ([ye] if cross else []), do)
    tol = 1e-5 if hw <= 64 else 1e-4

    def rel(a, b):
        return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))

    assert rel(o, ref) < tol
    assert rel(dx, dxe) < tol
    if cross:
        assert rel(dy[0], dye[0]) < tol


def test_small_attention_abi_rejects():
    """tgfr_attn_small_* refuse shapes they cannot hold (HW > 64) and, for
    self-attention, overlapping gradient column ranges."""
    from text_guided_face_recognition_amd import _hip
    x = torch.zeros(1, 65, 8, device="cuda")
    o = torch.zeros(1, 65, 4, device="cuda")
    p = torch.zeros(1, 65 * 65, device="cuda")
    args = (x.data_ptr(), 65 * 8, 8, None, 0, 0, 1, 65, 2, 2, 4, 4, 1.0, o.data_ptr(), 65 * 4,
            4, p.data_ptr(), _hip.stream())
    assert _hip.lib().tgfr_attn_small_fwd(*args) == 1001
    bad = (x.data_ptr(), 64 * 8, 8, None, 0, 0, 1, 64, 4, 2, 4, 4, 1.0, p.data_ptr(),
           o.data_ptr(), 64 * 4, 4, x.data_ptr(), 64 * 8, 8, None, 0, 0, _hip.stream())
    assert _hip.lib().tgfr_attn_small_bwd(*bad) == 1001      # dK [2, 6) overlaps dQ [0, 4)
