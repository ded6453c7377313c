"""Fused IMIM tail (csrc/tgfr_tail.hip; reference models/models.py:399-405 and
ProjectionHead :98-120): relu(conv1x1_1) -> relu(conv1x1_2) -> Linear ->
F.normalize, forward and backward.

Two references, both plain PyTorch fp32 on the GPU:
  * stage by stage through the C ABI: every stage's output against the same
    op with the kernel's operand rounding (bf16 operands, fp32 accumulation)
    applied to the kernel's own previous stage -- the kernel's logic, held
    to 1e-2 of the max magnitude on every output and gradient;
  * torch fp32 autograd of the reference ops: the numerics of bf16 mode, in
    relative Frobenius norm: 1e-2 on R and on the gradients above the ReLUs,
    8e-2 below them (a bf16 pre-activation within rounding of 0 flips its
    ReLU mask: ~0.2 % of the elements at these scales, ~6 % in norm)."""
import pytest
import torch
import torch.nn.functional as F

from text_guided_face_recognition_amd import kernels as K

pytestmark = pytest.mark.gpu


def _bf(t):
    return t.to(torch.bfloat16).float()


def _stagewise(z, w1, b1, w2, b2, wp, bp, dr, eps=1e-12):
    """Run the four C-ABI calls and check every stage against its bf16-operand
    restatement computed FROM THE KERNEL'S OWN previous stage (so a ReLU mask
    or a bf16 rounding that differs by accumulation order cannot cascade)."""
    from text_guided_face_recognition_amd import _hip
    from text_guided_face_recognition_amd._hip import call, ptr
    rows, dev = z.shape[0], z.device
    i16 = dict(dtype=torch.int16, device=dev)

    def bf(t):
        return (t.to(torch.int32) << 16).view(torch.float32)

    pk = torch.empty(_hip.lib().tgfr_tail_pack_elems(), **i16)
    call("tgfr_tail_pack", ptr(w1), ptr(w2), ptr(wp), ptr(pk), _hip.stream())
    r = torch.empty(rows, 256, device=dev)
    inv = torch.empty(rows, device=dev)
    zb, h1, h2 = (torch.empty(rows, n, **i16) for n in (256, 128, 256))
    call("tgfr_tail_fwd", ptr(z), 256, rows, ptr(pk), ptr(b1), ptr(b2), ptr(bp), eps, ptr(r),
         256, ptr(zb), ptr(h1), ptr(h2), ptr(inv), None, None, 0, 0, 0, _hip.stream())
    dz = torch.empty(rows, 256, device=dev)
    dp, dh2, dh1 = (torch.empty(rows, n, **i16) for n in (256, 256, 128))
    call("tgfr_tail_bwd", ptr(dr), 256, ptr(r), 256, ptr(inv), rows, eps, ptr(pk), ptr(h1),
         ptr(h2), ptr(dz), 256, ptr(dp), ptr(dh2), ptr(dh1), _hip.stream())
    ws = torch.empty(K.tail_dw_ws_floats(rows), device=dev)
    out = [torch.empty(*s, device=dev) for s in ((256, 256), (256,), (256, 128), (256,),
                                                 (128, 256), (128,))]
    call("tgfr_tail_dw", ptr(dp), ptr(h2), ptr(dh2), ptr(h1), ptr(dh1), ptr(zb), rows,
         *[ptr(o) for o in out], ptr(ws), _hip.stream())
    w1b, w2b, wpb = _bf(w1), _bf(w2), _bf(wp)
    Z, H1, H2, DP, DH2, DH1 = (bf(t) for t in (zb, h1, h2, dp, dh2, dh1))
    p = H2 @ wpb.t() + bp
    checks = {
        "Zb": (Z, _bf(z)),
        "H1": (H1, _bf(F.relu(Z @ w1b.t() + b1))),
        "H2": (H2, _bf(F.relu(H1 @ w2b.t() + b2))),
        "R": (r, p / p.norm(dim=-1, keepdim=True).clamp_min(eps)),
        "inv": (inv, 1.0 / p.norm(dim=-1).clamp_min(eps)),
        "dP": (DP, _bf((dr - r * (r * dr).sum(-1, keepdim=True)) * inv[:, None])),
        "dH2": (DH2, _bf((DP @ wpb) * (H2 > 0))),
        "dH1": (DH1, _bf((DH2 @ w2b) * (H1 > 0))),
        "dZ": (dz, DH1 @ w1b),
        "dWp": (out[0], DP.t() @ H2), "dbp": (out[1], DP.sum(0)),
        "dW2": (out[2], DH2.t() @ H1), "db2": (out[3], DH2.sum(0)),
        "dW1": (out[4], DH1.t() @ Z), "db1": (out[5], DH1.sum(0)),
    }
    return checks


def _fp32(z, w1, b1, w2, b2, wp, bp, dr):
    ts = [t.detach().clone().requires_grad_() for t in (z, w1, b1, w2, b2, wp, bp)]
    h1 = F.relu(ts[0] @ ts[1].t() + ts[2])
    h2 = F.relu(h1 @ ts[3].t() + ts[4])
    r = F.normalize(h2 @ ts[5].t() + ts[6], dim=-1)
    return (r,) + torch.autograd.grad(r, ts, dr)


def _maxrel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _frob(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _inputs(rows, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)

    def rnd(*s, scale=1.0):
        return torch.randn(*s, generator=g, device="cuda") * scale

    return (rnd(rows, 256), rnd(128, 256, scale=0.0625), rnd(128, scale=0.1),
            rnd(256, 128, scale=0.088), rnd(256, scale=0.1), rnd(256, 256, scale=0.0625),
            rnd(256, scale=0.1), rnd(rows, 256))


def _run(z, w1, b1, w2, b2, wp, bp, dr):
    ins = [z.clone().requires_grad_(), w1.reshape(128, 256, 1, 1).clone().requires_grad_(),
           b1.clone().requires_grad_(), w2.reshape(256, 128, 1, 1).clone().requires_grad_(),
           b2.clone().requires_grad_(), wp.clone().requires_grad_(), bp.clone().requires_grad_()]
    r = K.ImimTail.apply(*ins, 1e-12)
    gr = torch.autograd.grad(r, ins, dr)
    return (r.detach(), gr[0], gr[1].reshape(128, 256), gr[2], gr[3].reshape(256, 128), gr[4],
            gr[5], gr[6])


NAMES = ["R", "dZ", "dW1", "db1", "dW2", "db2", "dWp", "dbp"]


@pytest.mark.parametrize("rows", [12544, 588, 5])
def test_tail_stagewise(rows):
    torch.backends.cuda.matmul.allow_tf32 = False
    for n, (a, b) in _stagewise(*_inputs(rows, rows)).items():
        assert a.shape == b.shape, n
        assert _maxrel(a, b) <= 1e-2, (n, _maxrel(a, b))


@pytest.mark.parametrize("rows", [12544, 588])
def test_tail_vs_fp32(rows):
    torch.backends.cuda.matmul.allow_tf32 = False
    ins = _inputs(rows, rows + 1)
    got = _run(*ins)
    ref = _fp32(*ins)
    # order of _fp32's grads: z, w1, b1, w2, b2, wp, bp
    errs = {n: _frob(a, b.detach().reshape(a.shape)) for n, a, b in zip(NAMES, got, ref)}
    # above the ReLUs 1e-2; below them the bf16 pre-activations flip the
    # mask of ~0.2 % of the elements, which alone is ~6 % in Frobenius norm
    for n, e in errs.items():
        assert e <= (1e-2 if n in ("R", "dWp", "dbp") else 8e-2), errs


def test_tail_deterministic():
    """Two launches on the same inputs give identical bits (slice-ordered
    weight-gradient reduction, no atomics)."""
    ins = _inputs(2000, 7)
    a, b = _run(*ins), _run(*ins)
    for n, x, y in zip(NAMES, a, b):
        assert torch.equal(x, y), n


@pytest.mark.parametrize("rows,n,k,yf32", [(12544, 768, 256, True), (1000, 128, 384, False),
                                           (37, 256, 128, True)])
def test_dw_bf16_generic(rows, n, k, yf32):
    """tgfr_dw_bf16 (the q/k/v projection's weight gradient): dW = X^T Y and
    db = colsum(X) against torch on the same bf16-rounded operands, 1e-2 of
    the max magnitude (fp32 accumulation in a different order)."""
    from text_guided_face_recognition_amd import _hip
    from text_guided_face_recognition_amd._hip import call, ptr
    torch.backends.cuda.matmul.allow_tf32 = False
    g = torch.Generator(device="cuda").manual_seed(rows + n)
    x = torch.randn(rows, n, generator=g, device="cuda").to(torch.bfloat16)
    y = torch.randn(rows, k, generator=g, device="cuda")
    yb = y.to(torch.bfloat16)
    import ctypes
    out = (ctypes.c_longlong * 1)()
    assert _hip.lib().tgfr_dw_bf16_ws(rows, n, k, ctypes.addressof(out)) == 0
    ws = torch.empty(int(out[0]), device="cuda")
    dw = torch.empty(n, k, device="cuda")
    db = torch.empty(n, device="cuda")
    yarg = y if yf32 else yb.view(torch.int16)
    call("tgfr_dw_bf16", ptr(x.view(torch.int16)), ptr(yarg), int(yf32), rows, n, k, ptr(dw),
         ptr(db), ptr(ws), _hip.stream())
    ref = x.float().t() @ yb.float()
    assert _maxrel(dw, ref) <= 1e-2
    assert _maxrel(db, x.float().sum(0)) <= 1e-2


@pytest.mark.parametrize("precision", ["bf16", "fp16"])
def test_imim_operand_rows(gpu, precision):
    """The IMIM tail kernel writes R a second time in the word<->region
    operand layout (models/models.py:399-405 -> models/losses.py:96): those
    rows equal tgfr_prep_rows' hi plane of the returned R bit for bit (zero
    padding rows included), the norms |R_r| agree to rounding, and the tag is
    dropped once R changes in place."""
    from text_guided_face_recognition_amd import kernels as K
    from text_guided_face_recognition_amd.config import make_args
    from text_guided_face_recognition_amd.models.models import ImageHeading
    torch.manual_seed(3)
    args = make_args(precision=precision)
    head = ImageHeading(args).to(gpu)
    g = torch.randn(5, 512, device=gpu)
    local = torch.randn(5, 256, 14, 14, device=gpu)
    _, r = head(g, local)
    f16 = precision == "fp16"
    rows = K.attached_rows(r, f16)
    assert rows is not None and K.attached_rows(r, not f16) is None
    hi, _, nrm = K.prep_rows(K.regions_view(r.detach().float()), 196, 224, want_norms=True,
                             f16=f16)
    assert torch.equal(rows[0], hi)
    torch.testing.assert_close(rows[1], nrm, atol=1e-6, rtol=1e-5)
    with torch.no_grad():
        r.mul_(2.0)
    assert K.attached_rows(r, f16) is None


@pytest.mark.parametrize("n,hw", [(64, 196), (3, 49), (2, 32)])
def test_ln_tail_fused(n, hw):
    """IMIM's LayerNorm fused into the tail (kernels.ImimLnTail: the
    normalisation applied on the tail's load, the LayerNorm backward's sums in
    the tail backward's epilogue) against the two-Function composition
    LayerNormRows(ch = 256) -> ImimTail on the same inputs: R and every
    gradient (x, LN w / b, tail weights / biases).  The normalised values are
    the same fp32 expression, so the bf16 operands agree except where a
    rounding boundary is crossed: 2e-3 of the max on R, 1e-2 on gradients;
    odd hw makes 32-row workgroups straddle samples."""
    torch.backends.cuda.matmul.allow_tf32 = False
    z, w1, b1, w2, b2, wp, bp, dr = _inputs(n * hw, n + hw)
    g = torch.Generator(device="cuda").manual_seed(hw)
    x = (z * 2.0 + 0.5).reshape(n, hw, 256)
    lnw = torch.randn(256, hw, generator=g, device="cuda") * 0.3 + 1.0
    lnb = torch.randn(256, hw, generator=g, device="cuda") * 0.1
    dr = dr.reshape(n, hw, 256)

    def leaves():
        return [t.clone().requires_grad_() for t in (x, lnw, lnb, w1.reshape(128, 256, 1, 1),
                                                     b1, w2.reshape(256, 128, 1, 1), b2, wp, bp)]

    a = leaves()
    ra = K.ImimLnTail.apply(*a, 1e-5, 1e-12)
    ga = torch.autograd.grad(ra, a, dr)
    b = leaves()
    zb = K.layer_norm_rows(b[0], b[1], b[2], 1e-5, ch=256)
    rb = K.ImimTail.apply(zb.reshape(-1, 256), *b[3:], 1e-12).reshape(n, hw, 256)
    gb = torch.autograd.grad(rb, b, dr)
    assert _maxrel(ra, rb) <= 2e-3
    for i, (p, q) in enumerate(zip(ga, gb)):
        assert _maxrel(p, q) <= 1e-2, (i, _maxrel(p, q))


@pytest.mark.parametrize("n,precision", [(64, "bf16"), (3, "fp16")])
def test_imim_fused_node(gpu, n, precision):
    """The whole IMIM head as one autograd node (kernels.ImimFused: one weight
    preparation launch, the LayerNorm backward writing the attention
    backward's bf16 dO and D itself, the LayerNorm moments from the attention
    epilogue) against the two-node chain ImimAttention -> ImimLnTail on the same
    module.  The moments are summed in another order, so a bf16 rounding of
    the normalised map can differ: R and the attached operand rows within
    5e-3 of their max (measured 2.3e-3 at B = 64), every parameter gradient
    within 1e-2; BN's running statistics are updated once."""
    import copy
    from text_guided_face_recognition_amd.config import make_args
    from text_guided_face_recognition_amd.models.models import IMIM
    torch.manual_seed(11)
    args = make_args(precision=precision)
    a = IMIM(args, 256).to(gpu)
    for p_ in a.parameters():
        p_.data.add_(torch.randn_like(p_) * 0.05)
    b = copy.deepcopy(a)
    x = torch.randn(n, 256, 14, 14, device=gpu) * 1.5 + 0.3
    probe = torch.randn(n, 256, 14, 14, device=gpu)
    ra = a(x)
    assert K.attached_rows(ra, precision == "fp16") is not None
    (ra * probe).sum().backward()
    f16 = precision == "fp16"
    z = K.imim_attention(x, b.bn_img, b.sa, 1.0 / float(b.sa.sqrt_dim))
    zb, (rows_b, _) = K.imim_ln_tail(z, b.ln, b.conv1x1_1, b.conv1x1_2,
                                     b.project_local.projection,
                                     rows_spec=(196, K.RPAD, f16))
    rb = zb.reshape(n, 14, 14, -1).permute(0, 3, 1, 2)
    (rb * probe).sum().backward()
    assert _maxrel(ra.detach(), rb.detach()) <= 5e-3
    dt = torch.float16 if f16 else torch.bfloat16
    assert _maxrel(K.attached_rows(ra, f16)[0].view(dt).float(), rows_b.view(dt).float()) <= 5e-3
    # the key-role projection's bias only shifts every score of a query by the
    # same amount (softmax-invariant): its gradient is rounding noise, so the
    # three projection biases are held to the largest one's scale
    bscale = max(float(getattr(b.sa, m).bias.grad.abs().max())
                 for m in ("key_proj", "query_proj", "value_proj"))
    for (na, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        if pb.grad is None:
            assert pa.grad is None, na
            continue
        if na.startswith("sa.") and na.endswith("_proj.bias"):
            err = float((pa.grad - pb.grad).abs().max()) / bscale
        else:
            err = _maxrel(pa.grad, pb.grad)
        assert err <= 1e-2, (na, err)
    torch.testing.assert_close(a.bn_img.running_mean, b.bn_img.running_mean)
    torch.testing.assert_close(a.bn_img.running_var, b.bn_img.running_var)


@pytest.mark.parametrize("n,precision", [(64, "bf16"), (13, "bf16"), (3, "fp16")])
def test_imim_ln_dw_deferred(gpu, n, precision, monkeypatch):
    """The IMIM LayerNorm's dw / db summed by the weight gradients' reduce
    launch (tgfr_imim_dw_ln, TGFR_LN_DW_DEFER=1, the default) against its own
    reduce launch (ln_bwd_dw, TGFR_LN_DW_DEFER=0): the same group partials
    summed in the same order, so every gradient is bit-identical (n = 13: a
    ragged last group of 5 samples; n = 64: 8 groups)."""
    import copy
    from text_guided_face_recognition_amd.config import make_args
    from text_guided_face_recognition_amd.models.models import IMIM
    torch.manual_seed(n)
    a = IMIM(make_args(precision=precision), 256).to(gpu)
    for p_ in a.parameters():
        p_.data.add_(torch.randn_like(p_) * 0.05)
    b = copy.deepcopy(a)
    x = torch.randn(n, 256, 14, 14, device=gpu) * 1.5 + 0.3
    probe = torch.randn(n, 256, 14, 14, device=gpu)
    for m, flag in ((a, "1"), (b, "0")):
        monkeypatch.setenv("TGFR_LN_DW_DEFER", flag)
        (m(x) * probe).sum().backward()
    torch.cuda.synchronize()
    assert b.ln.weight.grad.abs().max() > 0
    for (na, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        assert (pa.grad is None) == (pb.grad is None), na
        if pa.grad is not None:
            assert torch.equal(pa.grad, pb.grad), na


@pytest.mark.parametrize("n,hw", [(64, 196), (5, 196), (3, 144)])
def test_bn_qkv_fused(gpu, n, hw):
    """tgfr_bn_qkv_bf16 (BN apply + the packed q/k/v projection in one launch,
    reading the NCHW map) against the two-pass path it replaces
    (tgfr_bn_fwd_cl_bf16's normalised map -> tgfr_linear_bf16io): the same
    bf16 xhat bit for bit, px within one bf16 rounding of it (the fp32 sums
    run in another order), and both against an fp32 torch reference of
    bn -> 1x1 projection on the same folded weights."""
    from text_guided_face_recognition_amd._hip import call, ptr, stream
    torch.manual_seed(hw + n)
    c, o = 256, 768
    x = (torch.randn(n, c, hw, device=gpu) * 1.7 + 0.4).contiguous()
    wf = torch.randn(o, c, device=gpu) / 16
    bf = torch.randn(o, device=gpu)
    mean = torch.empty(c, device=gpu)
    rstd = torch.empty(c, device=gpu)
    xh2 = torch.empty(n, hw, c, dtype=torch.int16, device=gpu)
    call("tgfr_bn_fwd_cl_bf16", ptr(x), n, c, hw, 1e-5, 0.1, 1, None, None, None, ptr(mean),
         ptr(rstd), ptr(xh2), stream())
    y2 = torch.empty(n * hw, o, dtype=torch.int16, device=gpu)
    call("tgfr_linear_bf16io", ptr(xh2), c, n * hw, c, ptr(wf), c, ptr(bf), o, ptr(y2), o,
         stream())
    xh1 = torch.empty_like(xh2)
    y1 = torch.empty_like(y2)
    wfb = wf.to(torch.bfloat16).view(torch.int16)     # (RNE, as the two-pass path rounds)
    call("tgfr_bn_qkv_bf16", ptr(x), n, c, hw, ptr(mean), ptr(rstd), ptr(wfb), ptr(bf), o,
         ptr(y1), ptr(xh1), stream())
    torch.cuda.synchronize()
    assert torch.equal(xh1, xh2)
    bf16 = lambda t: t.view(torch.bfloat16).float()   # noqa: E731
    p1, p2 = bf16(y1), bf16(y2)
    ref = bf16(xh2).reshape(n * hw, c) @ wf.to(torch.bfloat16).float().t() + bf
    scale = ref.abs().max().item()
    e12 = (p1 - p2).abs().max().item() / scale
    e1 = (p1 - ref).abs().max().item() / scale
    print(f"bn_qkv n={n} hw={hw}: fused vs two-pass {e12:.2e}, vs fp32 {e1:.2e} of max")
    assert e12 < 1e-2 and e1 < 1e-2
    assert torch.isfinite(p1).all()
