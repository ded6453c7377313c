"""GPU parity of the drop-in modules (models/*) against reference fixtures.

Reference weights (stored in the fixtures) are loaded into the drop-in
modules through their state-dict names, which match the reference's.
Tolerances: losses/logits 1e-3 absolute (fp32 mode); outputs 1e-4..1e-3;
gradients relative to their max magnitude.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden, t

pytestmark = pytest.mark.gpu


def _args(**kw):
    from text_guided_face_recognition_amd.config import make_args
    return make_args(**kw)


def _load(module, g, prefix=""):
    sd = module.state_dict()
    new = {}
    for k in sd:
        key = prefix + k.replace(".", "_")
        assert key in g, key
        new[k] = t(g[key])
    module.load_state_dict(new)
    return module


def _relerr(a, b):
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else a
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-12)


def _frob(a, b):
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else a
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-12)


def test_sent_global_clip(gpu):
    from text_guided_face_recognition_amd.models import losses as L
    args = _args()
    g = load_golden("sent_loss_b8")
    x = t(g["cnn_code"]).to(gpu).requires_grad_()
    s0, s1 = L.sent_loss(x, t(g["rnn_code"]).to(gpu), torch.arange(8, device=gpu),
                         g["class_ids"], 8, args)
    assert abs(s0.item() - float(g["loss0"])) < 1e-4
    assert abs(s1.item() - float(g["loss1"])) < 1e-4
    (s0 + s1).backward()
    assert _relerr(x.grad, g["d_cnn"]) < 1e-4

    g = load_golden("global_loss_b8")
    x = t(g["cnn_code"]).to(gpu).requires_grad_()
    gl = L.global_loss(x, t(g["rnn_code"]).to(gpu))
    assert abs(gl.item() - float(g["loss"])) < 1e-4
    gl.backward()
    assert _relerr(x.grad, g["d_cnn"]) < 1e-4

    g = load_golden("clip_loss_b8")
    x = t(g["image"]).to(gpu).requires_grad_()
    cl = L.ClipLoss()(t(g["text"]).to(gpu), x, args)
    assert abs(cl.item() - float(g["loss"])) < 1e-4
    cl.backward()
    assert _relerr(x.grad, g["d_image"]) < 1e-4

    g = load_golden("focal_loss_b8")
    x = t(g["logits"]).to(gpu).requires_grad_()
    fl = L.FocalLoss(gamma=2)(x, t(g["target"]).to(gpu))
    assert abs(fl.item() - float(g["loss"])) < 1e-5


@pytest.mark.parametrize("n", [8, 37, 64])
def test_sent_global_fused(gpu, n):
    """sent_loss + global_loss in one fused launch each way (kernels.SentGlobal,
    the single-process stage-1 path) against the oracle's two losses on the
    same inputs (duplicate class ids exercise the sent mask): losses 1e-4,
    the image-side gradient of s0 + 2 s1 + 3 gl 1e-4 of its max; and the
    reference's own sent_loss fixture."""
    from oracle import tgfr_oracle as O
    from text_guided_face_recognition_amd.models import losses as L
    gen = torch.Generator().manual_seed(n)
    x = torch.randn(n, 256, generator=gen)
    y = torch.randn(n, 256, generator=gen)
    cls = torch.randint(0, max(2, n // 3), (n,), generator=gen)
    xo = x.clone().requires_grad_()
    r0, r1, _ = O.sent_loss(xo, y, torch.arange(n), cls.numpy(), 10.0)
    rg, _ = O.global_loss(xo, y)
    (r0 + 2 * r1 + 3 * rg).backward()
    xg = x.to(gpu).requires_grad_()
    s0, s1, gl = L.sent_global_loss(xg, y.to(gpu), torch.arange(n, device=gpu), cls.numpy(), n,
                                    _args())
    for a, b in ((s0, r0), (s1, r1), (gl, rg)):
        assert abs(a.item() - b.item()) < 1e-4
    (s0 + 2 * s1 + 3 * gl).backward()
    assert _relerr(xg.grad, xo.grad.numpy()) < 1e-4
    if n == 8:
        g = load_golden("sent_loss_b8")
        xg = t(g["cnn_code"]).to(gpu).requires_grad_()
        s0, s1, _ = L.sent_global_loss(xg, t(g["rnn_code"]).to(gpu), torch.arange(8, device=gpu),
                                       g["class_ids"], 8, _args())
        assert abs(s0.item() - float(g["loss0"])) < 1e-4
        assert abs(s1.item() - float(g["loss1"])) < 1e-4
        (s0 + s1).backward()
        assert _relerr(xg.grad, g["d_cnn"]) < 1e-4


@pytest.mark.parametrize("n_r,world", [(64, 8), (16, 3), (37, 2), (64, 1), (128, 2), (100, 3),
                                       (128, 1)])
def test_sent_global_dist_ranks(gpu, n_r, world):
    """The per-rank sent_loss + global_loss kernels (tgfr_sent_global_dist_*,
    the one-process-per-GPU stage-1 path; n_r > 64 -- configs[4]'s 128 per
    rank -- in two 64-row tiles, each with its own column partials) with
    `world` ranks emulated in one process through the C ABI: every rank's
    forward, the column partials
    concatenated rank-major (what the all-gather delivers), every rank's loss
    and backward.  The summed contributions equal the oracle's global-batch
    losses (1e-4) and the stacked row gradients of s0 + 2 s1 + 3 gl its
    gradient (1e-4 of max); duplicate class ids exercise the sent mask across
    ranks (models/losses.py:19-57, :329-351)."""
    from oracle import tgfr_oracle as O
    from text_guided_face_recognition_amd import kernels as K
    from text_guided_face_recognition_amd._hip import call, ptr, stream
    n = n_r * world
    gen = torch.Generator().manual_seed(n + world)
    x = torch.randn(n, 256, generator=gen)
    y = torch.randn(n, 256, generator=gen)
    cls = torch.randint(0, max(2, n // 5), (n,), generator=gen)
    xo = x.clone().requires_grad_()
    r0, r1, _ = O.sent_loss(xo, y, torch.arange(n), cls.numpy(), 10.0)
    rg, _ = O.global_loss(xo, y)
    (r0 + 2 * r1 + 3 * rg).backward()
    xg, yg, cg = x.to(gpu), y.to(gpu), cls.to(gpu)
    n_rp, n_cp, n_st = K._sgd_ws(n_r, n)
    ranks = []
    for r in range(world):
        xr = xg[r * n_r:(r + 1) * n_r].contiguous()
        t_ = dict(cosv=torch.empty(n_r, n, device=gpu), rowpart=torch.empty(n_rp, device=gpu),
                  colpart=torch.empty(n_cp, device=gpu), nrm=torch.empty(n_r + n, device=gpu),
                  stats=torch.empty(n_st, device=gpu), loss=torch.empty(3, device=gpu), x=xr)
        call("tgfr_sent_global_dist_fwd", ptr(xr), 256, n_r, ptr(yg), 256, n, ptr(cg), r * n_r,
             10.0, 10.0, 1e-8, ptr(t_["cosv"]), ptr(t_["rowpart"]), ptr(t_["colpart"]),
             ptr(t_["nrm"]), stream())
        ranks.append(t_)
    parts = torch.stack([t_["colpart"] for t_ in ranks]).contiguous()
    gw = [torch.full((), v, device=gpu) for v in (1.0, 2.0, 3.0)]
    dx = torch.empty(n, 256, device=gpu)
    for r, t_ in enumerate(ranks):
        call("tgfr_sent_global_dist_loss", ptr(t_["cosv"]), n_r, n, r * n_r, 10.0, 10.0,
             ptr(t_["rowpart"]), ptr(parts), world, 0, 1.0 / n, ptr(t_["stats"]), ptr(t_["loss"]),
             stream())
        call("tgfr_sent_global_dist_bwd", ptr(gw[0]), ptr(gw[1]), ptr(gw[2]), ptr(t_["x"]), 256,
             n_r, ptr(yg), 256, n, ptr(cg), r * n_r, 10.0, 10.0, 1e-8, 1.0 / n,
             ptr(t_["cosv"]), ptr(t_["stats"]), ptr(t_["nrm"]), ptr(dx[r * n_r]), 256, stream())
    tot = torch.stack([t_["loss"] for t_ in ranks]).sum(0).cpu()
    for a, b in zip(tot.tolist(), (r0.item(), r1.item(), rg.item())):
        assert abs(a - b) < 1e-4, (a, b)
    assert _relerr(dx, xo.grad.numpy()) < 1e-4


@pytest.mark.parametrize("tag", ["c256_hw196", "c36_hw36"])
def test_self_attention(gpu, tag):
    from text_guided_face_recognition_amd.models.fusion_nets import SelfAttention
    g = load_golden(f"self_attention_{tag}")
    c = g["x"].shape[1]
    cross = tag == "c36_hw36"
    m = SelfAttention(c, scale=1).to(gpu)
    m.query_proj.weight.data = t(g["q_w"]).to(gpu)
    m.query_proj.bias.data = t(g["q_b"]).to(gpu)
    m.key_proj.weight.data = t(g["k_w"]).to(gpu)
    m.key_proj.bias.data = t(g["k_b"]).to(gpu)
    m.value_proj.weight.data = t(g["v_w"]).to(gpu)
    m.value_proj.bias.data = t(g["v_b"]).to(gpu)
    x = t(g["x"]).to(gpu).requires_grad_()
    y = t(g["y"]).to(gpu).requires_grad_() if cross else x
    out = m(x, y)
    assert _relerr(out, g["out"]) < 1e-4
    (out * t(g["probe"]).to(gpu)).sum().backward()
    assert _relerr(x.grad, g["d_x"]) < 2e-4
    if cross:
        assert _relerr(y.grad, g["d_y"]) < 2e-4
    assert _relerr(m.value_proj.weight.grad, g["d_v_w"]) < 2e-4
    assert _relerr(m.query_proj.weight.grad, g["d_q_w"]) < 2e-4


def test_working(gpu):
    from text_guided_face_recognition_amd.models.fusion_nets import Working
    g = load_golden("working_b3")
    net = _load(Working(256), g).to(gpu).train()
    img = t(g["img"]).to(gpu).requires_grad_()
    out = net(img, t(g["word"]).to(gpu), t(g["gl_img"]).to(gpu), t(g["sent"]).to(gpu))
    assert _relerr(out, g["out"]) < 1e-4
    (out * t(g["probe"]).to(gpu)).sum().backward()
    assert _relerr(img.grad, g["d_img"]) < 1e-3
    assert _relerr(net.sa.value_proj.weight.grad, g["d_sa_value_proj_weight"]) < 1e-3


@pytest.mark.parametrize("b,precision", [(256, "fp32"), (256, "bf16")])
def test_working_oracle_b256(gpu, b, precision):
    """Working (FCFM, fusion_nets.py:217-258) at the configs[3] batch B = 256
    against the oracle's restatement (oracle.working) with the same weights:
    output and the input / conv-weight gradients.  fp32 mode: 1e-4 output /
    1e-3 grads relative to the max.  bf16 mode: 3e-2 output relative to the
    max; gradients 1e-1 in relative Frobenius norm (a 2x2 pooling argmax that
    flips on a bf16 near-tie sends one element's gradient elsewhere, an O(1)
    error at that element that a max-relative bound cannot absorb)."""
    from oracle import tgfr_oracle as O
    from text_guided_face_recognition_amd.models.fusion_nets import Working, set_precision
    from test_gpu_step_parity import WORKING_KEYS, _cpu_params
    torch.manual_seed(7)
    net = set_precision(Working(256).to(gpu).train(), precision)
    gen = torch.Generator().manual_seed(b)
    img = torch.randn(b, 14, 14, 256, generator=gen)
    img = (img / img.norm(dim=-1, keepdim=True)).permute(0, 3, 1, 2)   # channels-last R
    word = torch.randn(b, 256, 22, generator=gen)
    gl, sent = torch.randn(b, 256, generator=gen), torch.randn(b, 256, generator=gen)
    probe = torch.randn(b, 640, generator=gen)
    p = _cpu_params(net, WORKING_KEYS)
    xo = img.clone().requires_grad_()
    ref = O.working(xo, word, gl, sent, p)
    (ref * probe).sum().backward()
    xg = img.to(gpu).requires_grad_()
    out = net(xg, word.to(gpu), gl.to(gpu), sent.to(gpu))
    (out * probe.to(gpu)).sum().backward()
    tol_o, tol_g = (1e-4, 1e-3) if precision == "fp32" else (3e-2, 1e-1)
    err = _relerr if precision == "fp32" else _frob
    assert _relerr(out, ref.detach().numpy()) < tol_o
    assert err(xg.grad, xo.grad.numpy()) < tol_g
    assert err(net.conv.weight.grad, p["conv_w"].grad.numpy()) < tol_g
    assert err(net.conv.bias.grad, p["conv_b"].grad.numpy()) < tol_g


@pytest.mark.parametrize("b,layout,precision", [
    (3, "cl", "fp32"), (5, "nchw", "fp32"), (64, "cl", "fp32"), (37, "cl", "bf16"),
    (256, "cl", "bf16"), (256, "cl", "fp32"), (1, "nchw", "bf16")])
def test_conv_relu_pool(gpu, b, layout, precision):
    """FCFM maxpool2(relu(conv3x3)) (fusion_nets.py:236-237) in one fused
    kernel each way (kernels.ConvReluPool) vs torch fp32 on the CPU: output,
    dx, dW, db.  The gradient reference routes the probe through the kernel's
    own 2x2 argmax / ReLU code, which is asserted equal to autograd's routing
    wherever the window's max is not a near-tie (and in fp32 mode, without
    near-ties, the gradients equal autograd's).  Tolerances relative to the
    max: fp32 mode 3e-5 out / 1e-4 grads; bf16 1e-2 / 2e-2."""
    import torch.nn.functional as F
    from text_guided_face_recognition_amd import kernels as K
    gen = torch.Generator().manual_seed(b * 1000 + 3)
    x = torch.randn(b, 256, 14, 14, generator=gen)
    wt = torch.randn(36, 256, 3, 3, generator=gen) / (3 * 256 ** 0.5)
    bias = torch.randn(36, generator=gen) * 0.1
    probe = torch.randn(b, 36, 6, 6, generator=gen)
    xo, wo, bo = (v.clone().requires_grad_() for v in (x, wt, bias))
    ref = F.max_pool2d(F.relu(F.conv2d(xo, wo, bo)), 2)
    (ref * probe).sum().backward()
    xd = x.to(gpu)
    if layout == "cl":
        xd = xd.contiguous(memory_format=torch.channels_last)
    xg, wg, bg = (v.to(gpu).requires_grad_() for v in (xd, wt, bias))
    out = K.conv_relu_pool(xg, wg, bg, mode=precision)
    assert out.shape == ref.shape
    (out * probe.to(gpu)).sum().backward()
    tol_o, tol_g = (3e-5, 1e-4) if precision == "fp32" else (1e-2, 2e-2)
    assert _relerr(out, ref.detach().numpy()) < tol_o
    # the probe routed by the kernel's own argmax / ReLU code
    _, code = K.conv_relu_pool_code(xg.detach(), wg.detach(), bg.detach(), mode=precision)
    code = code.long().cpu()
    sel = torch.nn.functional.one_hot(code.clamp(min=0), 4).float() * (code >= 0).unsqueeze(-1)
    # ... which is autograd's routing except at near-ties of the window's max
    conv = F.conv2d(x, wt, bias)
    win = conv.view(b, 36, 6, 2, 6, 2).permute(0, 1, 2, 4, 3, 5).reshape(b, 36, 6, 6, 4)
    top2 = win.topk(2, dim=-1).values
    thr = 1e-4 if precision == "fp32" else 3e-2
    clear = ((top2[..., 0] - top2[..., 1]) > thr) & (top2[..., 0].abs() > thr)
    ref_code = torch.where(win.amax(-1) > 0, win.argmax(-1), torch.full_like(code, -1))
    assert torch.equal(code[clear], ref_code[clear])
    gm = (sel * probe.unsqueeze(-1)).view(b, 36, 6, 6, 2, 2).permute(0, 1, 2, 4, 3, 5)
    gm = gm.reshape(b, 36, 12, 12)
    dx_ref = torch.nn.grad.conv2d_input(x.shape, wt, gm)
    dw_ref = torch.nn.grad.conv2d_weight(x, wt.shape, gm)
    assert _relerr(xg.grad, dx_ref.numpy()) < tol_g
    assert _relerr(wg.grad, dw_ref.numpy()) < tol_g
    assert _relerr(bg.grad, gm.sum(dim=(0, 2, 3)).numpy()) < tol_g
    if precision == "fp32" and bool(clear.all()):
        assert _relerr(xg.grad, xo.grad.numpy()) < tol_g
        assert _relerr(wg.grad, wo.grad.numpy()) < tol_g
        assert _relerr(bg.grad, bo.grad.numpy()) < tol_g


def test_image_heading(gpu):
    from text_guided_face_recognition_amd.models.models import ImageHeading
    g = load_golden("image_heading_b2")
    net = _load(ImageHeading(_args()), g).to(gpu).train()
    gi = t(g["global_image"]).to(gpu).requires_grad_()
    li = t(g["local_image"]).to(gpu).requires_grad_()
    gp, r = net(gi, li)
    assert _relerr(gp, g["g_out"]) < 1e-5
    assert _relerr(r, g["r_out"]) < 1e-4
    # R keeps the reference's channels-last physical layout
    assert r.stride() == (196 * 256, 1, 14 * 256, 256)
    ((gp * t(g["probe_g"]).to(gpu)).sum() + (r * t(g["probe_r"]).to(gpu)).sum()).backward()
    assert _relerr(gi.grad, g["d_global"]) < 1e-4
    assert _relerr(li.grad, g["d_local"]) < 1e-3
    assert _relerr(net.imim.sa.value_proj.weight.grad,
                   g["d_imim_sa_value_proj_weight"]) < 1e-3
    assert _relerr(net.imim.ln.weight.grad, g["d_imim_ln_weight"]) < 1e-3


def test_image_heading_bf16(gpu):
    """ImageHeading in bf16 mode (fused attention core operands in bf16, the
    fused IMIM tail) against the reference's fp32 outputs on the golden:
    relative Frobenius error <= 1e-2 on R and 1.2e-1 on the gradients (bf16
    operands; a ReLU mask flips where a pre-activation is within rounding of
    0, tests/test_gpu_tail.py)."""
    from text_guided_face_recognition_amd.models.models import ImageHeading
    g = load_golden("image_heading_b2")
    net = _load(ImageHeading(_args(precision="bf16")), g).to(gpu).train()
    assert net.imim.precision == "bf16"
    gi = t(g["global_image"]).to(gpu).requires_grad_()
    li = t(g["local_image"]).to(gpu).requires_grad_()
    gp, r = net(gi, li)

    def frob(a, ref):
        ref = torch.as_tensor(ref).to(a.device)
        return float((a.detach() - ref).norm() / ref.norm())

    assert frob(r, g["r_out"]) < 1e-2
    assert r.stride() == (196 * 256, 1, 14 * 256, 256)
    ((gp * t(g["probe_g"]).to(gpu)).sum() + (r * t(g["probe_r"]).to(gpu)).sum()).backward()
    errs = {"d_local": frob(li.grad, g["d_local"]),
            "d_v_w": frob(net.imim.sa.value_proj.weight.grad, g["d_imim_sa_value_proj_weight"]),
            "d_ln_w": frob(net.imim.ln.weight.grad, g["d_imim_ln_weight"]),
            "d_proj_w": frob(net.imim.project_local.projection.weight.grad,
                             g["d_imim_project_local_projection_weight"])}
    # the projection sits above the ReLUs; the rest see the flipped masks of
    # a 2-sample batch undamped
    assert errs["d_proj_w"] < 1e-2, errs
    assert max(errs.values()) < 1.2e-1, errs


@pytest.mark.parametrize("b", [64])
def test_image_heading_bf16_oracle(gpu, b):
    """ImageHeading in bf16 mode (the benchmarked IMIM: fused attention +
    fused tail) at the bench batch B = 64 against the oracle's fp32
    restatement (oracle.image_heading, models.py:328-405) on the same
    weights and inputs: relative Frobenius 1e-2 on g' and R, 1e-2 on the
    local projection's weight gradient, 1e-1 on every gradient below the
    ReLUs, and the key-role bias gradient ~0 (the softmax is invariant to it:
    1e-2 of the weight gradient's max).  Below the ReLUs the error is set by
    mask flips, not by rounding: a pre-activation within the bf16 operand
    error of 0 (~0.2 % of them) routes its gradient the other way, an O(1)
    error at that element, which is sqrt(0.2 %) ~ 5 % in relative Frobenius
    norm (measured: 5.0 - 8.9 %; R itself is within 1e-2)."""
    from oracle import tgfr_oracle as O
    from test_gpu_step_parity import HEAD_KEYS, _cpu_params
    from text_guided_face_recognition_amd.models.models import ImageHeading
    torch.manual_seed(11)
    net = ImageHeading(_args(precision="bf16")).to(gpu).train()
    keys = {k: v for k, v in HEAD_KEYS.items()}
    p = _cpu_params(net, keys)
    gen = torch.Generator().manual_seed(b)
    gi = torch.randn(b, 512, generator=gen)
    li = torch.randn(b, 256, 14, 14, generator=gen)
    probe_g = torch.randn(b, 256, generator=gen)
    probe_r = torch.randn(b, 256, 14, 14, generator=gen)
    gio, lio = gi.clone().requires_grad_(), li.clone().requires_grad_()
    g_ref, r_ref = O.image_heading(gio, lio, p)
    ((g_ref * probe_g).sum() + (r_ref * probe_r).sum()).backward()
    gig, lig = gi.to(gpu).requires_grad_(), li.to(gpu).requires_grad_()
    g_out, r_out = net(gig, lig)
    ((g_out * probe_g.to(gpu)).sum() + (r_out * probe_r.to(gpu)).sum()).backward()
    assert _frob(g_out, g_ref.detach().numpy()) < 1e-2
    assert _frob(r_out, r_ref.detach().numpy()) < 1e-2
    errs = {"d_global": _frob(gig.grad, gio.grad.numpy()),
            "d_local": _frob(lig.grad, lio.grad.numpy())}
    named = dict(net.named_parameters())
    zero = "imim.sa.query_proj.bias"   # key-role bias: softmax shift-invariant, gradient 0
    for k, v in keys.items():
        if k != zero and p[v].grad is not None and named[k].grad is not None:
            errs[k] = _frob(named[k].grad, p[v].grad.numpy())
    gq = named[zero].grad       # sum_j dS_ij = 0 only up to the bf16 rounding of dS
    assert gq is None or float(gq.abs().max()) < 1e-2 * float(
        named["imim.sa.query_proj.weight"].grad.abs().max())
    # the projection head and its input sit after the attention: bf16-operand
    # error only; through the attention / LN / BN backward the error of the
    # bf16 score and value products compounds (the fused kernel alone is held
    # to 2e-2, tests/test_gpu_attn.py)
    print("image_heading_bf16_oracle errs", {k: round(float(v), 5) for k, v in errs.items()})
    assert errs["d_global"] < 1e-3, errs
    assert errs["imim.project_local.projection.weight"] < 1e-2, errs
    assert max(errs.values()) < 1e-1, errs


def test_words_loss_module(gpu):
    """models.losses.words_loss end to end (fused kernel + CE kernel)."""
    from text_guided_face_recognition_amd.models import losses as L
    g = load_golden("words_loss_bert_b4_t30")
    args = _args(bert_words_num=int(g["bert_words_num"]))
    r = t(g["img_features"]).to(gpu).requires_grad_()
    l0, l1, att = L.words_loss(r, t(g["words_emb"]).to(gpu), torch.arange(4, device=gpu),
                               None, None, 4, args)
    assert abs(l0.item() - float(g["loss0"])) < 1e-3
    assert abs(l1.item() - float(g["loss1"])) < 1e-3
    assert len(att) == 4 and tuple(att[0].shape) == (1, 30, 14, 14)
    np.testing.assert_allclose(att[2][0].cpu().numpy(), g["att_diag"][2], atol=1e-4)
    (l0 + l1).backward()
    assert _relerr(r.grad, g["d_img"]) < 2e-3


def test_arc_margin_and_focal(gpu):
    """ArcMarginProduct (metrics.py:17-60) + FocalLoss (losses.py:313-325):
    fused kernels vs the oracle / the reference fixture, values and grads."""
    from oracle import tgfr_oracle as O
    from text_guided_face_recognition_amd.models.losses import FocalLoss
    from text_guided_face_recognition_amd.models.metrics import ArcMarginProduct
    torch.manual_seed(3)
    x = torch.randn(16, 256)
    head = ArcMarginProduct(256, 300, s=30, m=0.5).to(gpu)
    w = head.weight.detach().cpu().clone()
    lab = torch.randint(0, 300, (16,))
    xo, wo = x.clone().requires_grad_(), w.clone().requires_grad_()
    ref = O.focal_loss(O.arc_margin(xo, wo, lab, s=30, m=0.5), lab)
    ref.backward()
    xg = x.to(gpu).requires_grad_()
    out = FocalLoss(gamma=2)(head(xg, lab.to(gpu)), lab.to(gpu))
    out.backward()
    assert abs(out.item() - ref.item()) < 1e-4 * max(1.0, abs(ref.item()))
    assert _relerr(xg.grad, xo.grad.numpy()) < 1e-3
    assert _relerr(head.weight.grad, wo.grad.numpy()) < 1e-3

    g = load_golden("focal_loss_b8")
    lg = t(g["logits"]).to(gpu).requires_grad_()
    fl = FocalLoss(gamma=2)(lg, t(g["target"]).to(gpu))
    fl.backward()
    assert abs(fl.item() - float(g["loss"])) < 1e-5
    assert _relerr(lg.grad, g["d_logits"]) < 1e-4


@pytest.mark.parametrize("tag", ["s30_std", "s35_std", "s30_easy", "s35_easy"])
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_arc_margin_golden(gpu, tag, precision):
    """ArcMarginProduct against the REFERENCE's own outputs (models/metrics.py:
    17-60, tests/golden/arc_margin_b8.npz): logits 1e-5 relative, dW 1e-4,
    dx 1e-4 (fp32) / 1e-2 (the bf16 dx GEMM); rows on both sides of each
    margin branch.  Then both identity heads in one launch (kernels.IdentityHeads,
    text s=35 frozen input, image s=30) give the reference logits' focal losses
    (FocalLoss pinned by focal_loss_b8)."""
    from oracle import tgfr_oracle as O
    from text_guided_face_recognition_amd import kernels as K
    from text_guided_face_recognition_amd.models.metrics import ArcMarginProduct
    g = load_golden("arc_margin_b8")
    s_, kind = tag.split("_")
    easy = kind == "easy"
    head = ArcMarginProduct(256, 50, s=float(s_[1:]), m=float(g["m"]), easy_margin=easy).to(gpu)
    head.precision = precision
    with torch.no_grad():
        head.weight.copy_(t(g["weight"]))
    lab = t(g["label"]).to(gpu)
    x = t(g["x"]).to(gpu).requires_grad_()
    out = head(x, lab)
    (out * t(g["probe"]).to(gpu)).sum().backward()
    assert _relerr(out, g[f"out_{tag}"]) < 1e-5
    assert _relerr(head.weight.grad, g[f"d_w_{tag}"]) < 1e-4
    assert _relerr(x.grad, g[f"d_x_{tag}"]) < (1e-4 if precision == "fp32" else 1e-2)
    if kind == "std" and s_ == "s30":
        tc = ArcMarginProduct(256, 50, s=35, m=0.5).to(gpu)
        ic = ArcMarginProduct(256, 50, s=30, m=0.5).to(gpu)
        tc.precision = ic.precision = precision
        with torch.no_grad():
            tc.weight.copy_(t(g["weight"]))
            ic.weight.copy_(t(g["weight"]))
        xs = t(g["x"]).to(gpu)
        tid, iid = K.identity_heads(xs, tc, xs.clone().requires_grad_(), ic, lab, 2.0)
        lab_c = t(g["label"])
        rt = O.focal_loss(t(g["out_s35_std"]), lab_c).item()
        ri = O.focal_loss(t(g["out_s30_std"]), lab_c).item()
        assert abs(tid.item() - rt) < 1e-5 * max(1.0, rt)
        assert abs(iid.item() - ri) < 1e-5 * max(1.0, ri)


@pytest.mark.parametrize("b,d,c,easy,precision", [
    (64, 256, 4500, False, "bf16"), (64, 640, 1000, False, "fp32"), (13, 256, 300, True, "fp32"),
    (70, 128, 37, False, "bf16"), (256, 640, 4500, False, "bf16"), (200, 256, 300, True, "fp32")])
def test_arc_head_fused(gpu, b, d, c, easy, precision):
    """The fused ArcMarginProduct launches (tgfr_arc_fwd / tgfr_arc_bwd) vs torch
    fp32 autograd of F.linear(F.normalize(x), F.normalize(W)) + the margin:
    logits, dx (through the GEMM + l2-norm backward) and dW; ragged batch and
    class counts, D = 640 (the stage-2 head), easy margin; plus a frozen input
    (no dx path).  Tolerances: fp32 logits 1e-5, dW 1e-4, dx 1e-5 (the dx
    GEMM + l2-norm backward are exact fp32 in every mode, tgfr_arc_dx)."""
    import math
    from text_guided_face_recognition_amd.models.metrics import ArcMarginProduct
    gen = torch.Generator().manual_seed(b + d + c)
    x = torch.randn(b, d, generator=gen)
    lab = torch.randint(0, c, (b,), generator=gen)
    probe = torch.randn(b, c, generator=gen)
    head = ArcMarginProduct(d, c, s=30, m=0.5, easy_margin=easy).to(gpu)
    head.precision = precision
    w = head.weight.detach().cpu().clone()
    xo, wo = x.clone().requires_grad_(), w.clone().requires_grad_()
    cos = torch.nn.functional.linear(torch.nn.functional.normalize(xo),
                                     torch.nn.functional.normalize(wo))
    sine = torch.sqrt((1.0 - cos * cos).clamp(0, 1))
    phi = cos * math.cos(0.5) - sine * math.sin(0.5)
    if easy:
        phi = torch.where(cos > 0, phi, cos)
    else:
        phi = torch.where(cos > math.cos(math.pi - 0.5), phi,
                          cos - math.sin(math.pi - 0.5) * 0.5)
    one_hot = torch.zeros_like(cos).scatter_(1, lab.view(-1, 1), 1)
    ref = (one_hot * phi + (1 - one_hot) * cos) * 30
    (ref * probe).sum().backward()
    xg = x.to(gpu).requires_grad_()
    out = head(xg, lab.to(gpu))
    (out * probe.to(gpu)).sum().backward()
    assert _relerr(out, ref.detach().numpy()) < 1e-5
    assert _relerr(head.weight.grad, wo.grad.numpy()) < 1e-4
    assert _relerr(xg.grad, xo.grad.numpy()) < 1e-5
    # frozen input (the text classifier's sentence features): W grad only
    head.weight.grad = None
    out2 = head(x.to(gpu), lab.to(gpu))
    (out2 * probe.to(gpu)).sum().backward()
    assert _relerr(head.weight.grad, wo.grad.numpy()) < 1e-4


@pytest.mark.parametrize("b,c,precision", [(64, 4500, "fp32"), (64, 4500, "bf16"),
                                             (17, 300, "fp32"), (128, 4500, "fp32"),
                                             (100, 300, "fp32")])
def test_identity_heads(gpu, b, c, precision):
    """Both identity heads of the stage-1 step in one launch per direction
    (kernels.IdentityHeads: two ArcMargin heads, two focal losses, the focal
    gradient formed inside the ArcMargin backward) against the oracle's
    focal_loss(arc_margin(...)) per head (src/train_encoders_bert.py:293-306):
    losses 1e-5, dW of both heads 1e-4, dx of the trained (image) input 1e-5
    (exact fp32 in every mode, tgfr_arc_dx); the text input stays frozen."""
    from oracle import tgfr_oracle as O
    from text_guided_face_recognition_amd import kernels as K
    from text_guided_face_recognition_amd.models.metrics import ArcMarginProduct
    gen = torch.Generator().manual_seed(b + c)
    sent = torch.randn(b, 256, generator=gen)
    img = torch.randn(b, 256, generator=gen)
    lab = torch.randint(0, c, (b,), generator=gen)
    tc = ArcMarginProduct(256, c, s=35, m=0.5).to(gpu)
    ic = ArcMarginProduct(256, c, s=30, m=0.5).to(gpu)
    tc.precision = ic.precision = precision
    wt = tc.weight.detach().cpu().clone().requires_grad_()
    wi = ic.weight.detach().cpu().clone().requires_grad_()
    xo = img.clone().requires_grad_()
    rt = O.focal_loss(O.arc_margin(sent, wt, lab, s=35), lab)
    ri = O.focal_loss(O.arc_margin(xo, wi, lab, s=30), lab)
    (rt + 3.0 * ri).backward()
    xg = img.to(gpu).requires_grad_()
    tid, iid = K.identity_heads(sent.to(gpu), tc, xg, ic, lab.to(gpu), 2.0)
    assert abs(tid.item() - rt.item()) < 1e-5 and abs(iid.item() - ri.item()) < 1e-5
    (tid + 3.0 * iid).backward()
    assert _relerr(tc.weight.grad, wt.grad.numpy()) < 1e-4
    assert _relerr(ic.weight.grad, wi.grad.numpy()) < 1e-4
    assert _relerr(xg.grad, xo.grad.numpy()) < 1e-5


def test_l2norm_rows(gpu):
    from text_guided_face_recognition_amd import kernels as K
    torch.manual_seed(4)
    x = torch.randn(37, 256)
    x[5] = 1e-14                       # clamped row: y = x / eps
    xo = x.clone().requires_grad_()
    y_ref = torch.nn.functional.normalize(xo, dim=-1)
    probe = torch.randn_like(x)
    (y_ref * probe).sum().backward()
    xg = x.to(gpu).requires_grad_()
    y = K.l2norm_rows(xg)
    (y * probe.to(gpu)).sum().backward()
    torch.testing.assert_close(y.cpu(), y_ref.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(xg.grad.cpu(), xo.grad, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("rows,k,n,bias", [(64, 512, 256, True), (5, 512, 256, False),
                                           (33, 256, 96, True), (1, 612, 32, True),
                                           (300, 256, 96, True)])
def test_proj_l2norm(gpu, rows, k, n, bias):
    """normalize(x W^T + b) in one launch each way (kernels.ProjL2Norm:
    ImageHeading.project_global, models/models.py:98-120) vs torch float64 of
    F.normalize(F.linear(x, W, b)): values, dx, dW, db within 1e-5 relative
    (exact fp32 FMA); a zero row with no bias exercises the eps clamp; 300
    rows take the split-bf16 Linear + l2-norm path (5e-5)."""
    from text_guided_face_recognition_amd import kernels as K
    gen = torch.Generator().manual_seed(rows + k + n)
    x = torch.randn(rows, k, generator=gen)
    if not bias:
        x[2] = 0.0                                     # |y| = 0 < eps: y = 0, dy = dg / eps
    w = torch.randn(n, k, generator=gen) / k ** 0.5
    b = torch.randn(n, generator=gen) if bias else None
    probe = torch.randn(rows, n, generator=gen)
    xs = [t.double().clone().requires_grad_() for t in (x, w)] + \
        ([b.double().clone().requires_grad_()] if bias else [])
    ref = torch.nn.functional.normalize(
        torch.nn.functional.linear(xs[0], xs[1], xs[2] if bias else None), dim=1)
    (ref * probe.double()).sum().backward()
    xg = [t.to(gpu).requires_grad_() for t in (x, w)] + ([b.to(gpu).requires_grad_()] if bias
                                                          else [])
    y = K.proj_l2norm(xg[0], xg[1], xg[2] if bias else None)
    # the fused path for the trainers' batches (<= 64 rows), else Linear + l2-norm
    assert type(y.grad_fn).__name__ == ("ProjL2NormBackward" if rows <= 64
                                        else "L2NormRowsBackward")
    (y * probe.to(gpu)).sum().backward()
    tol = 1e-5 if rows <= 64 else 5e-5          # split-bf16 products on the fallback
    assert _relerr(y, ref.detach().numpy()) < tol
    for a, r in zip(xg, xs):
        assert _relerr(a.grad, r.grad.numpy()) < tol
    # a frozen input: no dx, the same dW
    w2 = w.to(gpu).requires_grad_()
    y2 = K.proj_l2norm(x.to(gpu), w2, b.to(gpu) if bias else None)
    (y2 * probe.to(gpu)).sum().backward()
    assert _relerr(w2.grad, xs[1].grad.numpy()) < tol


@pytest.mark.parametrize("rows,shape", [(64, (196, 256)), (3, (36, 6, 6)), (1, (4,))])
def test_layer_norm_rows(gpu, rows, shape):
    """Per-sample LayerNorm kernel vs torch fp32 F.layer_norm (values, dx, dw, db)."""
    from text_guided_face_recognition_amd import kernels as K
    gen = torch.Generator().manual_seed(5)
    x = (torch.randn(rows, *shape, generator=gen) * 3 + 1.5)
    w = torch.randn(*shape, generator=gen)
    b = torch.randn(*shape, generator=gen)
    probe = torch.randn(rows, *shape, generator=gen)
    xs = [x.clone().requires_grad_(), w.clone().requires_grad_(), b.clone().requires_grad_()]
    ref = torch.nn.functional.layer_norm(xs[0], shape, xs[1], xs[2], 1e-5)
    (ref * probe).sum().backward()
    xg = [x.to(gpu).requires_grad_(), w.to(gpu).requires_grad_(), b.to(gpu).requires_grad_()]
    y = K.layer_norm_rows(*xg, 1e-5)
    (y * probe.to(gpu)).sum().backward()
    torch.testing.assert_close(y.detach().cpu(), ref.detach(), rtol=1e-4, atol=1e-4)
    for a, r in zip(xg, xs):
        assert _relerr(a.grad, r.grad.numpy()) < 1e-4


@pytest.mark.parametrize("training", [True, False])
def test_bn_linear_fold(gpu, training):
    """bn_img folded into the q/k/v projection (kernels.BNLinear) vs torch
    BatchNorm2d + 1x1 conv in fp32: output, every gradient (incl. the BN affine
    and the input) and the running-statistics update."""
    from text_guided_face_recognition_amd import kernels as K
    torch.manual_seed(6)
    n, c, o = 3, 40, 72
    x = torch.randn(n, c, 5, 7) * 2 + 0.5
    bn = torch.nn.BatchNorm2d(c)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.normal_()
        bn.running_mean.normal_()
        bn.running_var.uniform_(0.5, 2.0)
    conv = torch.nn.Conv2d(c, o, 1)
    bn.train(training)
    bn_g = torch.nn.BatchNorm2d(c).to(gpu)
    bn_g.load_state_dict(bn.state_dict())
    bn_g.train(training)
    w = conv.weight.detach().clone().requires_grad_()
    b = conv.bias.detach().clone().requires_grad_()
    xr = x.clone().requires_grad_()
    ref = torch.nn.functional.conv2d(bn(xr), w, b)                # [n, o, 5, 7]
    ref_cl = ref.permute(0, 2, 3, 1).reshape(n, 35, o)
    probe = torch.randn(n, 35, o)
    (ref_cl * probe).sum().backward()
    wg = w.detach().to(gpu).requires_grad_()
    bg = b.detach().to(gpu).requires_grad_()
    xg = x.to(gpu).requires_grad_()
    y = K.bn_linear(xg, bn_g, wg, bg, mode="fp32")
    (y * probe.to(gpu)).sum().backward()
    assert _relerr(y, ref_cl.detach().numpy()) < 1e-5
    assert _relerr(xg.grad, xr.grad.numpy()) < 1e-4
    assert _relerr(wg.grad, w.grad.numpy()) < 1e-4
    assert _relerr(bg.grad, b.grad.numpy()) < 1e-5
    assert _relerr(bn_g.weight.grad, bn.weight.grad.numpy()) < 1e-4
    assert _relerr(bn_g.bias.grad, bn.bias.grad.numpy()) < 1e-5
    torch.testing.assert_close(bn_g.running_mean.cpu(), bn.running_mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(bn_g.running_var.cpu(), bn.running_var, rtol=1e-5, atol=1e-6)
    assert int(bn_g.num_batches_tracked) == int(bn.num_batches_tracked)


@pytest.mark.parametrize("n,c,h,w", [(4, 24, 5, 6), (64, 256, 14, 14), (13, 32, 3, 3)])
def test_layer_norm_rows_channel_major_affine(gpu, n, c, h, w):
    """IMIM layout: channels-last rows [HW, C] with the reference's [C, H, W]
    affine maps (ch = C; transposed once into the workspace)."""
    from text_guided_face_recognition_amd import kernels as K
    gen = torch.Generator().manual_seed(7)
    x = torch.randn(n, c, h, w, generator=gen) * 2 - 1
    wt = torch.randn(c, h, w, generator=gen)
    bs = torch.randn(c, h, w, generator=gen)
    probe = torch.randn(n, c, h, w, generator=gen)
    xs = [x.clone().requires_grad_(), wt.clone().requires_grad_(), bs.clone().requires_grad_()]
    ref = torch.nn.functional.layer_norm(xs[0], (c, h, w), xs[1], xs[2], 1e-5)
    (ref * probe).sum().backward()
    x_cl = x.permute(0, 2, 3, 1).reshape(n, h * w, c).contiguous().to(gpu).requires_grad_()
    wg, bg = wt.to(gpu).requires_grad_(), bs.to(gpu).requires_grad_()
    y = K.layer_norm_rows(x_cl, wg, bg, 1e-5, ch=c)
    p_cl = probe.permute(0, 2, 3, 1).reshape(n, h * w, c).to(gpu)
    (y * p_cl).sum().backward()
    ref_cl = ref.detach().permute(0, 2, 3, 1).reshape(n, h * w, c)
    torch.testing.assert_close(y.detach().cpu(), ref_cl, rtol=1e-4, atol=1e-4)
    dx_ref = xs[0].grad.permute(0, 2, 3, 1).reshape(n, h * w, c)
    assert _relerr(x_cl.grad, dx_ref.numpy()) < 1e-4
    assert _relerr(wg.grad, xs[1].grad.numpy()) < 1e-4
    assert _relerr(bg.grad, xs[2].grad.numpy()) < 1e-4
