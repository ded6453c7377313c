"""GPU parity of TextHeading (models/models.py:170-232) through the C ABI
(tgfr_text_heading): against the reference's own outputs in the fixtures,
and against the CPU oracle (oracle/tgfr_oracle.py:text_heading) on seeded
inputs up to BASELINE config 5's 64-token captions.

Tolerances: fp32 mode 1e-4 absolute on unit-norm words and sentence codes
(the conv contractions run as bf16 hi/lo MFMA triples, ~2^-17 relative per
product over 1536-3072 terms); bf16 mode 2e-2 absolute.  The per-token max
picks are checked exactly: every word row must equal the normalised max of
the oracle's relu'd maps up to that tolerance."""
import numpy as np
import pytest
import torch

from conftest import t, text_heading_golden
from oracle import tgfr_oracle as O

pytestmark = pytest.mark.gpu


def _head(L, precision="fp32"):
    from text_guided_face_recognition_amd.config import make_args
    from text_guided_face_recognition_amd.models.models import TextHeading
    args = make_args(bert_words_num=L, precision=precision)
    return TextHeading(args)


def _set(net, ws, bs, dev):
    with torch.no_grad():
        for conv, w, b in zip(net.bwm.convs1, ws, bs):
            conv.weight.copy_(torch.as_tensor(w))
            conv.bias.copy_(torch.as_tensor(b))
    return net.to(dev)


@pytest.mark.parametrize("tag", ["b3_l32", "b2_l24"])
def test_text_heading_reference_fixture(gpu, tag):
    g = text_heading_golden(f"text_heading_{tag}")
    L = int(g["bert_words_num"])
    net = _set(_head(L), g["conv_w"], g["conv_b"], gpu)
    with torch.no_grad():
        words, sent = net(t(g["words_emb"]).to(gpu), None)
    torch.cuda.synchronize()
    assert words.shape == g["words_out"].shape
    # the reference layout: [B, 256, L-2] view of [B, L-2, 256] storage
    assert words.stride(1) == 1 and words.stride(2) == 256
    np.testing.assert_allclose(words.cpu().numpy(), g["words_out"], atol=1e-4)
    np.testing.assert_allclose(sent.cpu().numpy(), g["sent_out"], atol=1e-4)


@pytest.mark.parametrize("b,L,precision,atol", [
    (64, 32, "fp32", 1e-4), (128, 64, "fp32", 1e-4), (5, 5, "fp32", 1e-4),
    (64, 32, "bf16", 2e-2), (7, 24, "bf16", 2e-2)])
def test_text_heading_vs_oracle(gpu, b, L, precision, atol):
    torch.manual_seed(b * 1000 + L)
    net = _head(L, precision).to(gpu)
    x = torch.randn(b, L - 1, 768)
    with torch.no_grad():
        words, sent = net(x.to(gpu))
        ow, os_ = O.text_heading(x, [c.weight.cpu() for c in net.bwm.convs1],
                                 [c.bias.cpu() for c in net.bwm.convs1], L)
    torch.cuda.synchronize()
    np.testing.assert_allclose(words.cpu().numpy(), ow.numpy(), atol=atol)
    np.testing.assert_allclose(sent.cpu().numpy(), os_.numpy(), atol=atol)
    # size-independent properties: unit rows
    n = words.float().norm(dim=1)
    assert torch.allclose(n, torch.ones_like(n), atol=1e-4)
    assert torch.allclose(sent.norm(dim=1), torch.ones(b, device=gpu), atol=1e-4)


def test_text_heading_contract(gpu):
    net = _head(32).to(gpu)
    x = torch.randn(2, 31, 768, device=gpu)
    with pytest.raises(RuntimeError):          # grads requested: forward-only
        net(x)
    with torch.no_grad(), pytest.raises(ValueError):
        net(torch.randn(2, 30, 768, device=gpu))   # token count != bert_words_num - 1


@pytest.mark.parametrize("L,precision", [(32, "bf16"), (64, "fp16"), (24, "fp16")])
def test_text_heading_operand_rows(gpu, L, precision):
    """In the bf16 / fp16 modes TextHeading's pooling launch also writes the
    words as the word<->region kernels' log2(e)-scaled operand rows (attached
    to the returned words): bit-equal to tgfr_prep_rows of the returned words,
    padding rows zero, norms equal to rounding -- and found through the view
    words_loss hands the kernels (models/losses.py:83-96)."""
    from text_guided_face_recognition_amd import kernels as K
    torch.manual_seed(L)
    net = _head(L, precision).to(gpu)
    with torch.no_grad():
        words, _ = net(torch.randn(9, L - 1, 768, device=gpu))
    T = L - 2
    t_pad = 32 if T <= 32 else 64
    f16 = precision == "fp16"
    view = K.words_view(words, T)
    rows = K.attached_rows(view, f16, scale=K.LOG2E)
    assert rows is not None and K.attached_rows(view, f16) is None
    hi, _, nrm = K.prep_rows(view.float(), T, t_pad, want_norms=True, scale=K.LOG2E, f16=f16)
    assert rows[0].shape == hi.shape and torch.equal(rows[0], hi)
    torch.testing.assert_close(rows[1], nrm, atol=1e-6, rtol=1e-5)
