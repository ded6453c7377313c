"""CPU checks of the word<->region host logic (kernels._wr_fwd / _wr_bwd)
with the C ABI replaced by a recorder: which entry points a call would
launch, with which guard arguments.  No kernel runs (no GPU here)."""
import torch

from text_guided_face_recognition_amd import kernels as K


def _record(monkeypatch):
    calls = []
    monkeypatch.setattr(K, "call", lambda name, *a: calls.append((name, a)))
    monkeypatch.setattr(K, "ptr", lambda t: None if t is None else t.data_ptr())
    monkeypatch.setattr(K._hip, "stream", lambda: 0)
    monkeypatch.setattr(K, "wr_bwd_ws_floats", lambda *a: 16)
    return calls


def _args(calls, name):
    return [a for n, a in calls if n == name]


def _inputs(nw, b_img=2, b_cap=3):
    torch.manual_seed(0)
    r = torch.randn(b_img, 256, 14, 14)
    w = torch.randn(b_cap, nw, 256)
    return r, w, torch.full((b_cap,), nw, dtype=torch.int32)


def test_t64_foreign_rows_get_device_guard(monkeypatch):
    """64-token captions, bounded (BERT path), words not made by this
    package's heads: the forward launches tgfr_wr_guard, passes the guard to
    tgfr_wr_fwd, prepares the exact twin's plain word rows, and the backward
    hands guard + plain rows to tgfr_wr_bwd_tok and tgfr_wr_bwd -- with no
    host read of the norms (VERDICT r4 missing #3)."""
    calls = _record(monkeypatch)
    item = torch.Tensor.item
    monkeypatch.setattr(torch.Tensor, "item", lambda t: (_ for _ in ()).throw(
        AssertionError("host read of a device value")))
    for mode in ("fp16", "bf16"):
        calls.clear()
        r, w, lens = _inputs(62)
        logits, att, saved, cfg = K._wr_fwd(r, w, lens, 4.0, 5.0, 10.0, mode, bounded=True)
        guard = _args(calls, "tgfr_wr_guard")
        assert len(guard) == 1
        fwd = _args(calls, "tgfr_wr_fwd")[0]
        assert fwd[-2] == guard[0][4] and fwd[-2] is not None      # the guard word
        assert fwd[-5] == 1 and fwd[-4] == 64                       # bounded, t_pad 64
        w_plain, g = saved[11], saved[12]
        assert w_plain is not None and g is not None and g.dtype == torch.int32
        # the plain rows are prepared unscaled (scale 1), the forward's scaled by log2(e)
        scales = [a[9] for n, a in calls if n in ("tgfr_prep_rows", "tgfr_prep_rows_f16")
                  and a[5] == 62]
        assert 1.0 in scales and any(abs(s - K.LOG2E) < 1e-6 for s in scales)

        def tok_call(stats, w_norm, r_norm, lens_, b_img, b_cap, fast, t_pad, tok, guard_):
            K.call("tgfr_wr_bwd_tok", None, None, None, None, b_img, b_cap, 4.0, 5.0, 10.0,
                   1e-8, None, b_cap, int(fast), t_pad, None, K.ptr(guard_), 0)
        calls.clear()
        K._wr_bwd(saved, cfg, tok_call)
        tok = _args(calls, "tgfr_wr_bwd_tok")[0]
        bwd = _args(calls, "tgfr_wr_bwd")[0]
        assert tok[-2] == g.data_ptr()
        assert bwd[-3] == w_plain.data_ptr() and bwd[-2] == g.data_ptr()
    monkeypatch.setattr(torch.Tensor, "item", item)


def test_t32_and_own_rows_take_no_guard(monkeypatch):
    """32-token captions decide per caption inside the max-free kernels (no
    guard, no plain rows); 64-token rows attached by this package's heads
    (unit rows) take no guard either."""
    calls = _record(monkeypatch)
    r, w, lens = _inputs(30)
    _, _, saved, _ = K._wr_fwd(r, w, lens, 4.0, 5.0, 10.0, "bf16", bounded=True)
    assert not _args(calls, "tgfr_wr_guard")
    assert _args(calls, "tgfr_wr_fwd")[0][-2] is None
    assert saved[11] is None and saved[12] is None
    # own rows: R and W carry the operand rows their producers attached
    calls.clear()
    r, w, lens = _inputs(62)
    rows_r = torch.zeros(2, K.RPAD, K.D, dtype=torch.int16)
    K.attach_rows(r, rows_r, torch.ones(2, K.RPAD), True)
    rows_w = torch.zeros(3, 64, K.D, dtype=torch.int16)
    K.attach_rows(w, rows_w, torch.ones(3, 64), True, scale=K.LOG2E)
    _, _, saved, _ = K._wr_fwd(r, w, lens, 4.0, 5.0, 10.0, "fp16", bounded=True, uniform=True)
    assert not _args(calls, "tgfr_wr_guard")
    assert saved[12] is None
