"""Calibrate the CPU oracle against the reference itself, timed side by side.

The reference is imported read-only in the build container (the SURVEY.md
8(c) recipe, as tests/golden/make_golden.py does: torchsummary / torchvision
stubbed, args.CUDA = False) and its own functions run on the SAME inputs, the
same cores and the same thread count as the oracle, interleaved rep by rep so
that clock drift hits both alike:

  words_loss fwd+bwd   B = 64, T = 30 (models/losses.py:61-135 vs oracle.words_loss)
  Working fwd+bwd      B = 256, T = 22 (models/fusion_nets.py:217-258 vs oracle.working)

The oracle must land within +-15 % of the reference.  Median
of 5 after 1 warm-up.  The reference is absent on GPU boxes: this runs here.

    PYTHONDONTWRITEBYTECODE=1 python tools/calibrate_oracle.py \
        [--reference /root/reference] [--threads 8] [--out profiles/r04/oracle_calibration.json]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import tgfr_oracle as O  # noqa: E402


def side_by_side(fa, fb, reps=5):
    """Median ms of fa and fb, one warm-up each, reps interleaved a, b, a, b..."""
    fa()
    fb()
    ta, tb = [], []
    for _ in range(reps):
        for fn, ts in ((fa, ta), (fb, tb)):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
    ta.sort()
    tb.sort()
    return ta[reps // 2] * 1000, tb[reps // 2] * 1000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r04",
                                                  "oracle_calibration.json"))
    a = ap.parse_args()
    from golden.make_golden import _Args, _import_reference
    _, ref_loss, ref_fus, _, _ = _import_reference(a.reference)
    torch.set_num_threads(a.threads)
    torch.manual_seed(100)
    unit = lambda x: x / x.norm(dim=-1, keepdim=True)  # noqa: E731

    # words_loss: the reference's own call (BERT path, labels = arange)
    b, nw = 64, 30
    r = unit(torch.randn(b, 14, 14, 256)).permute(0, 3, 1, 2).contiguous().requires_grad_()
    w = unit(torch.randn(b, nw, 256)).transpose(1, 2)
    labels = torch.arange(b)
    args = _Args("BERT", bert_words_num=nw + 2)

    def words_oracle():
        r.grad = None
        w0, w1, _, _ = O.words_loss(r, w, labels, None, nw, 4.0, 5.0, 10.0)
        (w0 + w1).backward()

    def words_ref():
        r.grad = None
        w0, w1, _ = ref_loss.words_loss(r, w, labels, None, None, b, args)
        (w0 + w1).backward()

    # Working (FCFM): the reference module and the oracle on the same weights
    from test_gpu_step_parity import WORKING_KEYS      # reference name -> oracle key
    bw, tw = 256, 22
    ref_net = ref_fus.Working(256).train()
    sd = ref_net.state_dict()
    p = {ok: sd[rk].detach().clone().requires_grad_() for rk, ok in WORKING_KEYS.items()}
    img = unit(torch.randn(bw, 14, 14, 256)).permute(0, 3, 1, 2).contiguous().requires_grad_()
    word = torch.randn(bw, 256, tw)
    gl, sent = torch.randn(bw, 256), torch.randn(bw, 256)

    def working_oracle():
        img.grad = None
        for v in p.values():
            v.grad = None
        O.working(img, word, gl, sent, p).sum().backward()

    def working_ref():
        img.grad = None
        ref_net.zero_grad(set_to_none=True)
        ref_net(img, word, gl, sent).sum().backward()

    res = {"threads": a.threads, "cpu": os.cpu_count(), "torch": torch.__version__,
           "protocol": "same process, same inputs and threads; median of 5 after 1 warm-up, "
                       "oracle and reference reps interleaved"}
    for name, fo, fr in (("words_loss_b64_t30", words_oracle, words_ref),
                         ("working_b256_t22", working_oracle, working_ref)):
        mo, mr = side_by_side(fo, fr)
        res[name] = {"oracle_ms": round(mo, 1), "reference_ms": round(mr, 1),
                     "ratio": round(mo / mr, 3), "within_15pct": abs(mo / mr - 1) <= 0.15}
        print(name, res[name], flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
