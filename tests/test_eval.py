"""Verification / identification metrics (eval.py; reference
utils/modules.py:40-88) on CPU, and the pair-score kernel on the GPU.

The reference's utils package does not import here (easydict / nltk are
absent), so the metric definitions are pinned by hand-built
cases: a separable score set, a known EER crossing, the nearest-FPR rule of
get_tpr, and the identification grouping."""
import numpy as np
import pytest
import torch

from text_guided_face_recognition_amd import eval as E


def test_get_tpr_nearest_point():
    fprs = np.array([0.0, 2e-5, 9e-5, 2e-3, 1.0])
    tprs = np.array([0.1, 0.2, 0.3, 0.4, 1.0])
    # 1e-5: fpr 0 and 2e-5 are equally near -> the first; 1e-4 -> 9e-5;
    # 1e-3 -> 9e-5 (9.1e-4 away) rather than 2e-3 (1e-3 away)
    assert E.get_tpr(fprs, tprs) == pytest.approx([10.0, 30.0, 30.0])


def test_separable_scores():
    y_true = np.array([1] * 50 + [0] * 50)
    y_score = np.concatenate([np.linspace(0.6, 1.0, 50), np.linspace(-1.0, 0.4, 50)])
    r = E.calculate_scores(y_score, y_true, verbose=False)
    assert r["auc"] == pytest.approx(1.0)
    assert r["eer"] == pytest.approx(0.0)
    assert r["tpr@1e-3"] == pytest.approx(100.0)


def test_eer_crossing():
    # genuine ~ N(1, 1), impostor ~ N(-1, 1): EER = Phi(-1) ~ 0.1587
    rng = np.random.default_rng(0)
    g = rng.normal(1.0, 1.0, 200000)
    i = rng.normal(-1.0, 1.0, 200000)
    r = E.calculate_scores(np.concatenate([g, i]),
                           np.concatenate([np.ones_like(g), np.zeros_like(i)]), verbose=False)
    assert r["eer"] == pytest.approx(0.1587, abs=3e-3)
    assert r["auc"] == pytest.approx(0.9214, abs=3e-3)     # Phi(2 / sqrt(2))


def test_identification():
    s = np.array([[0.9, 0.1, 0.2], [0.3, 0.8, 0.1], [0.7, 0.2, 0.1]]).reshape(-1)
    assert E.calculate_identification_acc(s, 3) == pytest.approx(200 / 3)


@pytest.mark.gpu
def test_pair_scores_gpu(gpu):
    g = torch.Generator().manual_seed(1)
    a = torch.randn(300, 640, generator=g)
    b = torch.randn(300, 640, generator=g)
    b[5] = 0.0                                     # clamped row
    ref = torch.nn.CosineSimilarity(dim=1, eps=1e-6)(a, b)
    got = E.pair_scores(a.to(gpu), b.to(gpu)).cpu()
    assert torch.allclose(got, ref, atol=1e-6)
    ev = E.Evaluator()
    for i in range(3):
        ev.add(a[100 * i:100 * (i + 1)].to(gpu), b[100 * i:100 * (i + 1)].to(gpu),
               (torch.arange(100) % 2).tolist())
    r = ev.result(verbose=False)
    ref_r = E.calculate_scores(ref.numpy(), (torch.arange(300) % 100 % 2).numpy(), verbose=False)
    assert r == pytest.approx(ref_r)
