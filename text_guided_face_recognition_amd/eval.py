"""Face verification / identification evaluation: the reference's
utils/modules.py:40-168.

The reference's ``test()`` runs the frozen encoders over image/caption pairs,
fuses the features (concat / linear / FCFM) and scores each pair by
``nn.CosineSimilarity(dim=1, eps=1e-6)`` (:152-153); ``calculate_scores`` then
reports ROC AUC, EER and TPR at FPR 1e-5 / 1e-4 / 1e-3 (:51-72) and
``calculate_identification_acc`` the rank-1 identification accuracy
(:76-88).  Here the pair scores come from the gfx950 kernel
``tgfr_pair_cosine`` and the metrics follow the reference's definitions
(sklearn's ROC curve, flipped; EER at the closest FNR = FPR point; TPR at the
ROC point nearest each target FPR).  ``Evaluator`` accumulates device scores
across batches with no host sync until ``result()``.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ._hip import call, ptr
from ._hip import stream as _stream

FPR_TARGETS = (1e-5, 1e-4, 1e-3)


def pair_scores(out1, out2, eps=1e-6):
    """Cosine of matched rows, [N, D] x [N, D] -> [N] (device tensors)."""
    if out1.shape != out2.shape or out1.dim() != 2:
        raise ValueError(f"pair_scores needs two [N, D] tensors, got {tuple(out1.shape)} "
                         f"and {tuple(out2.shape)}")
    x = out1.float()
    y = out2.float()
    if x.stride(1) != 1:
        x = x.contiguous()
    if y.stride(1) != 1:
        y = y.contiguous()
    out = torch.empty(x.shape[0], dtype=torch.float32, device=x.device)
    call("tgfr_pair_cosine", ptr(x), x.stride(0), ptr(y), y.stride(0), x.shape[0], x.shape[1],
         float(eps), ptr(out), _stream())
    return out


def get_tpr(fprs, tprs):
    """TPR (in %) at the ROC point whose FPR is nearest each of 1e-5, 1e-4,
    1e-3 (utils/modules.py:40-47; the first such point on ties)."""
    fprs = np.asarray(fprs)
    tprs = np.asarray(tprs)
    return [float(tprs[int(np.argmin(np.abs(fprs - f)))] * 100) for f in FPR_TARGETS]


def calculate_scores(y_score, y_true, args=None, verbose=True):
    """ROC metrics of utils/modules.py:51-72.  Returns a dict with auc, eer,
    tpr@1e-5, tpr@1e-4, tpr@1e-3 (%) and score (their sum); prints the
    reference's line when verbose, and with ``args.is_roc`` saves
    (y_true, y_score) to ``args.roc_file + '.npy'`` as the reference does."""
    from sklearn import metrics
    y_score = np.asarray(y_score, dtype=np.float64)
    y_true = np.asarray(y_true)
    fprs, tprs, _ = metrics.roc_curve(y_true, y_score)
    fprs = np.flipud(fprs)
    tprs = np.flipud(tprs)
    eer = float(fprs[np.nanargmin(np.absolute((1 - tprs) - fprs))])
    auc = float(metrics.auc(fprs, tprs))
    tpr = get_tpr(fprs, tprs)
    res = {"auc": auc, "eer": eer, "tpr@1e-5": tpr[0], "tpr@1e-4": tpr[1], "tpr@1e-3": tpr[2],
           "score": tpr[0] + tpr[1] + tpr[2]}
    if verbose:
        print("AUC {:.4f} | EER {:.4f} | TPR@FPR=1e-5 {:.4f} | TPR@FPR=1e-4 {:.4f} | "
              "TPR@FPR=1e-3 {:.4f} | score {:.4f}".format(auc, eer, *tpr, res["score"]))
    if args is not None and getattr(args, "is_roc", False):
        with open(os.path.join(".", args.roc_file + ".npy"), "wb") as f:
            np.save(f, y_true)
            np.save(f, y_score)
    return res


def calculate_identification_acc(y_score, total_sub):
    """Rank-1 identification accuracy in % (utils/modules.py:76-88): the
    scores are ``total_sub`` consecutive groups of equal size, and subject i
    is identified when the maximum of group i sits at position i."""
    y_score = np.asarray(y_score)
    per = len(y_score) // total_sub
    best = y_score[:total_sub * per].reshape(total_sub, per).argmax(axis=1)
    return float((best == np.arange(total_sub)).sum() / total_sub * 100)


class Evaluator:
    """Accumulates pair scores and labels over the test loader's batches
    (utils/modules.py:95-168's loop) and computes the metrics once."""

    def __init__(self, eps=1e-6):
        self.eps = eps
        self.scores = []
        self.labels = []

    def add(self, out1, out2, pair_label):
        self.scores.append(pair_scores(out1, out2, self.eps))
        self.labels.append(torch.as_tensor(pair_label).reshape(-1))

    def result(self, args=None, total_sub=None, verbose=True):
        scores = torch.cat(self.scores).cpu().numpy()
        labels = torch.cat([lab.cpu() for lab in self.labels]).numpy()
        res = calculate_scores(scores, labels, args, verbose=verbose)
        if total_sub:
            res["ident_acc"] = calculate_identification_acc(scores, total_sub)
        return res
