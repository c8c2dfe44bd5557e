"""Classification metrics of a whole-image prediction: the reference's `metrics`
(utils.py:585-663), which main.py:505 calls on the argmax of `test()`'s probabilities.

The counting step runs on the device: `vc_confusion_matrix` (metrics.hip) histograms the
(target, prediction) pairs of every non-ignored pixel into an n_classes x n_classes matrix, so a
full-image map never leaves HBM.  The per-class scores are then evaluated on that small matrix
with the reference's arithmetic (numpy float64; a class with no pixels gives NaN, as numpy
division does in the reference, and the average accuracy skips NaN recalls), so the returned
dict has the reference's keys and bit-identical values.
"""
from __future__ import annotations

import numpy as np
import torch

from ._lib import lib

MAX_CLASSES = 64


def _labels(a, device):
    return torch.as_tensor(a).to(device=device, dtype=torch.int64).contiguous().view(-1)


def confusion_matrix(prediction, target, ignored_labels=(), n_classes=None, device=None):
    """int64 [n_classes, n_classes] counts on the device (row = target label, column =
    prediction) over the pixels whose target is not ignored; pairs outside range(n_classes) are
    not counted (sklearn confusion_matrix(labels=range(n_classes)), utils.py:608-611)."""
    if device is None:
        device = prediction.device if torch.is_tensor(prediction) and prediction.is_cuda else torch.device("cuda")
    t, p = _labels(target, device), _labels(prediction, device)
    if t.numel() != p.numel():
        raise ValueError(f"prediction has {p.numel()} pixels, target {t.numel()}")
    ign = torch.as_tensor(list(ignored_labels), dtype=torch.int64).to(device)
    if n_classes is None:   # utils.py:605: max over the kept target labels
        kept = t[~torch.isin(t, ign)] if ign.numel() else t
        n_classes = int(kept.max().item()) + 1
    if not 0 < n_classes <= MAX_CLASSES:
        raise ValueError(f"n_classes must be in [1, {MAX_CLASSES}], got {n_classes}")
    table = torch.zeros(n_classes, dtype=torch.uint8, device=device)
    table[ign[(ign >= 0) & (ign < n_classes)]] = 1
    cm = torch.zeros(n_classes * n_classes, dtype=torch.int64, device=device)
    lib().vc_confusion_matrix(t.numel(), t.data_ptr(), p.data_ptr(), n_classes, table.data_ptr(), cm.data_ptr(),
                              torch.cuda.current_stream(device).cuda_stream)
    return cm.view(n_classes, n_classes)


def scores(cm) -> dict:
    """utils.py:613-661 on a confusion matrix: Accuracy (%), F1 scores, Precisions, AA, Kappa."""
    cm = np.asarray(cm, dtype=np.int64)
    diag = np.diagonal(cm)
    rows, cols = cm.sum(axis=1), cm.sum(axis=0)
    total = cm.sum()
    with np.errstate(divide="ignore", invalid="ignore"):
        recall = diag / rows
        pa = np.trace(cm) / float(total)
        pe = np.sum(cols * rows) / float(total * total)
        return {
            "Confusion matrix": cm,
            "Accuracy": diag.sum() * (100 / float(total)),
            "F1 scores": 2.0 * diag / (rows + cols),
            "Precisions": 1.0 * diag / rows,
            "AA": np.mean(recall[~np.isnan(recall)]),
            "Kappa": (pa - pe) / (1 - pe),
        }


def metrics(prediction, target, ignored_labels=[], n_classes=None):
    """Same signature and result dict as the reference's utils.metrics."""
    return scores(confusion_matrix(prediction, target, ignored_labels, n_classes).cpu().numpy())
