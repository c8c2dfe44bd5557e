"""CPU restatement of the reference's classification metrics — TEST INFRASTRUCTURE ONLY.

The checker for vitcnn_amd.metrics; imported by tests/ and nothing
else.  Restates utils.py:585-663 `metrics(prediction, target, ignored_labels, n_classes)`:
  * utils.py:596-601  pixels whose target is an ignored label are dropped;
  * utils.py:605      n_classes defaults to max(target) + 1 over the kept pixels;
  * utils.py:608-611  sklearn confusion_matrix(target, prediction, labels=range(n_classes)):
                      rows = target, columns = prediction, pairs outside the label set not counted;
  * utils.py:615-661  accuracy (percent), per-class F1 and "precision" (the row-normalised
                      diagonal), average accuracy over the classes whose recall is defined,
                      Cohen's kappa.
The arithmetic is numpy's, as in the reference: a class without pixels divides 0 by 0 and yields
NaN (the reference's ZeroDivisionError branches never fire for numpy scalars).
Pinned by tests/golden/metrics_golden.npz: the reference function itself run on seeded maps
(tests/golden/gen_metrics_golden.py).
"""
import numpy as np


def confusion_counts(prediction, target, ignored_labels=(), n_classes=None):
    t = np.asarray(target, dtype=np.int64).reshape(-1)
    p = np.asarray(prediction, dtype=np.int64).reshape(-1)
    keep = np.ones(t.shape, dtype=bool)
    for lab in ignored_labels:
        keep &= t != lab
    t, p = t[keep], p[keep]
    if n_classes is None:
        n_classes = int(t.max()) + 1
    ok = (t >= 0) & (t < n_classes) & (p >= 0) & (p < n_classes)
    cm = np.zeros((n_classes, n_classes), dtype=np.int64)
    np.add.at(cm, (t[ok], p[ok]), 1)
    return cm


def scores(cm):
    cm = np.asarray(cm, dtype=np.int64)
    n = cm.shape[0]
    total = cm.sum()
    correct = 0
    for i in range(n):
        correct += cm[i, i]
    res = {"Confusion matrix": cm, "Accuracy": correct * (100 / float(total))}
    f1, prec, recalls = np.zeros(n), np.zeros(n), []
    with np.errstate(divide="ignore", invalid="ignore"):
        for i in range(n):
            row, col = cm[i, :].sum(), cm[:, i].sum()
            f1[i] = 2.0 * cm[i, i] / (row + col)
            prec[i] = 1.0 * cm[i, i] / row
            r = cm[i, i] / row
            if not np.isnan(r):
                recalls.append(r)
        res["F1 scores"] = f1
        res["Precisions"] = prec
        res["AA"] = np.mean(recalls)
        pa = np.trace(cm) / float(total)
        pe = np.sum(cm.sum(axis=0) * cm.sum(axis=1)) / float(total * total)
        res["Kappa"] = (pa - pe) / (1 - pe)
    return res


def metrics(prediction, target, ignored_labels=(), n_classes=None):
    return scores(confusion_counts(prediction, target, ignored_labels, n_classes))
