"""Classification metrics (reference utils.py:585-663).

CPU: the oracle restatement reproduces the reference's own outputs (tests/golden/metrics_golden.npz,
made by tests/golden/gen_metrics_golden.py from the reference function) bit for bit, NaNs
included.  GPU: vitcnn_amd.metrics (device confusion counts via vc_confusion_matrix) reproduces
the same golden outputs and the oracle on a full Houston2013-size map (349 x 1905)."""
import numpy as np
import pytest
import torch

from helpers import load_npz
from oracle import metrics_oracle as MO

KEYS = (("cm", "Confusion matrix"), ("acc", "Accuracy"), ("f1", "F1 scores"), ("prec", "Precisions"),
        ("aa", "AA"), ("kappa", "Kappa"))


def _cases():
    g = load_npz("metrics_golden.npz")
    for i in range(int(g["n_cases"])):
        ncls = int(g[f"ncls_{i}"])
        yield (g[f"pred_{i}"], g[f"tgt_{i}"], [int(v) for v in g[f"ign_{i}"]], None if ncls < 0 else ncls,
               {k: g[f"{k}_{i}"] for k, _ in KEYS})


def _check(res, exp):
    for k, name in KEYS:   # assert_array_equal treats NaN == NaN
        np.testing.assert_array_equal(np.asarray(res[name]), exp[k], err_msg=name)


def test_oracle_matches_reference_golden():
    n = 0
    for pred, tgt, ign, ncls, exp in _cases():
        _check(MO.metrics(pred, tgt, ign, ncls), exp)
        n += 1
    assert n == 5


def test_golden_covers_nan_classes():
    g = load_npz("metrics_golden.npz")
    assert np.isnan(g["f1_1"]).any() and np.isnan(g["prec_4"]).any() and not np.isnan(g["aa_1"])


@pytest.mark.gpu
def test_device_metrics_match_reference_golden():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vitcnn_amd.metrics import metrics
    for pred, tgt, ign, ncls, exp in _cases():
        _check(metrics(pred, tgt, ign, ncls), exp)


@pytest.mark.gpu
def test_device_confusion_full_image():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vitcnn_amd.metrics import confusion_matrix, metrics
    rng = np.random.default_rng(7)
    tgt = rng.integers(0, 16, size=(349, 1905))
    pred = np.where(rng.random(tgt.shape) < 0.8, tgt, rng.integers(0, 16, size=tgt.shape))
    exp = MO.metrics(pred, tgt, [0], 16)
    res = metrics(pred, tgt, [0], 16)
    for _, name in KEYS:
        np.testing.assert_array_equal(np.asarray(res[name]), np.asarray(exp[name]), err_msg=name)
    # device tensors in, nothing ignored, out-of-range predictions dropped
    t, p = torch.from_numpy(tgt).cuda(), torch.from_numpy(pred).cuda()
    p[0, :10] = 99
    cm = confusion_matrix(p, t, [], 16).cpu().numpy()
    np.testing.assert_array_equal(cm, MO.confusion_counts(p.cpu().numpy(), tgt, [], 16))
    assert cm.sum() == tgt.size - 10
