"""Golden vectors for the classification metrics: the reference's
own utils.metrics (utils.py:585-663) executed in this container on seeded synthetic
prediction / target maps.  utils.py's plotting, visdom and hyperspectral-IO imports are not used
by metrics() and are absent here, so those modules are stubbed before utils.py is loaded by path.
Writes metrics_golden.npz (inputs and outputs only).
usage: python tests/golden/gen_metrics_golden.py [REFERENCE_ROOT]"""
import importlib
import importlib.util
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def _stub(name):
    m = types.ModuleType(name)
    sys.modules[name] = m
    return m


def load_reference_utils(ref):
    for name in ("seaborn", "spectral", "visdom"):
        try:
            importlib.import_module(name)
        except ImportError:
            _stub(name)
    spec = importlib.util.spec_from_file_location("reference_utils", os.path.join(ref, "utils.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def cases():
    rng = np.random.default_rng(2024)
    out = []
    # Houston2013 label set (15 classes + ignored 0), ~80 % correct
    t = rng.integers(0, 16, size=(40, 50))
    p = np.where(rng.random(t.shape) < 0.8, t, rng.integers(1, 16, size=t.shape))
    out.append((p, t, [0], 16))
    # MUUFL label set (11 + 0); classes 5 and 9 absent from target and prediction -> NaN F1 /
    # precision, skipped by AA
    t = rng.integers(0, 12, size=(30, 30))
    t[(t == 5) | (t == 9)] = 1
    p = np.where(rng.random(t.shape) < 0.7, t, rng.integers(1, 12, size=t.shape))
    p[(p == 5) | (p == 9)] = 2
    out.append((p, t, [0], 12))
    # n_classes inferred from the target, nothing ignored
    t = rng.integers(0, 7, size=(25, 20))
    p = np.where(rng.random(t.shape) < 0.6, t, rng.integers(0, 7, size=t.shape))
    out.append((p, t, [], None))
    # two ignored labels; predictions may land on ignored classes
    t = rng.integers(0, 10, size=(33, 17))
    p = rng.integers(0, 10, size=t.shape)
    out.append((p, t, [0, 3], 10))
    # a class predicted but never in the target (row of zeros, non-zero column), class 7 absent
    t = rng.integers(1, 6, size=(16, 16))
    p = t.copy()
    p[::3, ::2] = 6
    out.append((p, t, [0], 8))
    return out


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    U = load_reference_utils(ref)
    arrays = {}
    cs = cases()
    for i, (p, t, ign, ncls) in enumerate(cs):
        with np.errstate(divide="ignore", invalid="ignore"):
            r = U.metrics(p, t, ignored_labels=ign, n_classes=ncls)
        arrays.update({
            f"pred_{i}": p.astype(np.int64), f"tgt_{i}": t.astype(np.int64),
            f"ign_{i}": np.asarray(ign, dtype=np.int64), f"ncls_{i}": np.int64(-1 if ncls is None else ncls),
            f"cm_{i}": np.asarray(r["Confusion matrix"], dtype=np.int64),
            f"acc_{i}": np.float64(r["Accuracy"]),
            f"f1_{i}": np.asarray(r["F1 scores"], dtype=np.float64),
            f"prec_{i}": np.asarray(r["Precisions"], dtype=np.float64),
            f"aa_{i}": np.float64(r["AA"]), f"kappa_{i}": np.float64(r["Kappa"]),
        })
    arrays["n_cases"] = np.int64(len(cs))
    np.savez_compressed(os.path.join(HERE, "metrics_golden.npz"), **arrays)
    print("wrote", len(cs), "cases")


if __name__ == "__main__":
    main()
