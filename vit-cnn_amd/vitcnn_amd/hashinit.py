"""Counter-hash deterministic fills for parameters and synthetic inputs.

Every value is a pure function of (tensor name, flat element index), computed
with splitmix64 in numpy uint64 arithmetic.  The same numbers come out on any
host, any device and any rank, without relying on a framework RNG stream, so
golden fixtures generated in one container reproduce bit-for-bit on the GPU box
(SURVEY.md section 7, step 0).

Fill rules (chosen so every parameter is non-zero and every gradient path is
exercised):
  * conv / linear weights (ndim >= 2): U(-1, 1) / sqrt(fan_in)
  * ``A_log``: log(1..N) + 0.1 U(-1, 1)       (S4D-real init, perturbed)
  * mixer ``D``: 1 + 0.2 U(-1, 1)
  * ``dt_proj.bias``: softplus^-1 of a log-uniform dt in [1e-3, 1e-1]
  * ``pos_embed``: 0.02 U(-1, 1)
  * direction gate ``weights``: U(-1, 1)
  * other 1-D ``weight`` (BatchNorm / LayerNorm gamma): 0.75 + 0.5 U
  * other 1-D ``bias``: 0.1 U(-1, 1)
"""
from __future__ import annotations

import math

import numpy as np

_M64 = (1 << 64) - 1


def _fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for ch in s.encode("utf-8"):
        h ^= ch
        h = (h * 0x100000001B3) & _M64
    return h


def hash_u01(name: str, n: int) -> np.ndarray:
    """n uniform floats in [0, 1) (24-bit resolution, exact in fp32), keyed by name."""
    seed = np.uint64(_fnv1a64(name))
    with np.errstate(over="ignore"):
        z = seed + (np.arange(n, dtype=np.uint64) + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(40)).astype(np.float64) / float(1 << 24)


def param_fill(name: str, shape) -> np.ndarray:
    """Deterministic fp32 value for a named parameter of the given shape."""
    shape = tuple(int(s) for s in shape)
    n = int(np.prod(shape)) if shape else 1
    u = hash_u01(name, n)
    s = 2.0 * u - 1.0
    leaf = name.rsplit(".", 1)[-1]
    if leaf == "A_log":
        nstate = shape[-1]
        base = np.log(np.tile(np.arange(1, nstate + 1, dtype=np.float64), n // nstate))
        v = base + 0.1 * s
    elif leaf == "D" and len(shape) == 1:
        v = 1.0 + 0.2 * s
    elif name.endswith("dt_proj.bias"):
        dt = np.exp(u * (math.log(1e-1) - math.log(1e-3)) + math.log(1e-3))
        v = dt + np.log(-np.expm1(-dt))
    elif leaf == "pos_embed":
        v = 0.02 * s
    elif leaf == "weights":
        v = s
    elif len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        v = s / math.sqrt(fan_in)
    elif leaf == "weight":
        v = 0.75 + 0.5 * u
    else:
        v = 0.1 * s
    return v.astype(np.float32).reshape(shape)


def fill_module_(module, skip_buffers: bool = True) -> None:
    """Overwrite every parameter of a torch module in place with param_fill."""
    import torch

    with torch.no_grad():
        for name, p in module.named_parameters():
            p.copy_(torch.from_numpy(param_fill(name, p.shape)).to(p.device))


def synthetic_batch(tag: str, batch: int, c1: int, c2: int, patch: int, n_classes: int):
    """Deterministic (hsi, lidar, target) numpy batch.

    hsi ~ U[0,1) [B,C1,P,P] and lidar ~ U[0,1) [B,C2,P,P] (the reference
    min-max normalises every band to [0,1], datasets.py:125-133); labels are
    uniform in [1, n_classes-1] (class 0 is the ignored 'Unclassified' label,
    datasets.py:489-492).
    """
    hsi = hash_u01(f"{tag}.hsi", batch * c1 * patch * patch).astype(np.float32)
    lidar = hash_u01(f"{tag}.lidar", batch * c2 * patch * patch).astype(np.float32)
    lab = hash_u01(f"{tag}.target", batch)
    target = 1 + np.floor(lab * (n_classes - 1)).astype(np.int64)
    return (hsi.reshape(batch, c1, patch, patch), lidar.reshape(batch, c2, patch, patch), target)
