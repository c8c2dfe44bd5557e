"""Shared test helpers: hash-filled state dicts keyed by the reference's 1704 state_dict names."""
import json
import os

import numpy as np
import torch

from vitcnn_amd.hashinit import param_fill, synthetic_batch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def reference_keys():
    with open(os.path.join(GOLDEN, "state_dict_keys.json")) as f:
        return json.load(f)


def is_buffer(name):
    return name.endswith("running_mean") or name.endswith("running_var") or name.endswith("num_batches_tracked")


def hash_state_dict():
    """state_dict with every parameter from param_fill and BN buffers at their torch defaults."""
    sd = {}
    for e in reference_keys():
        n, shape = e["name"], tuple(e["shape"])
        if n.endswith("running_mean"):
            sd[n] = torch.zeros(shape)
        elif n.endswith("running_var"):
            sd[n] = torch.ones(shape)
        elif n.endswith("num_batches_tracked"):
            sd[n] = torch.zeros(shape, dtype=torch.int64)
        else:
            sd[n] = torch.from_numpy(param_fill(n, shape))
    return sd


def golden_batch(tag, batch):
    hsi, lidar, target = synthetic_batch(tag, batch, 144, 1, 9, 16)
    return torch.from_numpy(hsi), torch.from_numpy(lidar), torch.from_numpy(target)


def load_npz(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))
