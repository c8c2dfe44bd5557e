"""Diagnostic: tests/test_model_gpu.py::test_gradients_vs_reference_golden_b4's outcome with each mix of
the MFMA / legacy NonLocal forward and backward kernels (VITCNN_NL_LEGACY bit 0 forward, bit 1 backward)."""
import os
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, "vit-cnn_amd"); sys.path.insert(0, ".")
import torch
import test_model_gpu as T
from helpers import load_npz

g = load_npz("vitcnn_b4.npz")
keys = [k[5:] for k in g.files if k.startswith("grad/")]
for mode in ("0", "1", "2", "3"):
    os.environ["VITCNN_NL_LEGACY"] = mode
    b4 = T.b4._get_wrapped_function()()
    m, exact = b4["m"], b4["ref64_own"]
    flat = m.flat_params.grad.detach().cpu()
    named = dict(m.named_parameters())
    gmax = max(float(abs(g["grad/" + k]).max()) for k in keys)
    floor = 1e-5 * gmax
    direct, worst = 0, []
    for k in keys:
        ref = torch.from_numpy(g["grad/" + k]).double()
        off = m._poff[k]
        got = flat[off:off + named[k].numel()].view(named[k].shape).double()
        err = float((got - ref).abs().max())
        if err <= 1e-3 * float(ref.abs().max()) + floor:
            direct += 1
            continue
        ex = exact[k].double()
        r = float((got - ex).abs().max()) / (3.0 * float((ref - ex).abs().max()) + floor)
        worst.append((r, k))
    worst.sort(reverse=True)
    print(f"fwd {'legacy' if int(mode) & 1 else 'mfma'} bwd {'legacy' if int(mode) & 2 else 'mfma'}: direct {direct}, "
          f"failed {sum(w[0] > 1 for w in worst)}, worst {[(round(a, 2), b) for a, b in worst[:4]]}", flush=True)
