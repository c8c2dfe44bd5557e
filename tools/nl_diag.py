"""Diagnostic: the B=4 gradient comparison of tests/test_model_gpu.py (worst tensors relative to their
scale vs the float64 yardstick) with the MFMA NonLocal kernels and with the legacy ones (VITCNN_NL_LEGACY)."""
import os, sys, json
sys.path.insert(0, "tests"); sys.path.insert(0, "vit-cnn_amd"); sys.path.insert(0, ".")
import torch
import test_model_gpu as T
res = {}
for mode in ("0", "1"):
    os.environ["VITCNN_NL_LEGACY"] = mode
    b4 = T.b4._get_wrapped_function()()
    m, ref, ref64, ref64_own = b4["m"], b4["ref_grads"], b4["ref64"], b4["ref64_own"]
    flat = m.flat_params.grad.detach().cpu()
    named = dict(m.named_parameters())
    gmax = max(float(g.abs().max()) for g in ref64.values() if g is not None)
    floor = 1e-5 * gmax
    rows = []
    for n, off in m._poff.items():
        p = named[n]
        got = flat[off:off + p.numel()].view(p.shape).double()
        r64 = ref64.get(n)
        if r64 is None:
            continue
        err = float((got - r64).abs().max()); scale = float(r64.abs().max())
        err32 = float((ref[n].double() - ref64_own[n]).abs().max())
        # the test's criterion: err <= 1e-3 scale + floor  or  err <= 3 err32 + floor
        ratio = err / max(1e-3 * scale + floor, 3.0 * err32 + floor)
        rows.append((ratio, n, err, err32, scale))
    rows.sort(reverse=True)
    print("LEGACY" if mode == "1" else "MFMA", "failing:", sum(r[0] > 1 for r in rows), flush=True)
    for r in rows[:15]:
        print("  %.3f %s err=%.3e err32=%.3e scale=%.3e" % r, flush=True)
