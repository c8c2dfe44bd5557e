"""Diagnostic: the NonLocal attention kernels (MFMA and legacy) on the live B=4 training workspace's
inputs (hsi1 / hsi2 theta, pooled phi|g, dO) vs a float64 evaluation of the same inputs."""
import os
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, "vit-cnn_amd"); sys.path.insert(0, ".")
import torch
import test_model_gpu as T
import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
from vitcnn_amd._lib import lib

b4 = T.b4._get_wrapped_function()()
m = b4["m"]
ws = next(w for k, w in m._ws.items() if k[2] == ("train", "grad"))
L = lib()
s = torch.cuda.current_stream().cuda_stream
B = 4
for pfx, Hs, Cout in (("hsi1", 7, 256), ("hsi2", 5, 144)):
    S, Pk = Hs * Hs, (Hs // 2) ** 2
    Ci = Cout // 2
    th = ws.tensor(pfx + ".TH")[: B * S * Ci].clone()
    pp = ws.tensor(pfx + ".PP")[: B * Pk * 2 * Ci].clone()
    do = ws.tensor(pfx + ".dO")[: B * S * Ci].clone()
    t64 = th.double().cpu().view(B, S, Ci).requires_grad_(True)
    p64 = pp.double().cpu().view(B, Pk, 2 * Ci).requires_grad_(True)
    sc = t64 @ p64[..., :Ci].transpose(1, 2)
    a64 = torch.softmax(sc, -1)
    o64 = a64 @ p64[..., Ci:]
    o64.backward(do.double().cpu().view(B, S, Ci))
    print(pfx, "scores range", float(sc.min()), float(sc.max()), "att max", float(a64.max()),
          "|dO| max", float(do.abs().max()), flush=True)
    for mode in ("0", "1"):
        os.environ["VITCNN_NL_LEGACY"] = mode
        att = torch.empty(B * S * Pk, device="cuda")
        o = torch.empty(B * S * Ci, device="cuda")
        dth = torch.empty(B * S * Ci, device="cuda")
        dpp = torch.empty(B * Pk * 2 * Ci, device="cuda")
        L.vc_nonlocal_attn_fwd(B, S, Pk, Ci, th.data_ptr(), pp.data_ptr(), att.data_ptr(), o.data_ptr(), s)
        L.vc_nonlocal_attn_bwd(B, S, Pk, Ci, th.data_ptr(), pp.data_ptr(), att.data_ptr(), do.data_ptr(),
                               dth.data_ptr(), dpp.data_ptr(), s)
        torch.cuda.synchronize()

        def e(a, r):
            a = a.cpu().double().view(r.shape)
            return float((a - r).abs().max() / r.abs().max())
        print("  ", "legacy" if mode == "1" else "mfma  ", "att %.2e o %.2e dtheta %.2e dphi %.2e dg %.2e" % (
            e(att, a64.detach()), e(o, o64.detach()), e(dth, t64.grad),
            e(dpp.view(B, Pk, 2 * Ci)[..., :Ci], p64.grad[..., :Ci]),
            e(dpp.view(B, Pk, 2 * Ci)[..., Ci:], p64.grad[..., Ci:])), flush=True)
