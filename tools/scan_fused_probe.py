"""GPU probe: the Mamba mixer's per-block launch chains, fused (vc_mamba_scan_fwd_fused / _bwd_fused) vs
separate (dirconv + x_proj GEMM + scan; scan backward + dt_proj / x_proj data-gradient GEMMs + conv
backward), re-launched alone on the live workspace of one training step and timed with HIP events
(us per chain, median of rounds).  usage: scan_fused_probe.py [reps]"""
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))
import torch  # noqa: E402

import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
from vitcnn_amd import CrossEntropyLoss, Multimodality_Mamba, fused_train_step  # noqa: E402
from vitcnn_amd._lib import lib  # noqa: E402
from vitcnn_amd.model import NDIR, _Program  # noqa: E402


def timed(fn, reps, stream, rounds=5):
    for _ in range(3):
        fn()
    out = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        for _ in range(reps):
            fn()
        e.record(stream)
        e.synchronize()
        out.append(s.elapsed_time(e) / reps * 1e3)
    return sorted(out)[len(out) // 2]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    dev = torch.device("cuda", 0)
    B = 64
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16).to(dev).train()
    crit = CrossEntropyLoss(weight=torch.ones(16, device=dev))
    hsi, lidar = torch.rand(B, 144, 9, 9, device=dev), torch.rand(B, 1, 9, 9, device=dev)
    tgt = torch.randint(1, 16, (B,), device=dev)
    fused_train_step(m, crit, hsi, lidar, tgt)
    torch.cuda.synchronize()
    prog = _Program(m, dev, B, True, "grad")
    L = lib()
    st = torch.cuda.current_stream(dev)
    s = st.cuda_stream
    f = prog.ws.f
    P = prog.P
    G = torch.empty(m._n_params, device=dev)
    g0 = G.data_ptr()
    Gp = {n: g0 + 4 * o for n, o in m._poff.items()}
    ws = torch.empty(1 << 24, device=dev)
    wsp, wsn = ws.data_ptr(), ws.numel()
    for blk, pfx, H in ((m.hsi1, "hsi1", m.patch), (m.hsi2, "hsi2", m.patch - 2)):
        E = blk.embed
        D, R, Lt = E // 2, math.ceil(E / 16), H * H
        XW = R + 32
        rows, nr = B * Lt, NDIR * B * Lt
        mx, gv = pfx + ".global_view.layers.0", pfx + ".global_view"
        order, inv = prog.tab[("order", H)].data_ptr(), prog.tab[("inv", H)].data_ptr()
        U, XD, Y, XZ = f(pfx + ".U", nr * D), f(pfx + ".XD", nr * XW), f(pfx + ".Y", nr * D), f(pfx + ".XZ",
                                                                                             rows * 2 * D)
        CP, CKP = f(pfx + ".convpart", NDIR * B * 5 * D), f(pfx + ".CKP", L.vc_mamba_scan_ckpt_floats(B, Lt, D, NDIR))
        dYP, dU, dDTL = f(pfx + ".dYP", rows * D), f(pfx + ".dU", nr * D), f(pfx + ".dDTL", nr * D)
        dXD, dXZ = f(pfx + ".dXD", nr * XW), f(pfx + ".dXZ", rows * 2 * D)
        cw, cb, wx = P[mx + ".conv1d.weight"], P[mx + ".conv1d.bias"], P[mx + ".x_proj.weight"]
        wdt, bdt, alog, dsk, gl = (P[mx + ".dt_proj.weight"], P[mx + ".dt_proj.bias"], P[mx + ".A_log"],
                                   P[mx + ".D"], P[gv + ".weights"])

        def fwd_sep():
            L.vc_mamba_dirconv_fwd(B, Lt, D, NDIR, order, XZ, cw, cb, U, s)
            L.vc_gemm(0, 1, nr, XW, D, 1.0, U, D, 0, wx, D, 0, 0.0, XD, XW, 0, 1, None, None, 0, 0, 0, None, wsp, wsn,
                      s)
            L.vc_mamba_scan_fwd(B, Lt, D, R, NDIR, U, XD, order, wdt, bdt, alog, dsk, Y, CKP, s)

        def fwd_fused():
            L.vc_mamba_scan_fwd_fused(B, Lt, D, R, NDIR, XZ, order, cw, cb, wx, wdt, bdt, alog, dsk, U, XD, Y, CKP,
                                      s)

        def scan_bwd():
            L.vc_mamba_scan_bwd(B, Lt, D, R, NDIR, U, XD, order, wdt, bdt, alog, dsk, gl, Y, dYP, CKP, dU, dDTL, dXD,
                                None, None, None, wsp, wsn, s)

        def bwd_sep():
            scan_bwd()
            L.vc_gemm(0, 0, nr, R, D, 1.0, dDTL, D, 0, wdt, R, 0, 0.0, dXD, XW, 0, 1, None, None, 0, 0, 0, None, wsp,
                      wsn, s)
            L.vc_gemm(0, 0, nr, D, XW, 1.0, dXD, XW, 0, wx, D, 0, 1.0, dU, D, 0, 1, None, None, 0, 0, 0, None, wsp,
                      wsn, s)
            L.vc_mamba_dirconv_bwd(B, Lt, D, NDIR, order, inv, XZ, cw, cb, dU, dXZ, Gp[mx + ".conv1d.weight"],
                                   Gp[mx + ".conv1d.bias"], wsp, wsn, s)

        def scan_bwd_fused():
            L.vc_mamba_scan_bwd_fused(B, Lt, D, R, NDIR, U, XD, order, XZ, cw, cb, wx, wdt, bdt, alog, dsk, gl, Y, dYP,
                                      CKP, dU, dDTL, dXD, CP, None, None, None, wsp, wsn, s)

        def tail_mask(mask):   # measurement only: parts of the tail skipped (VITCNN_SCAN_TAIL bits)
            def fn():
                os.environ["VITCNN_SCAN_TAIL"] = str(mask)
                try:
                    scan_bwd_fused()
                finally:
                    del os.environ["VITCNN_SCAN_TAIL"]
            return fn

        def bwd_fused():
            scan_bwd_fused()
            L.vc_mamba_dirconv_bwd_gather(B, Lt, D, NDIR, inv, cw, dU, dXZ, s)

        def conv_wgrad():
            L.vc_mamba_conv_params(B, D, NDIR, CP, Gp[mx + ".conv1d.weight"], Gp[mx + ".conv1d.bias"], s)

        res = {}
        for nm, fn in (("fwd_separate", fwd_sep), ("fwd_fused", fwd_fused), ("scan_bwd", scan_bwd),
                       ("bwd_separate", bwd_sep), ("scan_bwd_fused", scan_bwd_fused),
                       ("tail_none", tail_mask(0)), ("tail_staging_only", tail_mask(1)),
                       ("tail_a", tail_mask(3)), ("tail_bc", tail_mask(5)), ("bwd_fused", bwd_fused),
                       ("conv_params (off path)", conv_wgrad)):
            res[nm] = timed(fn, reps, st)
        print(pfx, "  ".join(f"{k} {v:.1f}" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
