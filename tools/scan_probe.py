"""GPU probe: the selective-scan kernels of both hsiMamba blocks re-launched on the live workspace
of one training step and timed with HIP events (us per launch).  usage: scan_probe.py [reps]"""
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


def timed(fn, reps, stream):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(stream)
    for _ in range(reps):
        fn()
    e.record(stream)
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
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
    f = prog.ws.f
    P = prog.P
    outs = torch.empty(1 << 16, device=dev)
    for blk, pfx, H in ((m.hsi1, "hsi1", m.patch), (m.hsi2, "hsi2", m.patch - 2)):
        E = blk.embed
        D, R, Lt = E // 2, math.ceil(E / 16), H * H
        XW = R + 32
        rows, nr = B * Lt, NDIR * B * Lt
        mx, gv = pfx + ".global_view.layers.0", pfx + ".global_view"
        order = prog.tab[("order", H)].data_ptr()
        o = outs.data_ptr()
        ckp = f(pfx + ".CKP", L.vc_mamba_scan_ckpt_floats(B, Lt, D, NDIR))

        def fwd():
            L.vc_mamba_scan_fwd(B, Lt, D, R, NDIR, f(pfx + ".U", nr * D), f(pfx + ".XD", nr * XW), order,
                                P[mx + ".dt_proj.weight"], P[mx + ".dt_proj.bias"], P[mx + ".A_log"], P[mx + ".D"],
                                f(pfx + ".Y", nr * D), ckp, st.cuda_stream)

        def bwd():
            L.vc_mamba_scan_bwd(B, Lt, D, R, NDIR, f(pfx + ".U", nr * D), f(pfx + ".XD", nr * XW), order,
                                P[mx + ".dt_proj.weight"], P[mx + ".dt_proj.bias"], P[mx + ".A_log"], P[mx + ".D"],
                                P[gv + ".weights"], f(pfx + ".Y", nr * D), f(pfx + ".dYP", rows * D),
                                ckp,
                                f(pfx + ".dU", nr * D), f(pfx + ".dDTL", nr * D), f(pfx + ".dXD", nr * XW),
                                o, o + 4 * D * 16, o + 4 * (D * 16 + D), prog.scr_p, prog.scr_n, st.cuda_stream)

        print(f"{pfx}: scan_fwd {timed(fwd, reps, st):7.1f} us   scan_bwd(+reductions) {timed(bwd, reps, st):7.1f} us",
              flush=True)
        # grid scaling of the backward kernel alone (sequences = 10 x b; buffers sized for B = 64):
        # flat time over b = a per-block latency chain, linear = throughput-bound
        for b in (64, 32, 16, 8, 4, 1):
            def bwd_b(b=b):
                L.vc_mamba_scan_bwd(b, Lt, D, R, NDIR, f(pfx + ".U", nr * D), f(pfx + ".XD", nr * XW), order,
                                    P[mx + ".dt_proj.weight"], P[mx + ".dt_proj.bias"], P[mx + ".A_log"],
                                    P[mx + ".D"], P[gv + ".weights"], f(pfx + ".Y", nr * D), f(pfx + ".dYP", rows * D),
                                    ckp, f(pfx + ".dU", nr * D), f(pfx + ".dDTL", nr * D), f(pfx + ".dXD", nr * XW),
                                    None, None, None, prog.scr_p, prog.scr_n, st.cuda_stream)
            print(f"    scan_bwd kernel, {NDIR * b:4d} sequences: {timed(bwd_b, reps, st):7.1f} us", flush=True)
        # the select-based dB / dC reduce-scatter (A/B against the bank-masked default)
        os.environ["VITCNN_SCAN_SELECT_RS"] = "1"
        print(f"    scan_bwd kernel, select reduce-scatter: {timed(lambda: bwd_b(64), reps, st):7.1f} us",
              flush=True)
        del os.environ["VITCNN_SCAN_SELECT_RS"]
        # the dB / dC partial combine after every segment (A/B against every second segment, the default)
        os.environ["VITCNN_SCAN_RBS"] = "1"
        print(f"    scan_bwd kernel, combine every segment: {timed(lambda: bwd_b(64), reps, st):7.1f} us", flush=True)
        del os.environ["VITCNN_SCAN_RBS"]


if __name__ == "__main__":
    main()
