"""GPU probe: the TokenLearner kernels (vc_tl_pixel_stats, vc_tl_fwd, vc_tl_bwd) of hsi1's channel token (B = 64,
HW = 81, C = 256, S = 49) and hsi2's (B = 64, HW = 49, C = 144, S = 25) timed alone with HIP events (us per call).
usage: python tools/tl_probe.py [reps]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))
import torch  # noqa: E402

import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
from vitcnn_amd._lib import lib  # noqa: E402


def timed(fn, reps):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda", 0)
    L = lib()
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device=dev).manual_seed(0)
    for name, B, HW, C, S in (("hsi1", 64, 81, 256, 49), ("hsi2", 64, 49, 144, 25)):
        M = B * HW
        x = torch.randn(M, C, device=dev, generator=g)
        mx, avg = torch.empty(M, device=dev), torch.empty(M, device=dev)
        amx = torch.empty(M, dtype=torch.int32, device=dev)
        ws = torch.empty((L.vc_tl_ws_floats(B, HW, S) + 1) // 2, dtype=torch.float64, device=dev)
        par = torch.randn(S * 5, device=dev, generator=g) * 0.5
        buf = torch.ones(S * 2, device=dev)
        stats = torch.empty(2 * S + 8, dtype=torch.float64, device=dev)
        Z = torch.empty(B * S * C, device=dev)
        dZ = torch.randn(B * S * C, device=dev, generator=g)
        amap = torch.empty(B * S * HW, device=dev)
        dx = torch.empty(M, C, device=dev)
        dpar = torch.empty(S * 5, device=dev)

        def pix():
            L.vc_tl_pixel_stats(M, C, x.data_ptr(), C, mx.data_ptr(), amx.data_ptr(), avg.data_ptr(), ws.data_ptr(), st)

        def fwd():
            L.vc_tl_fwd(1, B, HW, C, S, x.data_ptr(), C, mx.data_ptr(), avg.data_ptr(), par.data_ptr(), buf.data_ptr(),
                        1e-5, 0.1, ws.data_ptr(), stats.data_ptr(), amap.data_ptr(), Z.data_ptr(), st)

        def bwd():
            L.vc_tl_bwd(1, B, HW, C, S, x.data_ptr(), C, mx.data_ptr(), avg.data_ptr(), amx.data_ptr(), par.data_ptr(),
                        stats.data_ptr(), amap.data_ptr(), dZ.data_ptr(), ws.data_ptr(), dx.data_ptr(), C,
                        dpar.data_ptr(), st)

        pix()
        fwd()
        print(f"{name}: pixel_stats {timed(pix, reps):6.1f} us  tl_fwd {timed(fwd, reps):6.1f} us  "
              f"tl_bwd (da + dx) {timed(bwd, reps):6.1f} us", flush=True)


if __name__ == "__main__":
    main()
