"""GPU tool: fp32 GEMM accuracy vs float64 for long-K shapes (legacy kernel vs the current one, several
split counts): max |C - C64| / max(sum_k |a b|) per configuration.  usage: python tools/gemm_err.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))
import torch  # noqa: E402

import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
knobs.use_probe()   # vc_gemm_tune: the probe library
from vitcnn_amd._lib import lib  # noqa: E402


def main():
    L = lib()
    dev = torch.device("cuda", 0)
    ws = torch.empty(1 << 25, device=dev)
    for (ta, tb, M, N, K) in [(0, 1, 484, 1024, 9216), (1, 0, 1024, 9216, 484), (0, 0, 484, 9216, 1024),
                              (0, 1, 3136, 256, 1296)]:
        g = torch.Generator().manual_seed(1)
        A = torch.randn((K, M) if ta else (M, K), generator=g)
        B = torch.randn((N, K) if tb else (K, N), generator=g)
        Ao, Bo = (A.t() if ta else A).double(), (B.t() if tb else B).double()
        ref = Ao @ Bo
        mag = (Ao.abs() @ Bo.abs()).max().item()
        cpu32 = ((A.t() if ta else A) @ (B.t() if tb else B)).double()
        print(f"ta={ta} tb={tb} M={M} N={N} K={K}: cpu fp32 err {float((cpu32 - ref).abs().max()) / mag:.2e}")
        Ad, Bd = A.to(dev), B.to(dev)
        for flags, ns in [(4, 0), (0, 1), (0, 0), (0, 8), (0, 32)]:
            L.vc_gemm_tune(0, 0, ns, 0, -1)
            C = torch.empty(M, N, device=dev)
            L.vc_gemm(ta, tb, M, N, K, 1.0, Ad.data_ptr(), M if ta else K, 0, Bd.data_ptr(), K if tb else N, 0, 0.0,
                      C.data_ptr(), N, 0, 1, None, None, 0, 0, flags, None, ws.data_ptr(), ws.numel(),
                      torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            err = float((C.cpu().double() - ref).abs().max()) / mag
            print(f"   {'legacy' if flags == 4 else 'v2'} nsplit={ns or 'auto'}: {err:.2e}")
        L.vc_gemm_tune(0, 0, 0, 0, -1)


if __name__ == "__main__":
    main()
