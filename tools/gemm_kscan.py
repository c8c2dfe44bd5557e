"""GPU tool: fixed vs per-k-step cost of the GEMM kernels.  Times C[M,N] = A[M,K] W[N,K]^T (no split-K)
for growing K with each kernel family (legacy fp32 k-major, v2 fp32, v2 bf16), back-to-back launches on
one stream, HIP events.  (Measured: ~3 us fixed + ~1 us per 32 of K at one wave per SIMD, fp32.)
usage: python tools/gemm_kscan.py [M] [N]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))
import torch  # noqa: E402

import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
from vitcnn_amd._lib import lib  # noqa: E402


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 3136
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    L = lib()
    raw = L.raw["vc_gemm_ex"]
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    Kmax = 2048
    A = torch.rand(M, Kmax, device=dev)
    W = torch.rand(N, Kmax, device=dev)
    C = torch.empty(M, N, device=dev)
    fill = torch.empty(256, device=dev)

    def t_us(fn, reps=50):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            fn()
        e1.record(st)
        e1.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3

    print(f"fill 256 floats: {t_us(lambda: L.vc_fill(256, fill.data_ptr(), 1.0, st.cuda_stream)):.2f} us")
    fams = [("legacy", 4), ("v2f32", 8), ("v2bf16", 2)]
    print(f"M={M} N={N}: us per launch (no split-K)")
    print("    K " + " ".join(f"{n:>8s}" for n, _ in fams))
    for K in (16, 32, 64, 128, 256, 512, 1024, 2048):
        row = []
        for _, fl in fams:
            def fn(K=K, fl=fl):
                raw(0, 1, M, N, K, 1.0, A.data_ptr(), Kmax, 0, W.data_ptr(), Kmax, 0, 0.0, C.data_ptr(), N, 0, 1,
                    None, None, 0, 0, fl, None, None, 0, None, 0, st.cuda_stream)
            row.append(t_us(fn))
        print(f"{K:5d} " + " ".join(f"{v:8.2f}" for v in row))


if __name__ == "__main__":
    main()
