"""GPU tool: one vc_gemm_ex shape, repeated, for kernel-level profiling (rocprofv3 --pmc / --stats).
usage: [VITCNN_TUNE=bm,bn,nsplit] python tools/gemm_one.py TA TB M N K [flags] [reps] [bias_grad]
Prints the average time per call (HIP events) and TFLOP/s."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))
import torch  # noqa: E402

import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
from vitcnn_amd._lib import lib  # noqa: E402


def main():
    ta, tb, M, N, K = (int(v) for v in sys.argv[1:6])
    flags = int(sys.argv[6]) if len(sys.argv) > 6 else 0
    reps = int(sys.argv[7]) if len(sys.argv) > 7 else 200
    bgrad = len(sys.argv) > 8 and sys.argv[8] == "1"
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    A = torch.rand((K, M) if ta else (M, K), device=dev, generator=g) * 2 - 1
    B = torch.rand((N, K) if tb else (K, N), device=dev, generator=g) * 2 - 1
    C = torch.empty(M, N, device=dev)
    bg = torch.empty(M, device=dev) if bgrad else None
    ws = torch.empty(1 << 24, device=dev)
    cnt = torch.zeros(1 << 16, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    L = lib()
    args = (ta, tb, M, N, K, 1.0, A.data_ptr(), M if ta else K, 0, B.data_ptr(), K if tb else N, 0, 0.0,
            C.data_ptr(), N, 0, 1, None, None, 0, 0, flags, bg.data_ptr() if bgrad else None, ws.data_ptr(),
            ws.numel(), cnt.data_ptr(), cnt.numel(), st)
    tune = os.environ.get("VITCNN_TUNE")   # "bm,bn,nsplit": forced tile / split (probe library)
    if tune:
        from vitcnn_amd._lib import probe_lib
        L = probe_lib()
        bm, bn, ns = (int(v) for v in tune.split(","))
        L.vc_gemm_tune(bm, bn, ns, 0, -1)
    for _ in range(5):
        L.vc_gemm_ex(*args)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        L.vc_gemm_ex(*args)
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    print(f"ta={ta} tb={tb} M={M} N={N} K={K} flags={flags}: {us:.2f} us, {2.0 * M * N * K / us * 1e-6:.1f} TFLOP/s")


if __name__ == "__main__":
    main()
