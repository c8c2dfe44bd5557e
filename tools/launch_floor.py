"""Launch-floor probe: device time per dependent kernel under hipGraph replay on this GPU.

  (a) N serial trivial kernels (vc_fill of 256 floats) on one stream, captured and replayed;
  (b) N serial small GEMMs (64x64x64) the same way.
Prints microseconds per kernel; a step of n_critical dependent launches costs at least
n_critical x (a)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))

import torch  # noqa: E402

import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
from vitcnn_amd._lib import lib  # noqa: E402


def replay_us(fn, n, reps=20):
    s = torch.cuda.current_stream()
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(s)
    with torch.cuda.stream(side):
        fn()
    s.wait_stream(side)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps / n * 1e6


def main():
    L = lib()
    n = 300
    buf = torch.empty(1 << 20, device="cuda")
    scr = torch.empty(1 << 22, device="cuda")

    def fills():
        st = torch.cuda.current_stream().cuda_stream
        for i in range(n):
            L.vc_fill(256, buf.data_ptr(), float(i), st)

    a = torch.randn(64, 64, device="cuda")
    w = torch.randn(64, 64, device="cuda")
    c = torch.empty(64, 64, device="cuda")

    def gemms():
        st = torch.cuda.current_stream().cuda_stream
        for _ in range(n):
            L.vc_gemm(0, 1, 64, 64, 64, 1.0, a.data_ptr(), 64, 0, w.data_ptr(), 64, 0, 0.0, c.data_ptr(), 64, 0, 1,
                      None, None, 0, 0, 0, None, scr.data_ptr(), scr.numel(), st)

    print(f"serial trivial kernel (fill 256): {replay_us(fills, n):.2f} us/kernel")
    print(f"serial small gemm 64x64x64:      {replay_us(gemms, n):.2f} us/kernel")


if __name__ == "__main__":
    main()
