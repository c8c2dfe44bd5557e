"""GPU probe: what a kernel boundary costs inside a replayed single-stream hipGraph.

In the serial ViT-CNN step every kernel, even a one-thread one, spans >= ~4.8 us start to start
(tools/step_timeline.py), while a chain of 256-float fills costs ~1.6 us per kernel (edge_probe.py).
This separates the candidates: the bytes the previous kernel left dirty (fills of growing size),
the kernel-argument block (a 1x1x1 GEMM with its ~200-byte GemmArgs), and a single-thread kernel.
usage: python tools/boundary_probe.py [N]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))
import torch  # noqa: E402

import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
from vitcnn_amd._lib import lib  # noqa: E402


def replay_us(build, n, reps=50):
    s0 = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    s0.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s0):
        build()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        build()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps / n * 1e6


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    L = lib()
    big = torch.empty(1 << 24, device="cuda")
    a = torch.rand(64, 64, device="cuda")
    c = torch.empty(64, 64, device="cuda")
    ws = torch.empty(1 << 20, device="cuda")
    ctr = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")

    def fills(size, stride=0):
        def fn():
            s = torch.cuda.current_stream().cuda_stream
            for i in range(n):
                L.vc_fill(size, big.data_ptr() + 4 * ((i * stride) % (1 << 22)), 1.0, s)
        return fn

    def gemms():
        s = torch.cuda.current_stream().cuda_stream
        for _ in range(n):
            L.vc_gemm_ex(0, 1, 16, 16, 16, 1.0, a.data_ptr(), 64, 0, a.data_ptr(), 64, 0, 0.0, c.data_ptr(), 64, 0, 1,
                         None, None, 0, 0, 0, None, ws.data_ptr(), ws.numel(), ctr.data_ptr(), ctr.numel(), s)

    def gemms_64():
        s = torch.cuda.current_stream().cuda_stream
        for _ in range(n):
            L.vc_gemm_ex(0, 1, 64, 64, 64, 1.0, a.data_ptr(), 64, 0, a.data_ptr(), 64, 0, 0.0, c.data_ptr(), 64, 0, 1,
                         None, None, 0, 0, 0, None, ws.data_ptr(), ws.numel(), ctr.data_ptr(), ctr.numel(), s)

    def mixed():
        s = torch.cuda.current_stream().cuda_stream
        for i in range(n // 2):
            L.vc_fill(1 << 20, big.data_ptr(), 1.0, s)
            L.vc_fill(256, big.data_ptr() + 4 * (1 << 23), 1.0, s)

    cases = [("fill 256 floats", fills(256)), ("fill 64K floats", fills(1 << 16)),
             ("fill 1M floats (4 MB)", fills(1 << 20)), ("fill 4M floats (16 MB)", fills(1 << 22)),
             ("fill 1M, moving 4 MB window", fills(1 << 20, 1 << 20)),
             ("gemm 16x16x16 (GemmArgs kernarg)", gemms), ("gemm 64x64x64", gemms_64),
             ("alternating fill 4 MB / fill 1 KB", mixed)]
    for name, fn in cases:
        print(f"{name:36s} {replay_us(fn, n):7.2f} us per kernel", flush=True)


if __name__ == "__main__":
    main()
