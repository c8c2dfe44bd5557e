"""GPU tool: the step's large fp32 GEMM shapes under the k-major kernel (F_LEGACY), the pipelined LDS-DMA
kernel (F_PIPE) and the automatic choice, timed in isolation (HIP events, back-to-back reps), each result
checked against the float64 product.  usage: python tools/gemm_pipe_bench.py [reps] [tune: bm,bn,nsplit ...]"""
import os
import sys

import knobs  # noqa: F401,E402
import torch

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 50
TUNES = [tuple(int(x) for x in a.split(",")) for a in sys.argv[2:]]
if TUNES:
    knobs.use_probe()
from vitcnn_amd._lib import lib  # noqa: E402

F_LEGACY, F_PIPE = 4, 16
# (tA, tB, M, N, K, bias_grad): the step's critical-path GEMMs (profiles/r03_critical_path_s2.txt)
SHAPES = [(0, 1, 3136, 256, 1296, 0), (0, 0, 3136, 1296, 256, 0), (1, 0, 256, 1296, 3136, 1),
          (0, 1, 1600, 144, 2304, 0), (1, 0, 144, 2304, 1600, 1), (0, 0, 1600, 2304, 144, 0),
          (1, 0, 256, 512, 3136, 1), (0, 0, 3136, 512, 256, 0), (0, 1, 3136, 256, 512, 0),
          (1, 0, 256, 144, 5184, 1), (0, 0, 5184, 144, 256, 0), (0, 1, 5184, 256, 144, 0),
          (0, 1, 3136, 256, 256, 0), (0, 1, 3136, 256, 128, 0), (0, 0, 3136, 256, 256, 0),
          (1, 0, 256, 256, 3136, 0), (1, 0, 128, 256, 3136, 1), (0, 1, 3136, 128, 272, 0),
          (0, 1, 1600, 144, 288, 0), (1, 0, 144, 288, 1600, 1), (0, 0, 1600, 288, 144, 0)]


def main():
    L = lib()
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    ws = torch.empty(1 << 25, device=dev)
    cnt = torch.zeros(1 << 16, dtype=torch.int32, device=dev)
    g = torch.Generator(device="cpu").manual_seed(0)
    tot = {}
    print(f"{'tA':>2} {'tB':>2} {'M':>5} {'N':>5} {'K':>5} bg   legacy    pipe    auto  (us)  TF(pipe)  err(pipe)")
    for ta, tb, M, N, K, bg in SHAPES:
        A = (torch.rand(K, M, generator=g) if ta else torch.rand(M, K, generator=g)) * 2 - 1
        B = (torch.rand(N, K, generator=g) if tb else torch.rand(K, N, generator=g)) * 2 - 1
        ref = ((A.t() if ta else A).double() @ (B.t() if tb else B).double())
        Ad, Bd = A.to(dev), B.to(dev)
        C = torch.empty(M, N, device=dev)
        bgr = torch.empty(M, device=dev) if bg else None
        lda, ldb = (M if ta else K), (K if tb else N)

        def call(flags):
            L.raw["vc_gemm_ex"](ta, tb, M, N, K, 1.0, Ad.data_ptr(), lda, 0, Bd.data_ptr(), ldb, 0, 0.0, C.data_ptr(),
                                N, 0, 1, None, None, 0, 0, flags, bgr.data_ptr() if bgr is not None else None,
                                ws.data_ptr(), ws.numel(), cnt.data_ptr(), cnt.numel(), st.cuda_stream)

        def timed(flags):
            with torch.cuda.stream(st):
                for _ in range(5):
                    call(flags)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(REPS):
                    call(flags)
                e1.record(st)
            e1.synchronize()
            return e0.elapsed_time(e1) / REPS * 1e3

        res = {}
        for name, fl in (("legacy", F_LEGACY), ("pipe", F_PIPE), ("auto", 0)):
            res[name] = timed(fl)
            tot[name] = tot.get(name, 0.0) + res[name]
        with torch.cuda.stream(st):
            C.fill_(float("nan"))     # on the stream the GEMM runs on
            call(F_PIPE)
        torch.cuda.synchronize()
        err = float((C.cpu().double() - ref).abs().max() / ref.abs().max())
        if bg:
            berr = float((bgr.cpu().double() - (A.double().sum(0))).abs().max() / A.double().sum(0).abs().max())
            err = max(err, berr)
        tf = 2.0 * M * N * K / res["pipe"] * 1e-6
        print(f"{ta:>2} {tb:>2} {M:>5} {N:>5} {K:>5} {bg:>2} {res['legacy']:8.1f} {res['pipe']:7.1f} {res['auto']:7.1f}"
              f"        {tf:7.1f}   {err:.1e}")
        for t in TUNES:
            L.vc_gemm_tune(t[0], t[1], t[2], 0, -1)
            tt = timed(F_PIPE)
            L.vc_gemm_tune(0, 0, 0, 0, -1)
            print(f"      tune {t}: {tt:7.1f} us  {2.0 * M * N * K / tt * 1e-6:6.1f} TF")
    print("sums (us): " + "  ".join(f"{k} {v:.1f}" for k, v in tot.items()))


if __name__ == "__main__":
    main()
