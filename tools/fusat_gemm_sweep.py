"""GPU tool: the vc_gemm_ex calls of one FusAtNet (config 5, B=64) training step, re-timed in isolation
with the automatic configuration and with forced output tiles (vc_gemm_tune bm x bn, split-K and
combine automatic).  Prints per-shape times and the step's summed GEMM time per configuration.
usage: python tools/fusat_gemm_sweep.py [reps]"""
import os
import sys
from collections import OrderedDict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))
import torch  # noqa: E402

import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
knobs.use_probe()   # vc_gemm_tune: the probe library
from vitcnn_amd._lib import lib  # noqa: E402
from vitcnn_amd.fusatnet import FusAtNet  # noqa: E402
from vitcnn_amd.losses import CrossEntropyLoss  # noqa: E402

CONFIGS = [(0, 0, 0), (64, 64, 0), (128, 64, 0), (64, 128, 0), (128, 128, 0)]
if os.environ.get("SWEEP_NSPLIT"):   # (bm, bn) automatic, forced split-K counts instead of tiles
    CONFIGS = [(0, 0, 0)] + [(0, 0, int(v)) for v in os.environ["SWEEP_NSPLIT"].split(",")]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = FusAtNet(144, 1, 16).to(dev).train()
    crit = CrossEntropyLoss(weight=torch.ones(16, device=dev))
    x1, x2 = torch.rand(64, 144, 11, 11, device=dev), torch.rand(64, 1, 11, 11, device=dev)
    t = torch.randint(1, 16, (64,), device=dev)
    L = lib()
    calls = []
    orig = L.vc_gemm_ex

    def spy(*a):
        calls.append(a)
        return orig(*a)

    L.vc_gemm_ex = spy
    crit(m(x1, x2), t).backward()
    torch.cuda.synchronize()
    L.vc_gemm_ex = orig
    raw = L.raw["vc_gemm_ex"]
    st = torch.cuda.Stream(dev)
    shapes = OrderedDict()
    for a in calls:
        key = (a[0], a[1], a[2], a[3], a[4], a[16])
        shapes.setdefault(key, []).append(a)

    def time_call(a, cfg):
        L.vc_gemm_tune(cfg[0], cfg[1], cfg[2], 0, -1)
        args = list(a[:-1]) + [st.cuda_stream]
        for _ in range(2):
            raw(*args)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            raw(*args)
        e1.record(st)
        e1.synchronize()
        L.vc_gemm_tune(0, 0, 0, 0, -1)
        return e0.elapsed_time(e1) / reps * 1e3

    tot = [0.0] * len(CONFIGS)
    best = 0.0
    print(f"{len(calls)} GEMM calls, {len(shapes)} shapes; times in us per call; configs (bm,bn,nsplit) {CONFIGS}")
    print("  tA tB      M      N      K batch count  " + "  ".join(f"{c[0]:>3d}x{c[1]:<3d}/{c[2]:<2d}" for c in CONFIGS) +
          "   TF(auto)")
    for key, lst in shapes.items():
        ts = [time_call(lst[0], c) for c in CONFIGS]
        n = len(lst)
        for i, v in enumerate(ts):
            tot[i] += v * n
        best += min(ts) * n
        ta, tb, M, N, K, batch = key
        print(f"  {ta:2d} {tb:2d} {M:6d} {N:6d} {K:6d} {batch:5d} {n:5d}  " + "  ".join(f"{v:7.1f}" for v in ts) +
              f"   {2.0 * M * N * K * batch / ts[0] * 1e-6:7.1f}", flush=True)
    print("summed over the step (us): " + "  ".join(f"{c[0]}x{c[1]}/{c[2]}: {v:.0f}" for c, v in zip(CONFIGS, tot)) +
          f"  best-of: {best:.0f}")


if __name__ == "__main__":
    main()
