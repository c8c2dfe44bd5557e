"""GPU tool: every distinct vc_gemm_ex shape of one ViT-CNN training step (B=64), re-timed in isolation
under each forced configuration (vc_gemm_tune: tile, split-K slices, prefetch depth, combine path) for
fp32 and bf16 operands.  Writes gpurun_out/gemm_sweep.json and prints, per shape, the automatic
choice's time against the best configuration found.
usage: python tools/gemm_sweep.py [reps] [--quick] [--only-ta1]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))
import torch  # noqa: E402

import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
knobs.use_probe()   # vc_gemm_tune: the probe library
from vitcnn_amd import CrossEntropyLoss, Multimodality_Mamba, fused_train_step  # noqa: E402
from vitcnn_amd._lib import lib  # noqa: E402


def capture_calls(dev):
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16).to(dev).train()
    crit = CrossEntropyLoss(weight=torch.ones(16, device=dev))
    hsi, lidar = torch.rand(64, 144, 9, 9, device=dev), torch.rand(64, 1, 9, 9, device=dev)
    tgt = torch.randint(1, 16, (64,), device=dev)
    fused_train_step(m, crit, hsi, lidar, tgt)
    torch.cuda.synchronize()
    L = lib()
    calls = []
    orig = L.vc_gemm_ex

    def spy(*a):
        calls.append(a)
        return orig(*a)

    L.vc_gemm_ex = spy
    fused_train_step(m, crit, hsi, lidar, tgt)
    torch.cuda.synchronize()
    L.vc_gemm_ex = orig
    return m, calls  # keep the model (and its workspace) alive: the captured pointers are into it


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 10
    quick = "--quick" in sys.argv
    dev = torch.device("cuda", 0)
    model, calls = capture_calls(dev)
    L = lib()
    raw = L.raw["vc_gemm_ex"]
    st = torch.cuda.Stream(dev)
    seen = {}
    for a in calls:
        key = (a[0], a[1], a[2], a[3], a[4], a[16], a[22] is not None)
        seen.setdefault(key, a)

    def time_call(a, flags):
        args = list(a[:-1]) + [st.cuda_stream]
        args[21] = (a[21] & 1) | flags
        for _ in range(2):
            raw(*args)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            raw(*args)
        e1.record(st)
        e1.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3

    splits = [1, 2, 4, 8, 16, 32, 64, 128, 256] if not quick else [1, 4, 16, 64]
    out = []
    only_ta1 = "--only-ta1" in sys.argv
    for key, a in seen.items():
        ta, tb, M, N, K, batch, bg = key
        if only_ta1 and not ta:
            continue
        for flags, KT in ((8, 32), (2, 64)):  # fp32: the K-contiguous kernel (8); bf16 (2)
            L.vc_gemm_tune(0, 0, 0, 0, -1)
            t_auto = time_call(a, flags)
            t_leg = time_call(a, 4) if flags == 8 else None
            best = (t_auto, "auto")
            res = []
            for bm in (64, 128):
                for bn in (64, 128):
                    for ns in splits:
                        if ns > 1 and ns * KT > K:
                            continue
                        for pf in (1, 2):
                            for comb in ((0, 1) if ns > 1 else (0,)):
                                L.vc_gemm_tune(bm, bn, ns, pf, comb)
                                t = time_call(a, flags)
                                res.append((t, bm, bn, ns, pf, comb))
                                if t < best[0]:
                                    best = (t, (bm, bn, ns, pf, comb))
            L.vc_gemm_tune(0, 0, 0, 0, -1)
            res.sort()
            out.append({"ta": ta, "tb": tb, "M": M, "N": N, "K": K, "batch": batch, "bgrad": bg,
                        "dtype": "bf16" if flags == 2 else "fp32", "auto_us": t_auto, "legacy_us": t_leg,
                        "best_us": best[0], "best": best[1], "top5": res[:5]})
            print(f"{'bf16' if flags == 2 else 'fp32'} ta={ta} tb={tb} M={M} N={N} K={K} b={batch} bg={int(bg)}: "
                  f"auto {t_auto:.1f} legacy {t_leg if t_leg else 0:.1f} best {best[0]:.1f} {best[1]}", flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "gemm_sweep.json"), "w") as f:
        json.dump(out, f, indent=1)
    for dt in ("fp32", "bf16"):
        rows = [r for r in out if r["dtype"] == dt]
        print(dt, "sum over distinct shapes: auto %.1f us, best %.1f us" % (sum(r["auto_us"] for r in rows),
                                                                         sum(r["best_us"] for r in rows)))


if __name__ == "__main__":
    main()
