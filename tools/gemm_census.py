"""GPU tool: every vc_gemm_ex / vc_gemm_group_add problem of one training step (B=64), re-timed in isolation with HIP events.
Prints shape, layout and time per call for the first-round fp32 kernel (legacy), the current fp32
kernel and the bf16-operand kernel, sorted by the current fp32 time.
usage: python tools/gemm_census.py [reps]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))
import torch  # noqa: E402

import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
from vitcnn_amd import CrossEntropyLoss, Multimodality_Mamba, fused_train_step  # noqa: E402
from vitcnn_amd._lib import lib  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16).to(dev).train()
    crit = CrossEntropyLoss(weight=torch.ones(16, device=dev))
    hsi, lidar = torch.rand(64, 144, 9, 9, device=dev), torch.rand(64, 1, 9, 9, device=dev)
    tgt = torch.randint(1, 16, (64,), device=dev)
    fused_train_step(m, crit, hsi, lidar, tgt)
    torch.cuda.synchronize()
    L = lib()
    calls = []
    orig, orig_add = L.vc_gemm_ex, L.vc_gemm_group_add

    def spy(*a):
        calls.append(a)
        return orig(*a)

    def spy_add(group, *a):   # grouped problems: vc_gemm_ex's arguments without the stream
        calls.append(a + (None,))
        return orig_add(group, *a)

    L.vc_gemm_ex, L.vc_gemm_group_add = spy, spy_add
    fused_train_step(m, crit, hsi, lidar, tgt)
    torch.cuda.synchronize()
    L.vc_gemm_ex, L.vc_gemm_group_add = orig, orig_add
    raw = L.raw["vc_gemm_ex"]
    st = torch.cuda.Stream(dev)
    def time_call(a, extra_flags):
        args = list(a[:-1]) + [st.cuda_stream]
        args[21] = a[21] | extra_flags
        for _ in range(3):
            raw(*args)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            raw(*args)
        e1.record(st)
        e1.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3

    rows = []
    for a in calls:
        ta, tb, M, N, K = a[0], a[1], a[2], a[3], a[4]
        batch = a[16]
        base = a[21] & ~(2 | 4 | 8 | 16 | 32)
        a = a[:21] + (base,) + a[22:]
        t_auto, t_leg, t_v2, t_bf = time_call(a, 0), time_call(a, 4), time_call(a, 16), time_call(a, 2)
        t_bfk = time_call(a, 2 | 32)   # bf16 on the K-contiguous kernel (no pipelined kernel)
        fl = 2.0 * M * N * K * batch
        rows.append((t_auto, t_leg, t_v2, t_bf, t_bfk, ta, tb, M, N, K, batch, a[22] is not None,
                     fl / min(t_leg, t_v2) * 1e-6, fl / t_bf * 1e-6))
    rows.sort(reverse=True)
    tots = [sum(r[i] for r in rows) for i in range(5)]
    print(f"{len(rows)} GEMMs, isolated sums (us): auto {tots[0]:.1f}  legacy {tots[1]:.1f}  pipe {tots[2]:.1f}  "
          f"bf16 {tots[3]:.1f}  bf16 (K-contiguous kernel) {tots[4]:.1f}")
    print("  auto legacy   pipe   bf16 bf16-k  tA tB      M      N      K  batch bgrad TF(fp32) TF(bf16)")
    for r in rows:
        print("%6.1f %6.1f %6.1f %6.1f %6.1f  %d  %d %6d %6d %6d %5d %5s %8.1f %8.1f" % r)


if __name__ == "__main__":
    main()
