"""Profiling driver: the bench's ViT-CNN B=64 training step (forward, CE, backward, AdamW) captured as
one hipGraph and replayed K times, nothing else — so a rocprofv3 --kernel-trace of it holds only
this step's kernels (tools/step_timeline.py takes the last full step out of it).
usage: python tools/prof_step.py [K] [fp32|bf16]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))
import torch  # noqa: E402

import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
from vitcnn_amd import AdamW, CrossEntropyLoss, Multimodality_Mamba, fused_train_step  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    prec = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16, precision=prec).to(dev).train()
    opt = AdamW(m.parameters(), lr=8e-4)
    w = torch.ones(16)
    w[0] = 0.0
    crit = CrossEntropyLoss(weight=w.to(dev))
    g = torch.Generator().manual_seed(1000)
    hsi = torch.rand(64, 144, 9, 9, generator=g).to(dev)
    lidar = torch.rand(64, 1, 9, 9, generator=g).to(dev)
    tgt = torch.randint(1, 16, (64,), generator=g).to(dev)
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(3):
            opt.zero_grad(set_to_none=True)
            fused_train_step(m, crit, hsi, lidar, tgt, optimizer=opt)
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize(dev)
    opt.zero_grad(set_to_none=True)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        fused_train_step(m, crit, hsi, lidar, tgt, optimizer=opt)
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(k):
        graph.replay()
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) / k * 1e3
    print(f"{prec}: {ms:.4f} ms/step ({64 / ms * 1e3:.1f} patches/s) over {k} graph replays", flush=True)


if __name__ == "__main__":
    main()
