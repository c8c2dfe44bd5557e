"""GPU tool: is the captured ViT-CNN step bound by the host's graph submission?  Times K graph.replay() calls on the
host alone (no synchronisation between them) and then the device drain, for the four-lane step and the
one-stream step (VITCNN_LANE_MAP=0,0,0,0 via tools/knobs.py).  usage: python tools/replay_host.py [K]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))
import torch  # noqa: E402

import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
from vitcnn_amd import AdamW, CrossEntropyLoss, Multimodality_Mamba, fused_train_step  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16).to(dev).train()
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
    for _ in range(10):
        graph.replay()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    hs = []
    for _ in range(k):
        a = time.perf_counter()
        graph.replay()
        hs.append(time.perf_counter() - a)
    t1 = time.perf_counter()
    torch.cuda.synchronize(dev)
    t2 = time.perf_counter()
    hs.sort()
    print(f"replay host call: median {hs[len(hs) // 2] * 1e3:.4f} ms, max {hs[-1] * 1e3:.4f} ms; {k} calls enqueued in "
          f"{(t1 - t0) * 1e3:.1f} ms, drained {(t2 - t1) * 1e3:.1f} ms later; {(t2 - t0) / k * 1e3:.4f} ms/step",
          flush=True)


if __name__ == "__main__":
    main()
