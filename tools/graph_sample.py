"""GPU probe: does the replay time of the captured ViT-CNN B=64 step depend on the capture (not only on the
process)?  Captures the step T times in one process and times each graph's replays.  Modes (GS_MODE):
  same  -- recapture on the same lane streams;
  new   -- fresh side-lane streams before every capture;
  shift -- fresh side-lane streams, created after `trial` throw-away streams (shifts which hardware queue
           each new stream is bound to).
usage: [GS_MODE=same|new|shift] python tools/graph_sample.py [T] [K] [fp32|bf16]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))
import torch  # noqa: E402

import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
from vitcnn_amd import AdamW, CrossEntropyLoss, Multimodality_Mamba, fused_train_step  # noqa: E402


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    prec = sys.argv[3] if len(sys.argv) > 3 else "fp32"
    mode = os.environ.get("GS_MODE", "same")
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
    keep = []
    for trial in range(trials):
        if mode in ("new", "shift"):
            m._device_tables(dev).pop("lanes", None)
            if mode == "shift":
                keep.append([torch.cuda.Stream(dev) for _ in range(trial % 4)])
        opt.zero_grad(set_to_none=True)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            fused_train_step(m, crit, hsi, lidar, tgt, optimizer=opt)
        for _ in range(5):
            graph.replay()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(k):
            graph.replay()
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t0) / k * 1e3
        print(f"{mode} trial {trial}: {prec} {ms:.4f} ms/step over {k} replays", flush=True)
        keep.append(graph)


if __name__ == "__main__":
    main()
