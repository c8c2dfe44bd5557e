"""GPU tool: the S2EFT config-5 train step (forward, weighted CE, backward, fused Adam) captured as one hipGraph and
replayed K times -- the bench leg alone, for A/B runs and rocprofv3 --kernel-trace.
usage: python tools/s2eft_step.py [K] [side 0|1|2]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))
import torch  # noqa: E402

import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
import vitcnn_amd.s2eft as S  # noqa: E402
from vitcnn_amd import CrossEntropyLoss  # noqa: E402
from vitcnn_amd.optim import AdamW  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    if len(sys.argv) > 2:
        S._SIDE_STREAM = int(sys.argv[2])
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = S.ViT(image_size=7, near_band=3, num_patches=144, num_classes=16, dim=64, depth=5, heads=4, mlp_dim=8,
              dropout=0.0, emb_dropout=0.0, mode="CAF").to(dev).train()
    opt = AdamW(m.parameters(), lr=5e-4, weight_decay=0.0)
    w = torch.ones(16, device=dev)
    w[0] = 0.0
    crit = CrossEntropyLoss(weight=w)
    g = torch.Generator().manual_seed(7)
    x = torch.rand(64, 145, 147, generator=g).to(dev)
    t = torch.randint(1, 16, (64,), generator=g).to(dev)
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(3):
            opt.zero_grad(set_to_none=True)
            crit(m(x), t).backward()
            opt.step()
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize(dev)
    opt.zero_grad(set_to_none=True)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        crit(m(x), t).backward()
        opt.step()
    for _ in range(5):
        graph.replay()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(k):
        graph.replay()
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) / k * 1e3
    print(f"s2eft side={int(S._SIDE_STREAM)}: {ms:.4f} ms/step over {k} graph replays", flush=True)


if __name__ == "__main__":
    main()
