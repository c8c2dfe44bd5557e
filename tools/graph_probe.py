"""GPU probe: eager vs hipGraph-captured training step of the multi-lane program (same result?)."""
import faulthandler
import os
import sys

faulthandler.enable()
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))
import torch  # noqa: E402

import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
from vitcnn_amd import CrossEntropyLoss, Multimodality_Mamba, fused_train_step  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "graph"
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16).to(dev).train()
    crit = CrossEntropyLoss(weight=torch.ones(16, device=dev))
    hsi = torch.rand(64, 144, 9, 9, device=dev)
    lidar = torch.rand(64, 1, 9, 9, device=dev)
    tgt = torch.randint(1, 16, (64,), device=dev)
    holder = {}

    def fb():
        if mode == "autograd":
            loss = crit(m(hsi, lidar), tgt)
            loss.backward()
        else:
            loss = fused_train_step(m, crit, hsi, lidar, tgt)
        holder["loss"] = loss

    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(3):
            m.zero_grad(set_to_none=True)
            fb()
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize()
    print("eager ok", float(holder["loss"]), flush=True)
    g_eager = m.flat_params.grad.clone()

    m.zero_grad(set_to_none=True)
    graph = torch.cuda.CUDAGraph()
    print("capturing", flush=True)
    with torch.cuda.graph(graph):
        fb()
    print("captured", flush=True)
    graph.replay()
    torch.cuda.synchronize()
    print("replayed", float(holder["loss"]), flush=True)
    g = m.flat_params.grad
    print("max |graph - eager| grad", float((g - g_eager).abs().max()), flush=True)


if __name__ == "__main__":
    main()
