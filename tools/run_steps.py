"""Run K eager training steps of the B=64 bench workload (profiling driver for rocprofv3 --pmc).
usage: python tools/run_steps.py [K] [fp32|bf16]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))
import torch  # noqa: E402

import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
from vitcnn_amd import AdamW, CrossEntropyLoss, Multimodality_Mamba, fused_train_step  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    prec = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16, precision=prec).to(dev).train()
    opt = AdamW(m.parameters(), lr=8e-4)
    crit = CrossEntropyLoss(weight=torch.ones(16, device=dev))
    hsi, lidar = torch.rand(64, 144, 9, 9, device=dev), torch.rand(64, 1, 9, 9, device=dev)
    tgt = torch.randint(1, 16, (64,), device=dev)
    for _ in range(k):
        opt.zero_grad(set_to_none=True)
        fused_train_step(m, crit, hsi, lidar, tgt, optimizer=opt)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
