"""Profiling driver for config 5 (rocprofv3 --pmc): K S2EFT train steps and one FusAtNet forward at
B = 64 (eager), so per-kernel counters of the MFMA attention / conv GEMMs can be read."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))
import torch  # noqa: E402

import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
from vitcnn_amd import CrossEntropyLoss  # noqa: E402
from vitcnn_amd.fusatnet import FusAtNet  # noqa: E402
from vitcnn_amd.optim import AdamW  # noqa: E402
from vitcnn_amd.s2eft import ViT  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = ViT(image_size=7, near_band=3, num_patches=144, num_classes=16, dim=64, depth=5, heads=4, mlp_dim=8).to(dev)
    opt = AdamW(m.parameters(), lr=5e-4, weight_decay=0.0)
    crit = CrossEntropyLoss(weight=torch.ones(16, device=dev))
    x = torch.rand(64, 145, 147, device=dev)
    t = torch.randint(1, 16, (64,), device=dev)
    for _ in range(k):
        opt.zero_grad(set_to_none=True)
        crit(m(x), t).backward()
        opt.step()
    f = FusAtNet(144, 1, 16).to(dev).train()
    with torch.no_grad():
        f(torch.rand(64, 144, 11, 11, device=dev), torch.rand(64, 1, 11, 11, device=dev))
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
