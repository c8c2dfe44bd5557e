"""GPU diagnostic: which GEMMs of the bf16 mode move the ViT-CNN logits most.  Runs the golden B=64
train-mode forward in bf16 with one GEMM issue index at a time kept fp32 (model._BF16_EXACT) and prints,
per call site, the logits deviation from the fp32 golden logits and the argmax agreement.
usage: python tools/bf16_sites.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "vit-cnn_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from helpers import golden_batch, hash_state_dict, load_npz  # noqa: E402
import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
from vitcnn_amd import Multimodality_Mamba  # noqa: E402
import vitcnn_amd.model as M  # noqa: E402


def main():
    ref = load_npz("vitcnn_b64.npz")["logits"]
    hsi, lidar, _ = golden_batch("golden.b64", 64)
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16, "multi_clock_gate", precision="bf16")
    m.load_state_dict(hash_state_dict())
    m = m.cuda().train()
    x1, x2 = hsi.cuda(), lidar.cuda()

    def run():
        with torch.no_grad():
            y = m(x1, x2).float().cpu().numpy()
        dev = float(np.abs(y - ref).max() / np.abs(ref).max())
        return dev, float((y.argmax(1) == ref.argmax(1)).mean())

    M._GEMM_SITES = []
    base = run()
    sites = M._GEMM_SITES
    M._GEMM_SITES = None
    print(f"bf16 all: dev {base[0]:.4e} agree {base[1]:.4f}  ({len(sites)} GEMMs)", flush=True)
    M._BF16_EXACT = {s[0] for s in sites}
    print("all exact:", run(), flush=True)
    res = []
    for s in sites:
        if s[-1]:
            continue
        M._BF16_EXACT = {s[0]}
        d, a = run()
        res.append((d, a, s))
    res.sort(key=lambda r: r[0])
    for d, a, s in res[:25]:
        print(f"exact #{s[0]:3d} {s[1]}:{s[2]} M{s[3]} N{s[4]} K{s[5]}: dev {d:.4e} agree {a:.4f}", flush=True)
    # greedy: keep the best sites exact cumulatively
    keep = set()
    for d, a, s in res[:12]:
        keep.add(s[0])
        M._BF16_EXACT = set(keep)
        print("cumulative", sorted(keep), run(), flush=True)


if __name__ == "__main__":
    main()
