"""Generate S2EFT golden vectors from the REFERENCE module (run in the build container only).

Imports `/root/reference/model/compare_method/S2EFT.py` (needs only torch + einops) and runs one
train-mode forward/backward of `ViT` as `model_utils.py:400-423` builds it, with dropout 0 (the
reference's own dropout 0.1 is random, so parity is only defined at p = 0).  The one patch to
reference behaviour: `torch.Tensor.cuda` is the identity while it runs, because the reference
allocates its gate's zero tensor with `.cuda()` (S2EFT.py:141) and this container has no GPU.

Inputs: x ~ U[0,1) [B, 145, 147] (144 HSI + 1 LiDAR band tokens x 7*7*3 near-band values), labels
in [1, 15], class weights with weight[0] = 0 (ignored class).  Stores the initial state_dict,
inputs, logits, loss and every parameter gradient (numbers only) in tests/golden/s2eft_b4.npz.

Run:  python tests/golden/gen_s2eft_golden.py
"""
from __future__ import annotations

import importlib.util
import os

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/model/compare_method/S2EFT.py"


def main(B=4, n_bands=144, ncls=16):
    N = n_bands + 1
    spec = importlib.util.spec_from_file_location("ref_s2eft", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    torch.manual_seed(0)
    net = mod.ViT(image_size=7, near_band=3, num_patches=n_bands, num_classes=ncls, dim=64, depth=5, heads=4,
                  mlp_dim=8, dropout=0.0, emb_dropout=0.0, mode="CAF")
    net.train()
    g = torch.Generator().manual_seed(1)
    x = torch.rand(B, N, 147, generator=g)
    target = torch.randint(1, ncls, (B,), generator=g)
    weight = torch.ones(ncls)
    weight[0] = 0.0
    sd0 = {k: v.detach().clone() for k, v in net.state_dict().items()}
    cuda = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *a, **k: self
    try:
        logits = net(x)
    finally:
        torch.Tensor.cuda = cuda
    loss = F.cross_entropy(logits, target, weight=weight)
    loss.backward()
    out = {"x": x.numpy(), "target": target.numpy(), "weight": weight.numpy(),
           "logits": logits.detach().numpy(), "loss": np.float32(loss.item())}
    for k, v in sd0.items():
        out["p:" + k] = v.numpy()
    for k, p in net.named_parameters():
        out["g:" + k] = (p.grad if p.grad is not None else torch.zeros_like(p)).numpy()
    np.savez_compressed(os.path.join(HERE, "s2eft_b4.npz"), **out)
    print("wrote s2eft_b4.npz", logits.shape, float(loss))


if __name__ == "__main__":
    main()
