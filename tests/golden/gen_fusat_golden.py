"""Generate FusAtNet golden vectors from the REFERENCE module (build container only).

Imports `/root/reference/model/compare_method/FusAtNet.py` (torch only), seeds torch with 0 and builds
`FusAtNet(144, 1, 16)` as `model_utils.py:109-118` does (patch 11).  The 36.9 M parameters are not
stored: the product module, created under the same seed in the same order, reproduces them, and
per-tensor sums are stored to pin that.  Stores (numbers only) in tests/golden/fusat_b4.npz: inputs
x1 ~ U[0,1) [4,144,11,11], x2 ~ U[0,1) [4,1,11,11], train-mode logits (batch statistics), the BN
running statistics' sums after that forward, and eval-mode logits afterwards.  No backward: the
reference's raises (in-place add on a saved ReLU output, FusAtNet.py:44).

Run:  python tests/golden/gen_fusat_golden.py
"""
import importlib.util
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/model/compare_method/FusAtNet.py"


def main(B=4):
    spec = importlib.util.spec_from_file_location("ref_fusat", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    torch.manual_seed(0)
    net = mod.FusAtNet(144, 1, 16)
    sums = {"s:" + k: np.float64(v.double().sum()) for k, v in net.state_dict().items() if v.is_floating_point()}
    g = torch.Generator().manual_seed(2)
    x1 = torch.rand(B, 144, 11, 11, generator=g)
    x2 = torch.rand(B, 1, 11, 11, generator=g)
    net.train()
    with torch.no_grad():
        lt = net(x1, x2)
    run = {"r:" + k: np.float64(v.double().sum()) for k, v in net.state_dict().items() if "running" in k}
    net.eval()
    with torch.no_grad():
        le = net(x1, x2)
    np.savez_compressed(os.path.join(HERE, "fusat_b4.npz"), x1=x1.numpy(), x2=x2.numpy(), logits_train=lt.numpy(),
                        logits_eval=le.numpy(), **sums, **run)
    print("wrote fusat_b4.npz", lt.shape)


if __name__ == "__main__":
    main()
