"""Diagnostic (GPU box): per-parameter gradient error of the HIP path vs a float64 oracle, next to the
fp32 oracle's own error.  usage: python tools/diag_grads.py [B]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "vit-cnn_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from helpers import golden_batch, hash_state_dict, masked_oracle_step, relu_masks_from_workspace  # noqa: E402
from oracle import vitcnn_oracle as O  # noqa: E402
import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
from vitcnn_amd import CrossEntropyLoss, Multimodality_Mamba  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    sd = hash_state_dict()
    hsi, lidar, target = golden_batch("golden.b4", 4) if B == 4 else golden_batch("golden.b64", 64)
    w = O.ce_class_weights(16)
    st32 = O.make_state(sd)
    O.train_step(st32, hsi, lidar, target, w)
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16)
    m.load_state_dict(sd)
    m = m.cuda().train()
    loss = CrossEntropyLoss(weight=w.cuda())(m(hsi.cuda(), lidar.cuda()), target.cuda())
    loss.backward()
    torch.cuda.synchronize()
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
    st64 = O.make_state(sd64)
    masked_oracle_step(O, st64, hsi.double(), lidar.double(), target, w.double(), relu_masks_from_workspace(m, B))
    flat = m.flat_params.grad.detach().cpu().double()
    named = dict(m.named_parameters())
    rows = []
    for n in O.param_names(st64):
        g64 = st64[n].grad
        if g64 is None:
            continue
        off = m._poff[n]
        got = flat[off:off + named[n].numel()].view(named[n].shape)
        e = float((got - g64).abs().max())
        e32 = float((st32[n].grad.double() - g64).abs().max())
        sc = float(g64.abs().max())
        rows.append((e / max(3 * e32, 1e-3 * sc, 1e-12), e, e32, sc, n))
    rows.sort(reverse=True)
    print("badness(err/max(3*err32,1e-3*scale))  err_gpu   err_fp32  scale     name")
    for r in rows[:60]:
        print("%.3e  %.2e  %.2e  %.2e  %s" % r)
    for blk in ("hsi1", "hsi2"):
        n = blk + ".global_view.pos_embed"
        off = m._poff[n]
        got = flat[off:off + named[n].numel()].view(named[n].shape)[0]
        g64 = st64[n].grad[0]
        per_tok = (got - g64).abs().max(dim=1).values / g64.abs().max()
        print(blk, "pos_embed per-token rel err (token: err):")
        print(" ".join(f"{i}:{v:.1e}" for i, v in enumerate(per_tok.tolist())))
        n = blk + ".global_view.layers.0.D"
        off = m._poff[n]
        got = flat[off:off + named[n].numel()]
        g64 = st64[n].grad
        print(blk, "D grad per-channel rel err:", " ".join(f"{v:.1e}" for v in ((got - g64).abs() / g64.abs().max()).tolist()))


if __name__ == "__main__":
    main()
