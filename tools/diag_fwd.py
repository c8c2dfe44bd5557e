"""Diagnostic (GPU box): forward-activation error of the HIP path vs a float64 oracle, stage by stage,
next to the fp32 CPU oracle's own error.  usage: python tools/diag_fwd.py [B]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "vit-cnn_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from helpers import golden_batch, hash_state_dict  # noqa: E402
from oracle import vitcnn_oracle as O  # noqa: E402
import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
from vitcnn_amd import CrossEntropyLoss, Multimodality_Mamba  # noqa: E402

HOOK = ["hsi_mamba", "token_learner", "bn_conv3_relu", "conv_bn_relu_1x1", "non_local", "layernorm", "fusion"]


def run_oracle(sd, hsi, lidar, target, w, dtype):
    caps = {}
    orig = {n: getattr(O, n) for n in HOOK}

    def wrap(name, fn):
        def inner(P, pfx, *a):
            out = fn(P, pfx, *a)
            if P.training:
                caps[pfx] = (tuple(x.detach().clone() for x in a if torch.is_tensor(x)), out.detach().clone())
            return out
        return inner

    for n in HOOK:
        setattr(O, n, wrap(n, orig[n]))
    try:
        sdd = {k: (v.to(dtype) if v.is_floating_point() else v) for k, v in sd.items()}
        st = O.make_state(sdd)
        O.train_step(st, hsi.to(dtype), lidar.to(dtype), target, w.to(dtype))
    finally:
        for n in HOOK:
            setattr(O, n, orig[n])
    return caps


def nhwc(t):
    """oracle NCHW [B,C,H,W] -> rows [B*H*W, C]; [B,S,C] -> [B*S, C]"""
    if t.dim() == 4:
        return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])
    return t.reshape(-1, t.shape[-1])


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    sd = hash_state_dict()
    hsi, lidar, target = golden_batch("golden.b4", 4) if B == 4 else golden_batch("golden.b64", 64)
    w = O.ce_class_weights(16)
    c32 = run_oracle(sd, hsi, lidar, target, w, torch.float32)
    c64 = run_oracle(sd, hsi, lidar, target, w, torch.float64)
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16)
    m.load_state_dict(sd)
    m = m.cuda().train()
    loss = CrossEntropyLoss(weight=w.cuda())(m(hsi.cuda(), lidar.cuda()), target.cuda())
    torch.cuda.synchronize()
    ws = next(v for k, v in m._ws.items() if k[2] == ("train", "grad"))
    gmap = {}
    for blk in ("hsi1", "hsi2"):
        gmap[blk + ".global_view"] = blk + ".G"
        gmap[blk + ".global_feature"] = blk + ".global_feature.Z"
        gmap[blk + ".channel_token"] = blk + ".channel_token.Z"
        gmap[blk + ".local_feature"] = blk + ".local_feature.out"
        gmap[blk + ".ln3"] = blk + ".Fg"
        gmap[blk + ".ln4"] = blk + ".Fc"
        gmap[blk + ".FusionLayer.FusionLayer"] = blk + ".FusionLayer.FusionLayer.out"
        gmap[blk + ".fusion.FusionLayer"] = blk + ".fusion.FusionLayer.out"
    for x in ("lidar1", "lidar2"):
        gmap[x] = x + ".out"
    for x in ("fusion1", "fusion2"):
        gmap[x + ".FusionLayer"] = x + ".FusionLayer.out"
    print("%-42s %10s %10s %8s  %s" % ("stage", "err_gpu", "err_fp32", "ratio", "relu-sign flips gpu/fp32"))
    for pfx, (ins64, out64) in c64.items():
        if pfx not in gmap:
            continue
        r64 = nhwc(out64)
        r32 = nhwc(c32[pfx][1]).double()
        got = ws.tensor(gmap[pfx])[: r64.numel()].view(r64.shape).double().cpu()
        sc = float(r64.abs().max())
        e = float((got - r64).abs().max()) / sc
        e32 = float((r32 - r64).abs().max()) / sc
        flips = int(((got > 0) != (r64 > 0)).sum()), int(((r32 > 0) != (r64 > 0)).sum())
        print("%-42s %10.2e %10.2e %8.1f  %s" % (pfx, e, e32, e / max(e32, 1e-30), flips))
    # pre-activation of the fusion layers (BN input) where ReLU masks are decided
    for seq in ("fusion1.FusionLayer", "fusion2.FusionLayer", "hsi1.fusion.FusionLayer", "hsi2.fusion.FusionLayer"):
        ins64, out64 = c64[seq]
        pre = ws.tensor(seq + ".pre")
        x64 = nhwc(ins64[0])
        print(seq, "input rows", tuple(x64.shape), "pre numel", pre.numel())
    print("loss", float(loss))


if __name__ == "__main__":
    main()
