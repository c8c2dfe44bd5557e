"""TokenLearner gradient stage-by-stage diagnosis.

Runs the DP-test scene's rank batches (tests/test_train_dp_gpu.py `_scene`, PatchBatcher rank r of 2)
through the fused HIP step on cuda:0 and through the float64 yardstick (helpers.masked_oracle_step's
rules: the HIP path's ReLU decisions and pooled values), with every TokenLearner intermediate kept:
dZ (grad of the TokenLearner output), da (grad of the attention map), df (grad of the 2->1 conv
output) and the five per-token parameter gradients.  For each stage it prints the worst tokens'
error against the float64 value, the fp32 CPU reference's own error at the same stage, and the
HIP attn_bwd recomputed in float64 FROM THE HIP path's own da (so an error that enters upstream of
attn_bwd is told apart from one made inside it).

    python tools/tl_grad_diag.py [--ranks 0,1] [--b 4]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "vit-cnn_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from helpers import hash_state_dict, relu_masks_from_workspace, tl_pooled_from_workspace  # noqa: E402
from oracle import vitcnn_oracle as O  # noqa: E402

TLS = ("hsi1.channel_token", "hsi1.global_feature", "hsi2.channel_token", "hsi2.global_feature")


def scene():
    from test_train_dp_gpu import _scene
    return _scene()


def oracle_run(sd, hsi, lidar, target, masks, pooled, dtype):
    """oracle step with TokenLearner intermediates retained; masks/pooled None = the oracle's own."""
    cap = {}
    orig = (O.bn_conv3_relu, O.conv_bn_relu_1x1, O.token_learner, O.layernorm, O.non_local)
    orig_ln = O.layernorm

    def non_local(P, pfx, x, y, z):   # NonLocal intermediates kept (NCHW / [B, HW, Ci] as the oracle has them)
        b = x.shape[0]
        theta = O.conv2d(P, pfx + ".theta", x)
        theta.retain_grad()
        th = theta.flatten(2).transpose(1, 2)
        phi_pre = O.conv2d(P, pfx + ".phi.0", y)
        phi_pre.retain_grad()
        phi = F.max_pool2d(phi_pre, 2).flatten(2)
        s_ = th @ phi
        s_.retain_grad()
        att = torch.softmax(s_, dim=-1)
        g_pre = O.conv2d(P, pfx + ".g.0", z)
        g_pre.retain_grad()
        g = F.max_pool2d(g_pre, 2).flatten(2).transpose(1, 2)
        o = (att @ g).transpose(1, 2).reshape(b, -1, *x.shape[2:])
        o.retain_grad()
        wy = O.batchnorm(P, pfx + ".W.1", O.conv2d(P, pfx + ".W.0", o))
        cap[pfx] = dict(theta=theta, phi_pre=phi_pre, g_pre=g_pre, o=o, s=s_, att=att, sv=s_, gpv=g_pre, ppv=phi_pre)
        return wy + z

    def layernorm(P, pfx, x):   # ln3 / ln4: keep the LayerNorm's input and output gradients
        y = orig_ln(P, pfx, x)
        if pfx.endswith(".ln3") or pfx.endswith(".ln4"):
            x.retain_grad()
            y.retain_grad()
            cap[pfx] = dict(x=x, y=y)
        return y

    def bn_conv3(P, pfx, x):
        pre = O.conv2d(P, pfx + ".conv", O.batchnorm(P, pfx + ".bn", x))
        return pre * masks[pfx].to(pre.dtype) if masks and pfx in masks else torch.relu(pre)

    def conv1x1(P, pfx, x):
        if pfx.endswith("FusionLayer.FusionLayer"):
            x.retain_grad()
            cap[pfx] = dict(cat=x)
        pre = O.batchnorm(P, pfx + ".1", O.conv2d(P, pfx + ".0", x))
        return pre * masks[pfx].to(pre.dtype) if masks and pfx in masks else torch.relu(pre)

    def token_learner(P, pfx, x, S):
        if pooled is not None:
            mx_h, amx_h, avg_h = (t.to(x.dtype) if t.is_floating_point() else t for t in pooled[pfx])
            g = torch.gather(x, 1, amx_h)
            m = x.mean(dim=1, keepdim=True)
            pool = torch.cat([mx_h + (g - g.detach()), avg_h + (m - m.detach())], dim=1)
        else:
            pool = torch.cat([x.max(dim=1, keepdim=True)[0], x.mean(dim=1, keepdim=True)], dim=1)
        toks, fs, As = [], [], []
        for i in range(S):
            t = f"{pfx}.tokenizers.{i}.conv"
            f = F.conv2d(pool, P[t + ".0.weight"], P[t + ".0.bias"])
            f.retain_grad()
            pre = O.batchnorm(P, t + ".1", f)
            a = torch.sigmoid(pre * masks[pfx][:, i:i + 1].to(pre.dtype) if masks else torch.relu(pre))
            a.retain_grad()
            fs.append(f)
            As.append(a)
            toks.append((x * a).mean(dim=(-2, -1)))
        Z = torch.stack(toks, dim=1)
        Z.retain_grad()
        cap[pfx] = dict(Z=Z, f=fs, a=As, x=x)
        return Z

    O.bn_conv3_relu, O.conv_bn_relu_1x1, O.token_learner, O.layernorm, O.non_local = (bn_conv3, conv1x1, token_learner,
                                                                                      layernorm, non_local)
    try:
        sdd = {k: (v.to(dtype) if v.is_floating_point() else v) for k, v in sd.items()}
        st = O.make_state(sdd)
        w = O.ce_class_weights(16).to(dtype)
        O.train_step(st, hsi.to(dtype), lidar.to(dtype), target, w)
    finally:
        O.bn_conv3_relu, O.conv_bn_relu_1x1, O.token_learner, O.layernorm, O.non_local = orig
    out = {}
    for pfx, c in cap.items():
        if "theta" in c or "cat" in c:
            out[pfx] = {k: (v.grad.detach().double() if k not in ("att", "sv", "gpv", "ppv") else v.detach().double()) for k, v in c.items()}
            continue
        if "f" not in c:
            out[pfx] = dict(lnx=c["x"].detach().double(), dlnx=c["x"].grad.detach().double(),
                            dlny=c["y"].grad.detach().double())
            continue
        S = len(c["f"])
        out[pfx] = dict(dZ=c["Z"].grad.detach().double(),                                  # [B,S,C]
                        da=torch.cat([a.grad for a in c["a"]], 1).detach().double(),       # [B,S,H,W]
                        df=torch.cat([f.grad for f in c["f"]], 1).detach().double(),       # [B,S,H,W]
                        x=c["x"].detach().double())
        out[pfx]["S"] = S
    grads = {k: st[k].grad.detach().double() for k in O.param_names(st) if st[k].grad is not None}
    return out, grads


def hip_attn_bwd64(mx, avg, par, stats, da, S, B, HW):
    """attn_bwd (csrc/tokenlearner.hip:197-277) in float64 from the HIP path's own inputs."""
    n = B * HW
    da = da.view(B, S, HW).permute(1, 0, 2).reshape(S, n)
    par = par.view(S, 5)
    w0, w1, bc, gam, bet = (par[:, j:j + 1] for j in range(5))
    mean, invstd = stats[0::2, None], stats[1::2, None]
    f = w0 * mx[None] + w1 * avg[None] + bc
    xh = (f - mean) * invstd
    bn = xh * gam + bet
    sg = torch.sigmoid(bn)
    g1 = torch.where(bn > 0, da * sg * (1 - sg), torch.zeros_like(da))
    s1, s2 = g1.sum(1, keepdim=True), (g1 * xh).sum(1, keepdim=True)
    d = gam * invstd * (g1 - s1 / n - xh * s2 / n)
    gw0, gw1, gb = (d * mx[None]).sum(1), (d * avg[None]).sum(1), d.sum(1)
    return d, torch.stack([gw0, gw1, gb, s2[:, 0], s1[:, 0]], 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="0,1")
    ap.add_argument("--b", type=int, default=4)
    ap.add_argument("--top", type=int, default=4)
    args = ap.parse_args()
    from vitcnn_amd import fused_train_step
    from vitcnn_amd import model_utils as mu
    from vitcnn_amd.window import PatchBatcher
    dev = torch.device("cuda", 0)
    B = args.b
    sd = hash_state_dict()
    model, opt, crit, hp = mu.get_model("Multimodality_Mamba", n_classes=16, n_bands=(144, 1), ignored_labels=[0],
                                        dataset="synthetic", device=dev)
    img1, img2, gt = scene()
    for rank in (int(r) for r in args.ranks.split(",")):
        loader = PatchBatcher(img1, img2, gt, 9, ignored_labels=[0], batch_size=B, device=dev, seed=5, rank=rank,
                              world=2)
        x1, x2, t = next(iter(loader))
        model.load_state_dict(sd)
        model.zero_grad(set_to_none=True)
        fused_train_step(model, crit, x1, x2, t)
        torch.cuda.synchronize()
        g = model.flat_params.grad.detach().double().cpu()
        masks = relu_masks_from_workspace(model, B)
        pooled = tl_pooled_from_workspace(model, B)
        ws = next(v for k, v in model._ws.items() if k[2][0] == "train")
        hsi, lidar, tt = x1.cpu(), x2.cpu(), t.cpu()
        y64, g64 = oracle_run(sd, hsi, lidar, tt, masks, pooled, torch.float64)
        y32, g32 = oracle_run(sd, hsi, lidar, tt, None, None, torch.float32)
        o64, go64 = oracle_run(sd, hsi, lidar, tt, None, None, torch.float64)
        print(f"=== rank {rank} batch targets {tt.tolist()}")
        for blk, H in (("hsi1", 9), ("hsi2", 7)):
            Hs = H - 2
            S = Hs * Hs
            C = model.hsi1.cout if blk == "hsi1" else model.hsi2.cout
            Ci = C // 2
            M = B * S
            nl = y64[blk + ".FusionLayer.cross_attention"]
            cat = y64[blk + ".FusionLayer.FusionLayer"]["cat"]
            cl = lambda t: t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])   # noqa: E731  NCHW -> rows x C
            def rep(name, hip, ref):
                e = (hip - ref).abs().max(1).values
                w = int(torch.argmax(e))
                print(f"   {blk} {name}: err {float(e.max()):.3e} (|ref| {float(ref.abs().max()):.3e}) worst row {w} "
                      f"(b {w // S}, s {w % S})")
            rep("dCAT1 local half", ws.tensor(blk + ".dCAT1")[:M * 2 * C].view(M, 2 * C)[:, :C].double().cpu(), cl(cat)[:, :C])
            rep("dCAT1 global half", ws.tensor(blk + ".dCAT1")[:M * 2 * C].view(M, 2 * C)[:, C:].double().cpu(), cl(cat)[:, C:])
            dpg = ws.tensor(blk + ".dPG")[:M * 2 * Ci].view(M, 2 * Ci).double().cpu()
            rep("dphi (pre-pool)", dpg[:, :Ci], cl(nl["phi_pre"]))
            rep("dg (pre-pool)", dpg[:, Ci:], cl(nl["g_pre"]))
            rep("dtheta", ws.tensor(blk + ".dTH")[:M * Ci].view(M, Ci).double().cpu(), cl(nl["theta"]))
            rep("dO", ws.tensor(blk + ".dO")[:M * Ci].view(M, Ci).double().cpu(), cl(nl["o"]))
            Pk = (Hs // 2) ** 2
            att_h = ws.tensor(blk + ".ATT")[:M * Pk].view(M, Pk).double().cpu()
            rep("att (fwd)", att_h, nl["att"].reshape(M, Pk))
            print(f"   {blk} scores: max |s| {float(nl['sv'].abs().max()):.3e}; att max {float(nl['att'].max()):.4f}")
            # max-pool decisions: HIP taps vs the float64 argmax, and how close the two candidates are
            pa = ws.tensor(blk + ".PA")[:B * Pk * 2 * Ci].view(B, Pk, 2 * Ci).cpu().long()
            pgh = ws.tensor(blk + ".PG")[:M * 2 * Ci].view(B, Hs, Hs, 2 * Ci).double().cpu()
            for name, pre, off in (("phi", nl["ppv"], 0), ("g", nl["gpv"], Ci)):
                ph = Hs // 2
                win = pre[:, :, :2 * ph, :2 * ph].reshape(B, Ci, ph, 2, ph, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, Ci, ph, ph, 4)
                t64 = win.argmax(-1)                                   # first max, like the kernels
                th = pa[:, :, off:off + Ci].transpose(1, 2).reshape(B, Ci, ph, ph)
                diff = (t64 != th).nonzero()
                print(f"   {blk} pool {name}: {len(diff)} of {th.numel()} windows choose a different tap than float64")
                for d in diff[:4].tolist():
                    bb, cc, i, j = d
                    w64 = win[bb, cc, i, j]
                    hw = pgh[bb, 2 * i:2 * i + 2, 2 * j:2 * j + 2, off + cc].reshape(4)
                    print(f"      b {bb} ch {cc} win ({i},{j}): f64 {w64.tolist()} -> tap {int(t64[bb, cc, i, j])}; "
                          f"HIP {hw.tolist()} -> tap {int(th[bb, cc, i, j])}")
        for pfx in TLS:
            blk = pfx.split(".")[0]
            H = 9 if blk == "hsi1" else 7
            HW, S = H * H, (H - 2) ** 2
            C = model.hsi1.cout if blk == "hsi1" else model.hsi2.cout
            dzname = blk + (".dZc" if "channel" in pfx else ".dZg")
            dZh = ws.tensor(dzname)[:B * S * C].view(B, S, C).double().cpu()
            dah = ws.tensor(pfx + ".da")[:B * S * HW].view(B, S, HW).double().cpu()
            dfh = ws.tensor(pfx + ".df")[:S * B * HW].view(S, B * HW).double().cpu() if pfx + ".df" in ws.t else None
            mx = ws.tensor(pfx + ".mx")[:B * HW].double().cpu()
            avg = ws.tensor(pfx + ".avg")[:B * HW].double().cpu()
            stats = ws.tensor(pfx + ".st")[:2 * S].double().cpu()
            off = model._poff[pfx + ".tokenizers.0.conv.0.weight"]
            par = model.flat_params.detach()[off:off + 5 * S].double().cpu()
            gh = g[off:off + 5 * S].view(S, 5)
            Y, Y32, Yo = y64[pfx], y32[pfx], o64[pfx]
            da64 = Y["da"].view(B, S, HW)
            df64 = Y["df"].view(B, S, HW).permute(1, 0, 2).reshape(S, B * HW)
            d_re, gp_re = hip_attn_bwd64(mx, avg, par, stats, dah, S, B, HW)
            g64t = torch.stack([torch.cat([g64[f"{pfx}.tokenizers.{s}.conv.0.weight"].reshape(-1),
                                           g64[f"{pfx}.tokenizers.{s}.conv.0.bias"].reshape(-1),
                                           g64[f"{pfx}.tokenizers.{s}.conv.1.weight"].reshape(-1),
                                           g64[f"{pfx}.tokenizers.{s}.conv.1.bias"].reshape(-1)]) for s in range(S)])
            g32t = torch.stack([torch.cat([g32[f"{pfx}.tokenizers.{s}.conv.{j}.{w}"].reshape(-1)
                                           for j, w in ((0, "weight"), (0, "bias"), (1, "weight"), (1, "bias"))])
                                for s in range(S)])
            go64t = torch.stack([torch.cat([go64[f"{pfx}.tokenizers.{s}.conv.{j}.{w}"].reshape(-1)
                                            for j, w in ((0, "weight"), (0, "bias"), (1, "weight"), (1, "bias"))])
                                 for s in range(S)])
            gmax = max(float(v.abs().max()) for v in g64.values())
            err_tok = (gh - g64t).abs().max(1).values
            worst = torch.argsort(err_tok, descending=True)[:args.top]
            print(f"-- {pfx}: S={S} gmax={gmax:.3e}; dZ err {float((dZh - Y['dZ']).abs().max()):.3e} "
                  f"(ref32 {float((Y32['dZ'].double() - Yo['dZ']).abs().max()):.3e}, |dZ| {float(Y['dZ'].abs().max()):.3e})")
            lnp = blk + (".ln4" if "channel" in pfx else ".ln3")
            lnY = y64[lnp]
            dyname = blk + (".dFc" if "channel" in pfx else ".dFg")
            dFh = ws.tensor(dyname)[:B * S * C].view(B * S, C).double().cpu()
            Zh = ws.tensor(pfx + ".Z")[:B * S * C].view(B * S, C).double().cpu()
            dFr = lnY["dlny"].reshape(B * S, C)
            Zr = lnY["lnx"].reshape(B * S, C)
            # LayerNorm backward in float64 from the HIP path's own dy and x
            w_ln = model.flat_params.detach()[model._poff[lnp + ".weight"]:model._poff[lnp + ".weight"] + C].double().cpu()
            mu = Zh.mean(1, keepdim=True)
            var = Zh.var(1, unbiased=False, keepdim=True)
            rs = 1.0 / torch.sqrt(var + 1e-6)
            xh = (Zh - mu) * rs
            gg = dFh * w_ln
            dZre = rs * (gg - gg.mean(1, keepdim=True) - xh * (gg * xh).mean(1, keepdim=True))
            rowerr = (dZh.reshape(B * S, C) - Y["dZ"].reshape(B * S, C)).abs().max(1).values
            wr = int(torch.argmax(rowerr))
            print(f"   LN {lnp}: dy err {float((dFh - dFr).abs().max()):.3e} (|dy| {float(dFr.abs().max()):.3e}); "
                  f"x err {float((Zh - Zr).abs().max()):.3e} (|x| {float(Zr.abs().max()):.3e}); "
                  f"dx(HIP) vs f64-LN-bwd(HIP dy, x) {float((dZh.reshape(B * S, C) - dZre).abs().max()):.3e}; "
                  f"worst dZ row {wr} (b {wr // S}, s {wr % S}) err {float(rowerr[wr]):.3e}, row std/|mean| "
                  f"{float(Zh[wr].std() / Zh[wr].mean().abs()):.3e}, rstd {float(rs[wr]):.3e}")
            for s in worst.tolist():
                ea = float((dah[:, s] - da64[:, s]).abs().max())
                ea32 = float((Y32["da"].view(B, S, HW)[:, s].double() - Yo["da"].view(B, S, HW)[:, s]).abs().max())
                ef = float((dfh[s] - df64[s]).abs().max()) if dfh is not None else float("nan")
                ef_re = float((d_re[s] - df64[s]).abs().max())
                sd_std = float(1.0 / stats[2 * s + 1])
                print(f"   tok {s:2d}: param err {float(err_tok[s]):.3e} (ref32 {float((g32t[s].double() - go64t[s]).abs().max()):.3e}) "
                      f"|g| {float(g64t[s].abs().max()):.3e}; da err {ea:.3e} (ref32 {ea32:.3e}, |da| {float(da64[:, s].abs().max()):.3e}); "
                      f"df err {ef:.3e} (recomputed from HIP da {ef_re:.3e}, |df| {float(df64[s].abs().max()):.3e}); "
                      f"bn std {sd_std:.3e}")
                print(f"           HIP gpar {gh[s].tolist()}\n           re(HIP da) {gp_re[s].tolist()}\n"
                      f"           f64 {g64t[s].tolist()}")


if __name__ == "__main__":
    main()
