"""Shared test helpers: hash-filled state dicts keyed by the reference's 1704 state_dict names."""
import json
import os

import numpy as np
import torch

from vitcnn_amd.hashinit import param_fill, synthetic_batch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def reference_keys():
    with open(os.path.join(GOLDEN, "state_dict_keys.json")) as f:
        return json.load(f)


def is_buffer(name):
    return name.endswith("running_mean") or name.endswith("running_var") or name.endswith("num_batches_tracked")


def hash_state_dict():
    """state_dict with every parameter from param_fill and BN buffers at their torch defaults."""
    sd = {}
    for e in reference_keys():
        n, shape = e["name"], tuple(e["shape"])
        if n.endswith("running_mean"):
            sd[n] = torch.zeros(shape)
        elif n.endswith("running_var"):
            sd[n] = torch.ones(shape)
        elif n.endswith("num_batches_tracked"):
            sd[n] = torch.zeros(shape, dtype=torch.int64)
        else:
            sd[n] = torch.from_numpy(param_fill(n, shape))
    return sd


def golden_batch(tag, batch):
    hsi, lidar, target = synthetic_batch(tag, batch, 144, 1, 9, 16)
    return torch.from_numpy(hsi), torch.from_numpy(lidar), torch.from_numpy(target)


def load_npz(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def relu_masks_from_workspace(model, B):
    """The HIP path's ReLU decisions for every conv3x3 / 1x1-fusion layer, as NCHW bool masks keyed by
    the oracle prefix (read from the saved channels-last post-ReLU activations `<pfx>.out`)."""
    ws = next(v for k, v in model._ws.items() if k[2][0] == "train")
    P = model.patch
    masks = {}

    def nchw(name, H, C):
        return ws.tensor(name)[: B * H * H * C].view(B, H, H, C).permute(0, 3, 1, 2).cpu()

    def grab(pfx, H, C):
        t = nchw(pfx + ".out", H, C)
        masks[pfx] = t > 0
        masks[pfx + "#out"] = t   # the HIP post-ReLU values (decision audit: the tensor's measured fp32 error)

    for blk, H, cout in (("hsi1", P, model.hsi1.cout), ("hsi2", P - 2, model.hsi2.cout)):
        S = H - 2
        grab(blk + ".local_feature", S, cout)
        grab(blk + ".FusionLayer.FusionLayer", S, cout)
        grab(blk + ".fusion.FusionLayer", S, cout)
    # TokenLearner BN(1) ReLUs: recomputed by the HIP path's own expression (vc_tl_relu_mask)
    from vitcnn_amd._lib import lib
    params = model._ptrs()[1]
    for blk, H, cout in (("hsi1", P, model.hsi1.cout), ("hsi2", P - 2, model.hsi2.cout)):
        S, HW = (H - 2) ** 2, H * H
        for tl in (".global_feature", ".channel_token"):
            pfx = blk + tl
            mask = torch.empty(B * S * HW, dtype=torch.uint8, device=ws.device)
            lib().vc_tl_relu_mask(B, HW, S, ws.tensor(pfx + ".mx").data_ptr(), ws.tensor(pfx + ".avg").data_ptr(),
                                  params[pfx + ".tokenizers.0.conv.0.weight"], ws.tensor(pfx + ".st").data_ptr(),
                                  mask.data_ptr(), torch.cuda.current_stream().cuda_stream)
            masks[pfx] = mask.view(B, S, H, H).cpu().bool()
            # the TokenLearner's HIP input (change_dim / channel_feature output) for the pooled-value audit
            masks[pfx + "#x"] = nchw(blk + (".CD" if tl == ".global_feature" else ".CF"), H, cout)
    grab("lidar1", P - 2, 16)
    grab("lidar2", P - 4, 32)
    grab("fusion1.FusionLayer", P - 2, 128)
    grab("fusion2.FusionLayer", P - 4, 128)
    # NonLocal 2x2 max-pool decisions of the phi | g maps (the winning tap of each window, [B, Pk, 2 Ci]):
    # windows whose values tie to within fp32 rounding are decisions, like the ReLU ties above (DESIGN.md s. 6)
    for blk, H, cout in (("hsi1", P, model.hsi1.cout), ("hsi2", P - 2, model.hsi2.cout)):
        Hs, Ci = H - 2, cout // 2
        Pk = (Hs // 2) ** 2
        pa = ws.tensor(blk + ".PA")[: B * Pk * 2 * Ci].view(B, Pk, 2 * Ci).cpu().long()
        masks[blk + ".FusionLayer.cross_attention.pool"] = pa
        masks[blk + ".FusionLayer.cross_attention.pool#val"] = ws.tensor(blk + ".PP")[: B * Pk * 2 * Ci].view(
            B, Pk, 2 * Ci).cpu()
    return masks


def tl_pooled_from_workspace(model, B):
    """The HIP path's TokenLearner pooled inputs per TokenLearner prefix: (channel max [B,1,H,H]
    float64, its channel index [B,1,H,H] int64, channel mean [B,1,H,H] float64), read from the
    saved `<pfx>.mx / .amx / .avg` rows of the training workspace."""
    ws = next(v for k, v in model._ws.items() if k[2][0] == "train")
    P = model.patch
    out = {}
    for blk, H in (("hsi1", P), ("hsi2", P - 2)):
        n = B * H * H
        for tl in (".global_feature", ".channel_token"):
            pfx = blk + tl
            mx = ws.tensor(pfx + ".mx")[:n].view(B, 1, H, H).cpu().double()
            amx = ws.tensor(pfx + ".amx")[:n].view(B, 1, H, H).cpu().long()
            avg = ws.tensor(pfx + ".avg")[:n].view(B, 1, H, H).cpu().double()
            out[pfx] = (mx, amx, avg)
    return out


EPS32 = float(np.finfo(np.float32).eps)
TIE_ULPS = 16   # a decision may differ from float64's only within this many fp32 ulps of the decision's scale


def _audit_relu(audit, site, pre, mask, out=None, kind="relu"):
    """One ReLU site: where the HIP decision `mask` differs from float64's (pre > 0), |pre| must be a near-tie --
    within TIE_ULPS ulps of the tensor's largest |pre|, or within 2x the HIP values' own measured deviation from
    float64 on that tensor (max |out - pre| over the elements both call positive)."""
    p = pre.detach()
    m = mask.to(torch.bool).expand_as(p)
    d = (p > 0) != m
    tie = TIE_ULPS * EPS32 * float(p.abs().max())
    e_obs = 0.0
    if out is not None:
        both = (p > 0) & m
        if bool(both.any()):
            e_obs = float((out.double() - p)[both].abs().max())
    tol = max(tie, 2.0 * e_obs)
    dist = float(p[d].abs().max()) if bool(d.any()) else 0.0
    audit.append(dict(site=site, kind=kind, n=p.numel(), disagree=int(d.sum()), dist=dist, tie=tie, e_obs=e_obs,
                      worst=dist / tol if tol > 0 else (0.0 if dist == 0 else float("inf")),
                      worst_ulp=dist / tie if tie > 0 else 0.0))


def _audit_pool(audit, site, pre, taps, vals=None):
    """One 2x2 max pool: where the HIP winning tap differs from float64's argmax (and is not an exact float64
    tie), the window's top-2 gap must be within TIE_ULPS ulps of the window maximum (or 2x the HIP pooled
    values' measured deviation from the float64 pooled values)."""
    b, c, h, w = pre.shape
    ph, pw = h // 2, w // 2
    win = pre.detach()[:, :, :2 * ph, :2 * pw].reshape(b, c, ph, 2, pw, 2).permute(0, 1, 2, 4, 3, 5).reshape(
        b, c, ph, pw, 4)
    t = taps.transpose(1, 2).reshape(b, c, ph, pw, 1)
    got = torch.gather(win, 4, t)[..., 0]
    best = win.max(dim=4).values
    gap = best - got
    d = gap > 0
    e_obs = 0.0
    if vals is not None:
        e_obs = float((vals.transpose(1, 2).reshape(b, c, ph, pw).double() - got).abs().max())
    tie = TIE_ULPS * EPS32 * best.abs()
    tol = torch.clamp(tie, min=2.0 * e_obs)
    ratio = float((gap[d] / tol[d]).max()) if bool(d.any()) else 0.0
    ratio_ulp = float((gap[d] / tie[d]).max()) if bool(d.any()) else 0.0
    audit.append(dict(site=site, kind="maxpool", n=best.numel(), disagree=int(d.sum()),
                      dist=float(gap[d].max()) if bool(d.any()) else 0.0, e_obs=e_obs, worst=ratio,
                      worst_ulp=ratio_ulp))


def _audit_tl_pool(audit, site, x, pooled, x_hip=None):
    """The TokenLearner pooled values the yardstick adopts from the HIP path: max / mean per pixel within the
    HIP input's own deviation from float64 (max is 1-Lipschitz in the sup norm; the mean adds its fp32 sum's
    rounding), and the HIP argmax channel a near-maximum of the float64 row."""
    mx_h, amx_h, avg_h = pooled
    x = x.detach()
    ex = (x_hip.double() - x).abs().max(dim=1, keepdim=True).values if x_hip is not None else torch.zeros_like(mx_h)
    xs = x.abs().max(dim=1, keepdim=True).values
    mx64 = x.max(dim=1, keepdim=True).values
    mean64 = x.mean(dim=1, keepdim=True)
    tol_max = ex + 2 * EPS32 * xs
    tol_mean = ex + TIE_ULPS * EPS32 * xs
    r_max = float(((mx_h - mx64).abs() / tol_max).max())
    r_mean = float(((avg_h - mean64).abs() / tol_mean).max())
    at = torch.gather(x, 1, amx_h)
    d = at < mx64
    r_arg = float(((mx64 - at)[d] / (2 * tol_max[d])).max()) if bool(d.any()) else 0.0
    rel = float(torch.cat([((mx_h - mx64).abs() / xs).flatten(), ((avg_h - mean64).abs() / xs).flatten()]).max())
    audit.append(dict(site=site, kind="tl_pool", n=mx_h.numel(), disagree=int(d.sum()), rel=rel,
                      worst=max(r_max, r_mean, r_arg)))


def audit_summary(audit):
    """{kind: [sites, decisions, disagreements, worst ratio to the tie bound, worst ratio to TIE_ULPS ulps alone]}
    + the failing records"""
    out = {}
    for r in audit:
        k = out.setdefault(r["kind"], [0, 0, 0, 0.0, 0.0])
        k[0] += 1
        k[1] += r["n"]
        k[2] += r["disagree"]
        k[3] = max(k[3], r["worst"])
        k[4] = max(k[4], r.get("worst_ulp", 0.0))
    return out, [r for r in audit if not r["worst"] <= 1.0]


def check_audit(audit, name):
    """assert every adopted HIP decision is a genuine fp32 near-tie; print the counts (and write them to
    gpurun_out/decision_audit_<name>.json when that directory exists)"""
    import json
    summary, bad = audit_summary(audit)
    print(f"decision audit {name}: " + ", ".join(f"{k}: {v[2]} of {v[1]} differ from float64 over {v[0]} sites "
                                                 f"(worst {v[3]:.3g} of the tie bound, {v[4]:.3g} of {TIE_ULPS} ulps)"
                                                 for k, v in summary.items()))
    if os.path.isdir("gpurun_out"):
        with open(f"gpurun_out/decision_audit_{name}.json", "w") as f:
            json.dump({"summary": summary, "records": audit}, f, indent=1)
    assert summary, "no decision was audited"
    assert not bad, bad[:5]
    return summary


def masked_oracle_step(O, state, hsi, lidar, target, weight, masks, pooled=None, audit=None):
    """oracle train step in which the conv/fusion ReLUs use the given masks (pre * mask) instead of
    their own sign test, and the NonLocal 2x2 max pools the given winning taps (`<prefix>.pool` entries).  A pre-activation within rounding distance of zero is an fp32 tie that the
    HIP path and the CPU reference may resolve differently; evaluating the float64 yardstick with the
    HIP path's decisions keeps such a tie from being scored as a gradient error.

    `pooled` ({prefix: (max, argmax, mean)} from tl_pooled_from_workspace): TokenLearner BN(1)
    normalises a 2->1 conv of the pooled channel max / mean whose spread is a tiny fraction of its
    mean, so the fp32 rounding of the pooled values is amplified by 1/std.  The yardstick then takes
    the HIP path's pooled VALUES (gradients still flow to the argmax channel and to every channel
    through the mean, exactly as in the reference).

    `audit` (a list): every adopted decision is also compared with the float64 decision at the same site and
    a record appended (helpers._audit_*: where the two differ, the float64 values must be a near-tie);
    check_audit asserts them (the yardstick may not absorb a non-tie decision)."""
    orig = (O.bn_conv3_relu, O.conv_bn_relu_1x1, O.token_learner, O.non_local)
    F = torch.nn.functional

    def pool_taps(pre, taps):
        """2x2 / stride-2 max pool of pre [B, C, H, W] with the given winning taps [B, Pk, C] (t = 2 dh + dw)"""
        b, c, h, w = pre.shape
        ph, pw = h // 2, w // 2
        win = pre[:, :, :2 * ph, :2 * pw].reshape(b, c, ph, 2, pw, 2).permute(0, 1, 2, 4, 3, 5).reshape(b, c, ph, pw, 4)
        idx = taps.transpose(1, 2).reshape(b, c, ph, pw, 1)
        return torch.gather(win, 4, idx)[..., 0]

    def non_local(P, pfx, x, y, z):   # oracle non_local (:140-159) with the HIP path's max-pool decisions
        key = pfx + ".pool"
        if key not in masks:
            return orig[3](P, pfx, x, y, z)
        b = x.shape[0]
        taps = masks[key]
        ci = taps.shape[2] // 2
        theta = O.conv2d(P, pfx + ".theta", x).flatten(2).transpose(1, 2)
        phi_pre, g_pre = O.conv2d(P, pfx + ".phi.0", y), O.conv2d(P, pfx + ".g.0", z)
        if audit is not None:
            vals = masks.get(key + "#val")
            _audit_pool(audit, key + ".phi", phi_pre, taps[:, :, :ci], None if vals is None else vals[:, :, :ci])
            _audit_pool(audit, key + ".g", g_pre, taps[:, :, ci:], None if vals is None else vals[:, :, ci:])
        phi = pool_taps(phi_pre, taps[:, :, :ci]).flatten(2)
        att = torch.softmax(theta @ phi, dim=-1)
        g = pool_taps(g_pre, taps[:, :, ci:]).flatten(2).transpose(1, 2)
        o = (att @ g).transpose(1, 2).reshape(b, -1, *x.shape[2:])
        wy = O.batchnorm(P, pfx + ".W.1", O.conv2d(P, pfx + ".W.0", o))
        return wy + z

    def bn_conv3(P, pfx, x):
        pre = O.conv2d(P, pfx + ".conv", O.batchnorm(P, pfx + ".bn", x))
        if audit is not None and pfx in masks:
            _audit_relu(audit, pfx, pre, masks[pfx], masks.get(pfx + "#out"))
        return pre * masks[pfx].to(pre.dtype) if pfx in masks else torch.relu(pre)

    def conv1x1(P, pfx, x):
        pre = O.batchnorm(P, pfx + ".1", O.conv2d(P, pfx + ".0", x))
        if audit is not None and pfx in masks:
            _audit_relu(audit, pfx, pre, masks[pfx], masks.get(pfx + "#out"))
        return pre * masks[pfx].to(pre.dtype) if pfx in masks else torch.relu(pre)

    def token_learner(P, pfx, x, S):   # oracle token_learner with the HIP path's decisions / pooling
        given = pooled is not None and pfx in pooled
        if pfx not in masks and not given:
            return orig[2](P, pfx, x, S)
        if given:
            mx_h, amx_h, avg_h = (t.to(x.dtype) if t.is_floating_point() else t for t in pooled[pfx])
            if audit is not None:
                _audit_tl_pool(audit, pfx, x, (mx_h, amx_h, avg_h), masks.get(pfx + "#x"))
            g = torch.gather(x, 1, amx_h)
            m = x.mean(dim=1, keepdim=True)
            pool = torch.cat([mx_h + (g - g.detach()), avg_h + (m - m.detach())], dim=1)
        else:
            pool = torch.cat([x.max(dim=1, keepdim=True)[0], x.mean(dim=1, keepdim=True)], dim=1)
        toks = []
        for i in range(S):
            t = f"{pfx}.tokenizers.{i}.conv"
            f = F.conv2d(pool, P[t + ".0.weight"], P[t + ".0.bias"])
            pre = O.batchnorm(P, t + ".1", f)
            if audit is not None and pfx in masks:
                _audit_relu(audit, f"{pfx}.tokenizers.{i}", pre, masks[pfx][:, i:i + 1], kind="tl_relu")
            a = torch.sigmoid(pre * masks[pfx][:, i:i + 1].to(pre.dtype) if pfx in masks else torch.relu(pre))
            toks.append((x * a).mean(dim=(-2, -1)))
        return torch.stack(toks, dim=1)

    O.bn_conv3_relu, O.conv_bn_relu_1x1, O.token_learner, O.non_local = bn_conv3, conv1x1, token_learner, non_local
    try:
        return O.train_step(state, hsi, lidar, target, weight)
    finally:
        O.bn_conv3_relu, O.conv_bn_relu_1x1, O.token_learner, O.non_local = orig
