"""ORACLE — test infrastructure only.  CPU fp32 restatement of the reference ViT-CNN.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import
this module, and only as the checker / the timed CPU baseline.  The product path
(`vit-cnn_amd/vitcnn_amd`) never imports it and has no CPU fallback.

What it restates: the reference's "ViT-CNN (ours)" model, `Multimodality_Mamba`
(`/root/reference/model/Multimodality_Mamba/Mutimodality_Mamba7.py:1141-1181`), in the
reference's own op order and fp32 arithmetic — including the 10-fold duplicated
LayerNorm / in_proj / out_proj of the direction batch and the naive per-timestep
selective scan of the transformers MambaMixer torch fallback
(transformers 5.15.0 `models/mamba/modeling_mamba.py:82-102, 175-283, 359-481`).
It is written functionally over a flat {state_dict name: tensor} mapping so that any
module with the reference's 1704 state_dict keys (the product model included) can be
evaluated by it.

Pinning: `tests/test_oracle_golden.py` checks this restatement against golden vectors
produced by importing the reference itself in the build container
(`tests/golden/gen_golden.py`): logits, loss, every parameter-gradient norm, small full
gradients, per-module activations, post-AdamW parameters, BN running statistics and
eval-mode logits.  One op is pinned only to an inference: `ChannelExchange` comes from
the absent `model/changer.py` (open-cd Changer, p = 1/2).
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F

Tensor = torch.Tensor

LN_EPS = 1e-6      # build_norm_layer(dict(type='LN', eps=1e-6)) — Mutimodality_Mamba7.py:216, :1069, :1073
BN_EPS = 1e-5      # nn.BatchNorm2d defaults
BN_MOMENTUM = 0.1


# ----------------------------------------------------------------------------------------
# scan orders (Mutimodality_Mamba7.py:609-640 for n=9, :788-806 for n=7), restated as rules
# ----------------------------------------------------------------------------------------
def _snake_columns(n):
    out = []
    for c in range(n):
        rows = range(n) if c % 2 == 0 else range(n - 1, -1, -1)
        out += [r * n + c for r in rows]
    return out


def _zigzag_antidiag(n, mirror=False):
    out = []
    for s in range(2 * n - 1):
        rows = [r for r in range(n) if 0 <= s - r < n]
        if s % 2 == 0:
            rows = rows[::-1]
        for r in rows:
            c = s - r
            out.append(r * n + (n - 1 - c if mirror else c))
    return out


def _spiral(n, clockwise=True):
    top, bot, left, right = 0, n - 1, 0, n - 1
    out = []
    while top <= bot and left <= right:
        if clockwise:
            out += [top * n + c for c in range(left, right + 1)]
            out += [r * n + right for r in range(top + 1, bot + 1)]
            if top < bot:
                out += [bot * n + c for c in range(right - 1, left - 1, -1)]
            if left < right:
                out += [r * n + left for r in range(bot - 1, top, -1)]
        else:
            out += [r * n + left for r in range(top, bot + 1)]
            out += [bot * n + c for c in range(left + 1, right + 1)]
            if left < right:
                out += [r * n + right for r in range(bot - 1, top - 1, -1)]
            if top < bot:
                out += [top * n + c for c in range(right - 1, left, -1)]
        top, bot, left, right = top + 1, bot - 1, left + 1, right - 1
    return out


def scan_orders(n):
    """The 10 token orders in gate order hf, hr, vf, vr, 37df, 37dr, 19df, 19dr, ltcw, ltacw
    (Mutimodality_Mamba7.py:653, :699-701)."""
    ident = list(range(n * n))
    vf = _snake_columns(n)
    d37 = _zigzag_antidiag(n)
    d19 = _zigzag_antidiag(n, mirror=True)
    return [ident, ident[::-1], vf, vf[::-1], d37, d37[::-1], d19, d19[::-1], _spiral(n, True), _spiral(n, False)]


# ----------------------------------------------------------------------------------------
# primitive ops
# ----------------------------------------------------------------------------------------
class Params:
    """Flat view of a state_dict: parameters (grad-tracked) plus mutable BN buffers."""

    def __init__(self, tensors: Dict[str, Tensor], training: bool = True):
        self.t = tensors
        self.training = training

    def __getitem__(self, k):
        return self.t[k]


def batchnorm(P: Params, pfx: str, x: Tensor) -> Tensor:
    """nn.BatchNorm2d forward (train: batch stats + running update; eval: running stats)."""
    rm, rv = P[pfx + ".running_mean"], P[pfx + ".running_var"]
    if P.training:
        nbt = P.t.get(pfx + ".num_batches_tracked")
        if nbt is not None:
            nbt.add_(1)
    return F.batch_norm(x, rm, rv, P[pfx + ".weight"], P[pfx + ".bias"], P.training, BN_MOMENTUM, BN_EPS)


def conv2d(P: Params, pfx: str, x: Tensor, bias=True) -> Tensor:
    return F.conv2d(x, P[pfx + ".weight"], P[pfx + ".bias"] if bias else None)


def layernorm(P: Params, pfx: str, x: Tensor) -> Tensor:
    return F.layer_norm(x, (x.shape[-1],), P[pfx + ".weight"], P[pfx + ".bias"], LN_EPS)


def mamba_mixer(P: Params, pfx: str, x: Tensor) -> Tensor:
    """transformers MambaMixer torch fallback (modeling_mamba.py:359-481, scan :175-283).

    x: [n, L, E] -> [n, L, E].  in_proj (no bias) -> causal depthwise conv1d k=4 + SiLU ->
    x_proj -> dt_proj (+bias inside the scan) -> softplus -> sequential selective scan with
    fp32 state -> + D*u -> * SiLU(z) -> out_proj (no bias).
    """
    n, L, _ = x.shape
    w_in = P[pfx + ".in_proj.weight"]
    d_inner = w_in.shape[0] // 2
    xz = (x @ w_in.t()).transpose(1, 2)                                   # [n, 2D, L]
    u, z = xz[:, :d_inner], xz[:, d_inner:]
    cw, cb = P[pfx + ".conv1d.weight"], P[pfx + ".conv1d.bias"]
    u = F.conv1d(u, cw, cb, padding=cw.shape[-1] - 1, groups=d_inner)[..., :L]
    u = F.silu(u)                                                         # [n, D, L]
    w_x = P[pfx + ".x_proj.weight"]
    w_dt = P[pfx + ".dt_proj.weight"]
    rank = w_dt.shape[1]
    nstate = (w_x.shape[0] - rank) // 2
    xdbl = u.transpose(1, 2) @ w_x.t()                                    # [n, L, R+2N]
    ts, Bm, Cm = torch.split(xdbl, [rank, nstate, nstate], dim=-1)
    dt = w_dt @ ts.transpose(1, 2)                                        # [n, D, L]
    dt = F.softplus(dt + P[pfx + ".dt_proj.bias"][:, None])
    A = -torch.exp(P[pfx + ".A_log"])
    dA = torch.exp(A[None, :, None, :] * dt[..., None])                   # [n, D, L, N]
    dBu = dt[..., None] * Bm[:, None, :, :] * u[..., None]
    h = torch.zeros(n, d_inner, nstate, dtype=x.dtype)
    ys = []
    for t in range(L):
        h = dA[:, :, t] * h + dBu[:, :, t]
        ys.append((h @ Cm[:, t, :, None])[..., 0])
    y = torch.stack(ys, dim=-1) + u * P[pfx + ".D"][None, :, None]
    y = y * F.silu(z)
    return y.transpose(1, 2) @ P[pfx + ".out_proj.weight"].t()


def hsi_mamba(P: Params, pfx: str, x: Tensor) -> Tensor:
    """hsiMamba with path '81_2+8' / '49_2+8', out_type 'featmap' (Mutimodality_Mamba7.py:419-1017)."""
    b, _, h, w = x.shape
    tok = F.conv2d(x, P[pfx + ".patch_embed.projection.weight"]).flatten(2).transpose(1, 2)
    tok = tok + P[pfx + ".pos_embed"]
    residual = tok
    orders = [torch.tensor(o) for o in scan_orders(h)]
    seqs = torch.cat([tok[:, o] for o in orders], dim=0)                  # [10B, L, E]
    seqs = layernorm(P, pfx + ".pre_norm", seqs)
    seqs = mamba_mixer(P, pfx + ".layers.0", seqs)
    parts = torch.split(seqs, b, dim=0)
    gate = torch.softmax(P[pfx + ".weights"], dim=1)                      # [1, 10, 1]
    mix = 0
    for k, (o, part) in enumerate(zip(orders, parts)):
        mix = mix + gate[:, k:k + 1] * part[:, torch.argsort(o)]
    tok = layernorm(P, pfx + ".ln1", residual + mix)
    return tok.reshape(b, h, w, -1).permute(0, 3, 1, 2)


def token_learner(P: Params, pfx: str, x: Tensor, S: int) -> Tensor:
    """TokenLearner(S) of SpatialAttention modules (Mutimodality_Mamba7.py:26-64) -> [B, S, C]."""
    mx = x.max(dim=1, keepdim=True)[0]
    avg = x.mean(dim=1, keepdim=True)
    pooled = torch.cat([mx, avg], dim=1)
    toks = []
    for i in range(S):
        t = f"{pfx}.tokenizers.{i}.conv"
        f = F.conv2d(pooled, P[t + ".0.weight"], P[t + ".0.bias"])
        a = torch.sigmoid(F.relu(batchnorm(P, t + ".1", f)))
        toks.append((x * a).mean(dim=(-2, -1)))
    return torch.stack(toks, dim=1)


def non_local(P: Params, pfx: str, x: Tensor, y: Tensor, z: Tensor) -> Tensor:
    """NONLocalBlock2D(sub_sample=True, bn_layer=True) forward(x, y, z) (Mutimodality_Mamba7.py:140-159)."""
    b = x.shape[0]
    theta = conv2d(P, pfx + ".theta", x).flatten(2).transpose(1, 2)       # [B, HW, Ci]
    phi = F.max_pool2d(conv2d(P, pfx + ".phi.0", y), 2).flatten(2)        # [B, Ci, P]
    att = torch.softmax(theta @ phi, dim=-1)                              # no 1/sqrt(d) scaling
    g = F.max_pool2d(conv2d(P, pfx + ".g.0", z), 2).flatten(2).transpose(1, 2)
    o = (att @ g).transpose(1, 2).reshape(b, -1, *x.shape[2:])
    wy = batchnorm(P, pfx + ".W.1", conv2d(P, pfx + ".W.0", o))
    return wy + z


def conv_bn_relu_1x1(P: Params, pfx: str, x: Tensor) -> Tensor:
    """Sequential(Conv2d 1x1, BatchNorm2d, ReLU) — the FusionLayer of GLfusionBlock/fusionBlock."""
    return F.relu(batchnorm(P, pfx + ".1", conv2d(P, pfx + ".0", x)))


def bn_conv3_relu(P: Params, pfx: str, x: Tensor) -> Tensor:
    """ms_conv_bn_relu: BN -> 3x3 valid conv (+bias) -> ReLU (Mutimodality_Mamba7.py:1035-1048)."""
    return F.relu(conv2d(P, pfx + ".conv", batchnorm(P, pfx + ".bn", x)))


def channel_exchange(x1: Tensor, x2: Tensor):
    """Swap every channel c with c % 2 == 0 between x1 and x2 (inferred ChannelExchange, p=1/2)."""
    even = (torch.arange(x1.shape[1]) % 2 == 0).view(1, -1, 1, 1)
    return torch.where(even, x2, x1), torch.where(even, x1, x2)


def fusion(P: Params, pfx: str, x1: Tensor, x2: Tensor) -> Tensor:
    """fusionBlock (Mutimodality_Mamba7.py:1119-1139)."""
    if x1.shape[1] == x2.shape[1]:
        x1, x2 = channel_exchange(x1, x2)
    return conv_bn_relu_1x1(P, pfx + ".FusionLayer", torch.cat([x1, x2], dim=1))


def global_local_block(P: Params, pfx: str, x: Tensor) -> Tensor:
    """GlobalLocalBlock (Mutimodality_Mamba7.py:1050-1091)."""
    b, _, h, _ = x.shape
    s = (h - 2) * (h - 2)
    gv = hsi_mamba(P, pfx + ".global_view", x)
    gf = token_learner(P, pfx + ".global_feature", conv2d(P, pfx + ".change_dim", gv), s)
    gf = layernorm(P, pfx + ".ln3", gf).reshape(b, h - 2, h - 2, -1).permute(0, 3, 1, 2)
    lf = bn_conv3_relu(P, pfx + ".local_feature", x)
    cf = token_learner(P, pfx + ".channel_token", conv2d(P, pfx + ".channel_feature", x), s)
    cf = layernorm(P, pfx + ".ln4", cf).reshape(b, h - 2, h - 2, -1).permute(0, 3, 1, 2)
    # GLfusionBlock(x1=channel, x2=local) (:1107-1117)
    globalf = lf + cf
    localf = non_local(P, pfx + ".FusionLayer.cross_attention", lf, cf, cf) + lf
    fm = conv_bn_relu_1x1(P, pfx + ".FusionLayer.FusionLayer", torch.cat([localf, globalf], dim=1))
    return fusion(P, pfx + ".fusion", gf, fm)


def forward(P: Params, hsi: Tensor, lidar: Tensor) -> Tensor:
    """Multimodality_Mamba.forward (Mutimodality_Mamba7.py:1164-1181) -> logits [B, ncls]."""
    h1 = global_local_block(P, "hsi1", hsi)
    h2 = global_local_block(P, "hsi2", h1)
    l1 = bn_conv3_relu(P, "lidar1", lidar)
    l2 = bn_conv3_relu(P, "lidar2", l1)
    f1 = fusion(P, "fusion1", h1, l1)
    f2 = fusion(P, "fusion2", h2, l2)
    feat = f1.mean(dim=(2, 3)) + f2.mean(dim=(2, 3))
    return feat @ P["classifier.weight"].t() + P["classifier.bias"]


def weighted_ce(logits: Tensor, target: Tensor, weight: Tensor) -> Tensor:
    """nn.CrossEntropyLoss(weight) with reduction='mean' (model_utils.py:311): sum w_y nll / sum w_y."""
    return F.cross_entropy(logits, target, weight=weight)


def ce_class_weights(n_classes: int, ignored=(0,)) -> Tensor:
    """model_utils.py:63-66."""
    w = torch.ones(n_classes)
    w[list(ignored)] = 0.0
    return w


# ----------------------------------------------------------------------------------------
# whole-model helpers used by tests and the CPU baseline
# ----------------------------------------------------------------------------------------
def unused_param_prefixes():
    """hsiMamba owns a TokenLearner + ln3 its forward never calls (Mutimodality_Mamba7.py:361-363)."""
    return ("hsi1.global_view.tokenlearner.", "hsi1.global_view.ln3.",
            "hsi2.global_view.tokenlearner.", "hsi2.global_view.ln3.")


def make_state(state_dict: Dict[str, Tensor], requires_grad=True) -> Dict[str, Tensor]:
    """Detached CPU fp32 copies; float params become leaves that track gradients."""
    out = {}
    for k, v in state_dict.items():
        v = v.detach().to("cpu").clone()
        if v.is_floating_point() and not (k.endswith("running_mean") or k.endswith("running_var")):
            v.requires_grad_(requires_grad)
        out[k] = v
    return out


def param_names(state: Dict[str, Tensor]):
    return [k for k, v in state.items() if v.is_floating_point() and v.requires_grad]


def train_step(state: Dict[str, Tensor], hsi: Tensor, lidar: Tensor, target: Tensor, weight: Tensor,
               opt=None):
    """One reference training iteration (model_utils.py:918-936): zero_grad, forward, CE,
    backward, optimizer step (AdamW lr 8e-4, model_utils.py:309-310), loss.item()."""
    if opt is not None:
        opt.zero_grad()
    P = Params(state, training=True)
    logits = forward(P, hsi, lidar)
    loss = weighted_ce(logits, target, weight)
    loss.backward()
    if opt is not None:
        opt.step()
    return logits.detach(), loss.item()


def make_adamw(state: Dict[str, Tensor], lr=8e-4):
    return torch.optim.AdamW([state[k] for k in param_names(state)], lr=lr)


def gflop_per_patch() -> float:
    """De-duplicated algorithmic work per training patch: 0.5235 GFLOP."""
    return 0.5235
