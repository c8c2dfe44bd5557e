"""ORACLE — test infrastructure only.  CPU fp32 restatement of the reference S2EFT model.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py` may import this module, and only as the
checker; the product path (`vit-cnn_amd/vitcnn_amd/s2eft.py`) never imports it.

Restates `/root/reference/model/compare_method/S2EFT.py` functionally over a {state_dict name:
tensor} mapping, in the reference's op order (dropout only where the caller supplies keep masks,
see `forward`):
  spectral gate            :134-143   mean/max over the last dim, conv1d k7 pad3, sigmoid, `.data` >= 0.4
  embedding                :146-153   Linear(patch_dim -> dim), cls token first, + pos_embedding[:, :n+1]
  Transformer 'CAF'/'ViT'  :92-108    last_output list, skipcat Conv2d(T, T, [1, 2]) from layer 2 on
  Residual(PreNorm(Attention)) :5-19, :45-74   LayerNorm eps 1e-5, qkv no bias, heads x 16, scale 16^-0.5
  Residual(PreNorm(FeedForward)) :21-32        Linear, GELU (erf), Linear
  head                     :155-162   x[:, 0] -> LayerNorm -> Linear
Gradients come from torch autograd over this restatement (the checker's yardstick).

Pinning: `tests/test_oracle_golden.py::test_s2eft_oracle_matches_reference` compares it with
golden vectors made by importing the reference module itself (`tests/golden/gen_s2eft_golden.py`).
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F


def forward(sd: Dict[str, torch.Tensor], x: torch.Tensor, depth: int = 5, heads: int = 4, mode: str = "CAF",
            beta: float = 0.4, drop=None) -> torch.Tensor:
    """drop: optional {site: (keep mask 0/1, p)} applying nn.Dropout's x * mask / (1 - p) at the
    reference's sites -- "emb" (:151), "<layer>.attn" (to_out :43), "<layer>.ff1" / "<layer>.ff2"
    (FeedForward :26, :28) -- with masks supplied by the caller (the checker feeds the HIP path's)."""
    drop = drop or {}

    def dp(site, t):
        if site not in drop:
            return t
        mk, p = drop[site]
        return t * mk.reshape(t.shape) * (1.0 / (1.0 - p))

    b, n, c = x.shape
    avg = x.mean(dim=-1, keepdim=True)
    mx = x.max(dim=-1, keepdim=True)[0]
    g = torch.cat([avg, mx], dim=-1).transpose(1, 2)                     # [b, 2, n]
    g = torch.sigmoid(F.conv1d(g, sd["conv2d.weight"], sd["conv2d.bias"], padding=3)).transpose(1, 2)
    mask = (g.detach() >= beta).to(x.dtype)                               # [b, n, 1], no gradient
    x = x * mask
    x = F.linear(x, sd["patch_to_embedding.weight"], sd["patch_to_embedding.bias"])
    dim = x.shape[-1]
    x = torch.cat([sd["cls_token"].expand(b, 1, dim), x], dim=1)
    x = dp("emb", x + sd["pos_embedding"][:, :n + 1])
    last = []
    for li in range(depth):
        p = f"transformer.layers.{li}"
        if mode == "CAF":
            last.append(x)
            if li > 1:
                z = torch.cat([x.unsqueeze(3), last[li - 2].unsqueeze(3)], dim=3)
                k = f"transformer.skipcat.{li - 2}"
                x = F.conv2d(z, sd[k + ".weight"], sd[k + ".bias"]).squeeze(3)
        y = F.layer_norm(x, (dim,), sd[p + ".0.fn.norm.weight"], sd[p + ".0.fn.norm.bias"], 1e-5)
        qkv = F.linear(y, sd[p + ".0.fn.fn.to_qkv.weight"])
        q, kk, v = (t.reshape(b, n + 1, heads, -1).transpose(1, 2) for t in qkv.chunk(3, dim=-1))
        dh = q.shape[-1]
        att = torch.softmax(torch.einsum("bhid,bhjd->bhij", q, kk) * dh ** -0.5, dim=-1)
        o = torch.einsum("bhij,bhjd->bhid", att, v).transpose(1, 2).reshape(b, n + 1, heads * dh)
        x = dp(f"{li}.attn", F.linear(o, sd[p + ".0.fn.fn.to_out.0.weight"], sd[p + ".0.fn.fn.to_out.0.bias"])) + x
        y = F.layer_norm(x, (dim,), sd[p + ".1.fn.norm.weight"], sd[p + ".1.fn.norm.bias"], 1e-5)
        h = dp(f"{li}.ff1", F.gelu(F.linear(y, sd[p + ".1.fn.fn.net.0.weight"], sd[p + ".1.fn.fn.net.0.bias"])))
        x = dp(f"{li}.ff2", F.linear(h, sd[p + ".1.fn.fn.net.3.weight"], sd[p + ".1.fn.fn.net.3.bias"])) + x
    c0 = F.layer_norm(x[:, 0], (dim,), sd["mlp_head.0.weight"], sd["mlp_head.0.bias"], 1e-5)
    return F.linear(c0, sd["mlp_head.1.weight"], sd["mlp_head.1.bias"])


def train_step(sd: Dict[str, torch.Tensor], x, target, weight, **kw):
    """(logits, weighted-mean CE loss, {name: grad}) for one batch (model_utils.py:918-933)."""
    params = {k: v.detach().clone().requires_grad_(True) for k, v in sd.items()}
    logits = forward(params, x, **kw)
    loss = F.cross_entropy(logits, target, weight=weight)
    loss.backward()
    grads = {k: (p.grad if p.grad is not None else torch.zeros_like(p)) for k, p in params.items()}
    return logits.detach(), loss.detach(), grads
