"""Parameter holders that reproduce the reference's module tree and state_dict names.

These classes carry parameters and BatchNorm buffers only; they have no forward.  The
tree (attribute names, registration order, shapes, default initialisation) follows the
reference so that `state_dict()` has the reference's 1704 keys and `.pth` checkpoints
interchange in both directions (model_utils.py:1047-1064, main.py:472-473):

  Multimodality_Mamba            Mutimodality_Mamba7.py:1141-1160
  GlobalLocalBlock               :1050-1076
  hsiMamba ('globalview1/2')     :176-363   (+ mmcv PatchEmbed projection, transformers MambaMixer)
  TokenLearner / SpatialAttention :26-64
  NONLocalBlock2D                :66-173
  GLfusionBlock / fusionBlock    :1093-1139
  ms_conv_bn_relu                :1035-1048
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn


class SpatialAttentionParams(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv = nn.Sequential(nn.Conv2d(2, 1, kernel_size=1), nn.BatchNorm2d(1), nn.ReLU())


class TokenLearnerParams(nn.Module):
    def __init__(self, S: int):
        super().__init__()
        self.S = S
        self.tokenizers = nn.ModuleList([SpatialAttentionParams() for _ in range(S)])


class PatchEmbedParams(nn.Module):
    """mmcv PatchEmbed(conv_type='Conv2d', kernel 1, stride 1, bias=False) -> `projection`."""

    def __init__(self, cin: int, embed: int):
        super().__init__()
        self.projection = nn.Conv2d(cin, embed, kernel_size=1, stride=1, bias=False)


class MambaMixerParams(nn.Module):
    """transformers MambaMixer parameters (modeling_mamba.py:294-343), config of
    Mutimodality_Mamba7.py:314-323: state 16, conv 4, dt_rank ceil(E/16), conv bias, no linear bias."""

    def __init__(self, hidden: int, inner: int, state: int = 16, conv: int = 4):
        super().__init__()
        self.hidden, self.inner, self.state = hidden, inner, state
        self.rank = math.ceil(hidden / 16)
        self.conv1d = nn.Conv1d(inner, inner, kernel_size=conv, groups=inner, padding=conv - 1, bias=True)
        self.in_proj = nn.Linear(hidden, 2 * inner, bias=False)
        self.x_proj = nn.Linear(inner, self.rank + 2 * state, bias=False)
        self.dt_proj = nn.Linear(self.rank, inner, bias=True)
        self.A_log = nn.Parameter(torch.empty(inner, state))
        self.D = nn.Parameter(torch.empty(inner))
        self.out_proj = nn.Linear(inner, hidden, bias=False)
        self._init_ssm()

    @torch.no_grad()
    def _init_ssm(self, dt_min=1e-3, dt_max=1e-1, dt_floor=1e-4, dt_scale=1.0):
        # MambaMixer.init_mamba_weights (time_step_init_scheme 'random', MambaConfig defaults)
        A = torch.arange(1, self.state + 1, dtype=torch.float32)[None, :].expand(self.inner, -1)
        self.A_log.copy_(torch.log(A))
        self.D.fill_(1.0)
        std = self.rank ** -0.5 * dt_scale
        nn.init.uniform_(self.dt_proj.weight, -std, std)
        dt = torch.exp(torch.rand(self.inner) * (math.log(dt_max) - math.log(dt_min)) + math.log(dt_min))
        dt = dt.clamp(min=dt_floor)
        self.dt_proj.bias.copy_(dt + torch.log(-torch.expm1(-dt)))


class HsiMambaParams(nn.Module):
    """hsiMamba(arch 'globalview1'/'globalview2', patch 1, out_type 'featmap', path '81_2+8'/'49_2+8')."""

    def __init__(self, cin: int, embed: int, img: int):
        super().__init__()
        n = img * img
        self.pos_embed = nn.Parameter(torch.zeros(1, n, embed))     # learnable PE, init_weights never called
        self.patch_embed = PatchEmbedParams(cin, embed)
        self.layers = nn.ModuleList([MambaMixerParams(embed, embed // 2)])
        self.pre_norm = nn.LayerNorm(embed, eps=1e-6)
        self.ln1 = nn.LayerNorm(embed, eps=1e-6)
        self.weights = nn.Parameter(torch.zeros(1, 10, 1))           # direction gate logits
        self.tokenlearner = TokenLearnerParams((img - 2) * (img - 2))  # unused by the reference forward
        self.ln3 = nn.LayerNorm(embed, eps=1e-6)                      # unused by the reference forward


class NonLocalParams(nn.Module):
    """NONLocalBlock2D(in_channels=C, sub_sample=True, bn_layer=True); W[1] BN zero-initialised (:114-115)."""

    def __init__(self, c: int):
        super().__init__()
        ci = max(c // 2, 1)
        self.inter = ci
        self.g = nn.Sequential(nn.Conv2d(c, ci, 1), nn.MaxPool2d(2))
        self.W = nn.Sequential(nn.Conv2d(ci, c, 1), nn.BatchNorm2d(c))
        nn.init.constant_(self.W[1].weight, 0)
        nn.init.constant_(self.W[1].bias, 0)
        self.theta = nn.Conv2d(c, ci, 1)
        self.phi = nn.Sequential(nn.Conv2d(c, ci, 1), nn.MaxPool2d(2))


class GLfusionParams(nn.Module):
    def __init__(self, c1: int, c2: int, out: int):
        super().__init__()
        self.cross_attention = NonLocalParams(c1)
        self.FusionLayer = nn.Sequential(nn.Conv2d(c1 + c2, out, 1), nn.BatchNorm2d(out), nn.ReLU())


class FusionParams(nn.Module):
    def __init__(self, c1: int, c2: int, out: int):
        super().__init__()
        self.FusionLayer = nn.Sequential(nn.Conv2d(c1 + c2, out, 1), nn.BatchNorm2d(out), nn.ReLU())


class ConvBnReluParams(nn.Module):
    """ms_conv_bn_relu: bn (on the input) -> conv3x3 (valid, bias) -> ReLU."""

    def __init__(self, cin: int, cout: int):
        super().__init__()
        self.bn = nn.BatchNorm2d(cin)
        self.conv = nn.Conv2d(cin, cout, 3, 1, 0, 1, 1, True)
        self.activation = nn.ReLU()


class GlobalLocalParams(nn.Module):
    def __init__(self, img: int, cin: int, cout: int, embed: int):
        super().__init__()
        s = (img - 2) * (img - 2)
        self.img, self.cin, self.cout, self.embed = img, cin, cout, embed
        self.global_view = HsiMambaParams(cin, embed, img)
        self.global_feature = TokenLearnerParams(s)
        # reference wires change_dim with in_channels although it consumes the embed-dim map
        # (:1068 vs :181); equal for Houston2013.  The generalisation uses the embed width.
        self.change_dim = nn.Conv2d(embed, cout, kernel_size=1)
        self.ln3 = nn.LayerNorm(cout, eps=1e-6)
        self.local_feature = ConvBnReluParams(cin, cout)
        self.channel_feature = nn.Conv2d(cin, cout, kernel_size=1)
        self.channel_token = TokenLearnerParams(s)
        self.ln4 = nn.LayerNorm(cout, eps=1e-6)
        self.FusionLayer = GLfusionParams(cout, cout, cout)
        self.fusion = FusionParams(cout, cout, cout)
