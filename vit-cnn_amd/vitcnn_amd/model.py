"""ViT-CNN ("Multimodality_Mamba") on MI355X: flat parameter storage + HIP forward/backward programs.

Drop-in for the reference module `Multimodality_Mamba`
(`/root/reference/model/Multimodality_Mamba/Mutimodality_Mamba7.py:1141-1181`):
same constructor signature, same state_dict (1704 keys, `layers.py`), same
`forward(hsi[B,C1,P,P], lidar[B,C2,P,P]) -> logits[B,ncls]` contract, train/eval BatchNorm
semantics, `.to(device)`, `parameters()`, `load_state_dict()`.

MI355X-first design:
  * all parameters live in ONE flat fp32 buffer (nn.Parameters are views of it), BN running
    stats in one flat fp32 buffer, `num_batches_tracked` in one int64 buffer.  Gradients come
    back as one flat tensor (`model.flat_params.grad`), so AdamW is one kernel and the data-
    parallel all-reduce is one RCCL call;
  * activations are channels-last `[rows, C]` in a per-batch-size workspace whose addresses
    never change, so a whole training step can be captured into a hipGraph;
  * every op runs in a hand-written gfx950 kernel of libvitcnn_hip.so (C ABI, include/vitcnn.h);
    there is no CPU path: a CPU tensor or a missing library raises.
"""
from __future__ import annotations

import contextlib
import ctypes
import math
import sys
import weakref
from typing import Dict

import torch
import torch.nn as nn

from ._lib import lib
from .flat import install_grad_views
from .layers import ConvBnReluParams, FusionParams, GlobalLocalParams
from .scan_orders import scan_orders

F32 = 4
LN_EPS = 1e-6
BN_EPS = 1e-5
BN_MOM = 0.1
NDIR = 10
N_SIDE = 3                 # side streams: 1 = local/non-local branch, 2 = channel branch, 3 = LiDAR branch
_ONE_PARAM_REDUCE = True   # a hsiMamba block's scan / conv1d parameter gradients in one reduction launch
WGRAD_LANE = 2             # backward: lane 0's deferred weight gradients (lane 2 is idle after the forward)
WGRAD1_LANE = 3            # backward: lane 1's deferred weight gradients (lane 3: after the fusion1 / LiDAR chain)
# Program switches.  Module constants -- the product reads no environment: each selects between two
# forms the tests hold to the same parity (or bit-identity), and the measurement tools set them from
# VITCNN_<NAME> variables through tools/knobs.py (tools/ab_env.sh A/B runs).  The defaults are the
# measured-fastest forms.
#
# 3x3 convs of ViT-CNN: im2col + vc_gemm by default; VITCNN_IMPLICIT_CONV=1 selects the implicit GEMM
# (vc_conv3x3_*), measured slower on this step (2.39 -> 2.55 ms: the per-element gather with the fused
# BN affine costs more VALU than the small im2col matrices cost bandwidth); FusAtNet, whose col
# matrices reach 611 MB, always uses the implicit GEMM
_IMPLICIT_CONV = False
# lane-0 weight gradients are batched and issued on the weight-gradient lane at a few flush points
# (one fork each); forking each one separately measured slower (2.39 -> 2.63 ms: every cross-lane
# graph edge costs more than one GEMM's overlap gains); False: every weight gradient in place
_DEFER_WGRAD = True
# lane 1's weight gradients (GLfusion, local conv, channel feature) queued and issued on WGRAD1_LANE at the end
# of the block's lane-1 chain, so lane 1 -- the critical path since round 3 -- runs the data gradients only.
# Measured slower: 1.80-1.81 -> 1.99-2.02 ms (profiles/r04_ab_defer_wgrad1.log): the block's grouped weight
# gradients then run beside lane 0's scan backward and stretch it more than lane 1 gains
_DEFER_WGRAD1 = False
SIDE_SCRATCH = 1 << 23     # floats of scratch per side stream
PARAM_ALIGN = 4            # floats: flat-buffer alignment (16 B) of every parameter of >= ALIGN_MIN elements
ALIGN_MIN = 64
GEMM_GROUP_BYTES = 16384   # VC_GEMM_GROUP_BYTES (include/vitcnn.h)
GEMM_MASK = 64             # vc_gemm flags: the addend is a ReLU mask (include/vitcnn.h)
# capture order of a GlobalLocal block's forward: lane 0's global view (the hsiMamba chain) captured before the local /
# channel branches it runs beside (the same DAG, bit-identical).  Measured 1.695 vs 1.687 ms (3 rounds x 300 replays,
# profiles/r06_ab_global_first.log): kept off
_GLOBAL_FIRST = False
# conv1x1 + BatchNorm (+ ReLU) forward: the statistics partials computed in the GEMM epilogue (vc_gemm_colstats)
_GEMM_BNSTATS = True
# GLfusion forward: the NonLocal phi | g projection on the channel lane (2) right after ln4, theta alone on lane 1
_PG_LANE2 = False   # measured slower: 1.745 -> 1.758-1.762 ms (profiles/r05_ab_pg_lane2.log)
N_COUNTERS = 1 << 16       # split-K tile counters per stream

# the Mamba direction conv + x_proj folded into the scan launch and the dt_proj / x_proj data gradients +
# conv1d backward into the scan backward's tail (vc_mamba_scan_fwd_fused / _bwd_fused); False restores the
# separate launches
_SCAN_FUSED = True
# patch_embed + pre_norm + in_proj and combine + out_proj + ln1 + change_dim as one launch each
# (vc_rowchain_front / _back); False restores the separate launches
_ROW_CHAIN = True
# GLfusion: the phi | g max pool inside the non-local attention forward and its backward inside the
# attention backward, the concat gradient's add + copy as one launch (vc_nonlocal_attn_pool_fwd / _bwd,
# vc_add2_2d_dup); False restores the separate launches
_GLF_FUSED = True
# the local conv's data gradient as the tap-major implicit GEMM (vc_conv3x3_tap_dgrad, no dcol matrix, no
# col2im) over the weights packed tap-major by lane 0 in the forward: opt-in, measured slower on the B=64
# step (1.90-1.94 -> 1.99-2.01 ms: at 7x7 / 9x9 maps the row gathers cost more than dcol + col2im)
_TAP_DGRAD = False
_LANES = True        # branch-level stream concurrency (False: every lane on the caller's stream)
_LANES_BWD = True    # the same for the backward alone
_TRACER = None   # launch-structure recorder of tools/critical_path.py (None in normal runs)
_GROUP = True        # grouped launches of independent fp32 GEMMs
# bf16 mode diagnostics (tools/bf16_sites.py): GEMM issue indices kept in fp32, and a log of call sites
_BF16_EXACT: set = set()
# bf16 mode: bf16 operands for products with K >= this that are not weight gradients; 0 = every GEMM
# bf16 (the reference's autocast mode).  Round 4: with bf16 MFMAs in the pipelined kernel (grouped like the
# fp32 problems) every GEMM in bf16 is the fastest: 1.67-1.69 vs 1.78 ms/step with 1024 (round 3's value,
# the im2col'ed 3x3 convs only) on one box, fp32 1.805 (profiles/r04_ab_bf16_min_k.log)
_BF16_MIN_K = 0
_GEMM_SITES = None
_LANE_MAP = []       # logical lane -> stream index (empty: lane i on stream i)
# the channel-feature backward chain's lane: 1 = after the local-conv chain on lane 1 (default); 3 = on
# lane 3 beside it (measured slower, round 3: 2.01 -> 2.23 ms).  Both chains accumulate into the block's
# input gradient dX; with _CH_ORDERED the side lane waits for the local chain before its accumulation,
# so the sum is formed in the same order under every schedule (without that wait
# the two read-modify-write GEMM epilogues race, and the result depends on the schedule)
_CH_LANE = 1
_CH_ORDERED = True
_BN_RELU_AFFINE = True   # BN + ReLU backward: the ReLU decisions recomputed from the BN input and affine
_BN_TICKETS = False  # BN reductions without dx in the last-arriving block: measured ~1% slower (every arrival is an
#                     agent-scope release = L2 writeback); with dx the counters select the one-launch kernels

UNUSED_PREFIXES = ("hsi1.global_view.tokenlearner.", "hsi1.global_view.ln3.",
                   "hsi2.global_view.tokenlearner.", "hsi2.global_view.ln3.")


PRECISIONS = ("fp32", "bf16")
GEMM_BF16 = 2              # vc_gemm flags bit: bf16 operands, fp32 accumulation


def _check_precision(p):
    if p not in PRECISIONS:
        raise ValueError(f"precision must be one of {PRECISIONS}, got {p!r}")
    return p


class _Workspace:
    """Named, persistent device buffers for one (device, batch, mode) — stable addresses."""

    def __init__(self, device):
        self.device = device
        self.t: Dict[str, torch.Tensor] = {}
        self.generation = 0

    def get(self, name, numel, dtype=torch.float32):
        t = self.t.get(name)
        if t is None or t.numel() != numel or t.dtype != dtype:
            t = torch.empty(max(int(numel), 1), dtype=dtype, device=self.device)
            self.t[name] = t
        return t

    def f(self, name, numel):
        return self.get(name, numel).data_ptr()

    def tensor(self, name):
        return self.t[name]


# the largest patch side the kernels take: hsi1's NonLocal attends over the 2x2-pooled (P - 2)^2 grid, at most 16
# pooled keys per query (csrc/attention.hip MAXP), i.e. P <= 11 -- MUUFL's 11x11 (SURVEY.md row A-MUUFL)
MAX_PATCH = 11


def _check_supported(P, c1):
    """Reject, at construction, a shape some kernel of the program would refuse mid-step: the patch
    side (NonLocal pooled keys), the HSI band count (TokenLearner / NonLocal channel bounds) and each TokenLearner
    call's LDS plan (vc_tl_check)."""
    if P > MAX_PATCH:
        raise ValueError(f"ViT-CNN patch {P}x{P} is not supported: at most {MAX_PATCH}x{MAX_PATCH} (the NonLocal "
                         f"attention takes at most 16 pooled keys, ((P - 2) // 2)^2)")
    if c1 > 512:
        raise ValueError(f"ViT-CNN with {c1} HSI bands is not supported: at most 512")
    L = lib()
    for hw, c, s in ((P * P, 256, (P - 2) ** 2), ((P - 2) ** 2, c1, (P - 4) ** 2)):
        if L.raw["vc_tl_check"](hw, c, s) != 0:
            raise ValueError(f"ViT-CNN TokenLearner over {hw} pixels x {c} channels with {s} tokens is not supported")


class Multimodality_Mamba(nn.Module):
    """ViT-CNN (ours).  Signature of Mutimodality_Mamba7.py:1142; like the reference, `patch_size`,
    `stride`, `dim_embedding` and `path_type` are accepted and ignored.  `img_size` is the patch
    side P (the reference hard-codes 9; other P follow the documented generalisation of
    SURVEY.md section 8 row A-MUUFL)."""

    def __init__(self, img_size=9, patch_size=1, stride=1, in_channels1=144, in_channels2=1, dim_embedding=32,
                 num_class=16, path_type="multi_clock_gate", *, precision="fp32"):
        super().__init__()
        self.precision = _check_precision(precision)
        P = int(img_size)
        if P < 7:
            raise ValueError("ViT-CNN needs patches of at least 7x7 (two valid 3x3 stages + 2x2 pooling)")
        _check_supported(P, int(in_channels1))
        self.patch, self.c1, self.c2, self.ncls = P, int(in_channels1), int(in_channels2), int(num_class)
        self.embedding_dim = dim_embedding
        plane_hsi = [self.c1, 256, self.c1]
        plane_lidar = [self.c2, 16, 32]
        self.hsi1 = GlobalLocalParams(P, plane_hsi[0], plane_hsi[1], 144)
        self.hsi2 = GlobalLocalParams(P - 2, plane_hsi[1], plane_hsi[2], 256)
        self.lidar1 = ConvBnReluParams(plane_lidar[0], plane_lidar[1])
        self.lidar2 = ConvBnReluParams(plane_lidar[1], plane_lidar[2])
        self.fusion1 = FusionParams(plane_hsi[1], plane_lidar[1], 128)
        self.fusion2 = FusionParams(plane_hsi[2], plane_lidar[2], 128)
        self.avg = nn.AdaptiveAvgPool2d(1)
        self.classifier = nn.Linear(128, self.ncls)
        self._build_flat()
        self._ws: Dict[tuple, _Workspace] = {}
        self._dev_cache: Dict[str, object] = {}

    # ------------------------------------------------------------------ flat storage
    def _build_flat(self):
        named = list(nn.Module.named_parameters(self))
        active = [(n, p) for n, p in named if not n.startswith(UNUSED_PREFIXES)]
        unused = [(n, p) for n, p in named if n.startswith(UNUSED_PREFIXES)]
        # NonLocal phi / g: the two weights, then the two biases, adjacent (stacked [2 Ci, Cout] / [2 Ci]),
        # so that both projections -- forward, data and weight gradient -- are one GEMM each
        for pfx in ("hsi1", "hsi2"):
            nl = pfx + ".FusionLayer.cross_attention."
            group = [nl + "phi.0.weight", nl + "g.0.weight", nl + "phi.0.bias", nl + "g.0.bias"]
            idx = {n: i for i, (n, _) in enumerate(active)}
            if all(n in idx for n in group):
                items = [active[idx[n]] for n in group]
                first = min(idx[n] for n in group)
                rest = [it for it in active if it[0] not in group]
                active = rest[:first] + items + rest[first:]
        # every parameter of >= ALIGN_MIN elements starts 16-B aligned (PARAM_ALIGN floats): the GEMM
        # kernels stage weights by 16-B LDS-DMA / float4 loads, which an arbitrary float offset would rule
        # out.  Smaller ones stay packed (the TokenLearner kernels address a block's S tokenizers'
        # 2 + 1 + 1 + 1 parameters as one run).  The gaps hold zeros in the parameters and in every
        # gradient (the backward zeroes them: vc_fill_index)
        def place(n, p, off):
            if p.numel() >= ALIGN_MIN:
                off = -(-off // PARAM_ALIGN) * PARAM_ALIGN
            self._poff[n] = off
            return off + p.numel()

        self._poff: Dict[str, int] = {}
        off = 0
        for n, p in active:
            off = place(n, p, off)
        self._n_active = -(-off // PARAM_ALIGN) * PARAM_ALIGN
        off = self._n_active
        for n, p in unused:
            off = place(n, p, off)
        self._n_params = off
        self._n_elems = sum(p.numel() for _, p in named)
        covered = torch.zeros(self._n_active, dtype=torch.bool)
        for n, p in active:
            covered[self._poff[n]:self._poff[n] + p.numel()] = True
        self._gaps = (~covered).nonzero().flatten().to(torch.int32).tolist()
        for pfx in ("hsi1", "hsi2"):   # the stacked phi | g projection needs its four tensors adjacent
            nl = pfx + ".FusionLayer.cross_attention."
            w, g_, b, gb = (self._poff.get(nl + k) for k in ("phi.0.weight", "g.0.weight", "phi.0.bias", "g.0.bias"))
            if w is not None:
                ci = dict(named)[nl + "phi.0.bias"].numel()
                cout = dict(named)[nl + "phi.0.weight"].numel() // ci
                if not (g_ == w + ci * cout and b == g_ + ci * cout and gb == b + ci):
                    raise RuntimeError(f"{nl}phi / g are not adjacent in the flat layout")
        device = named[0][1].device
        flat = torch.zeros(off, dtype=torch.float32, device=device)
        for n, p in named:
            flat[self._poff[n]:self._poff[n] + p.numel()].copy_(p.detach().reshape(-1))
        self._pnames = [n for n, _ in active + unused]
        self._pmods = {}
        for mn, m in nn.Module.named_modules(self):
            for pn in m._parameters:
                self._pmods[(mn + "." if mn else "") + pn] = (m, pn)
        # float buffers (BN running stats) and int64 counters
        self._boff, self._ioff = {}, {}
        fb, ib = [], []
        self._bmods = {}
        for mn, m in nn.Module.named_modules(self):
            for bn, b in m._buffers.items():
                if b is None:
                    continue
                full = (mn + "." if mn else "") + bn
                self._bmods[full] = (m, bn)
                (fb if b.is_floating_point() else ib).append((full, b))
        o = 0
        for n, b in fb:
            self._boff[n] = o
            o += b.numel()
        bflat = torch.empty(max(o, 1), dtype=torch.float32, device=device)
        for n, b in fb:
            bflat[self._boff[n]:self._boff[n] + b.numel()].copy_(b.reshape(-1))
        o = 0
        for n, b in ib:
            self._ioff[n] = o
            o += b.numel()
        iflat = torch.zeros(max(o, 1), dtype=torch.int64, device=device)
        for n, b in ib:
            iflat[self._ioff[n]:self._ioff[n] + b.numel()].copy_(b.reshape(-1))
        self._bshape = {n: tuple(b.shape) for n, b in fb + ib}
        # counters that a training forward increments: every BN the forward actually runs
        self._tracked = [self._ioff[n] for n, _ in ib if not n.startswith(UNUSED_PREFIXES)]
        self._rebind(flat, bflat, iflat)
        me = weakref.ref(self)
        for _, p in named:
            p._vc_owner = me

    def _rebind(self, flat, bflat, iflat):
        object.__setattr__(self, "_flat_store", flat.detach().requires_grad_(True))
        install_grad_views(self)
        object.__setattr__(self, "_bflat", bflat)
        object.__setattr__(self, "_iflat", iflat)
        base = self._flat_store.detach()
        for n in self._pnames:
            m, pn = self._pmods[n]
            p = m._parameters[pn]
            o = self._poff[n]
            p.data = base[o:o + p.numel()].view(p.shape)
        for n, (m, bn) in self._bmods.items():
            shape = self._bshape[n]
            numel = int(math.prod(shape)) if shape else 1
            if n in self._boff:
                o = self._boff[n]
                m._buffers[bn] = bflat[o:o + numel].view(shape)
            else:
                o = self._ioff[n]
                m._buffers[bn] = iflat[o:o + numel].view(shape)
        self._ptr_cache = None
        self._ws = {}
        self._dev_cache = {}
        # every rebind frees the workspaces / device tables: hipGraphs captured before it are stale
        # (TrainStepper compares this generation before replaying)
        self._bind_gen = getattr(self, "_bind_gen", 0) + 1

    def _flat_intact(self):
        base = self._flat_store.data_ptr()
        for n in (self._pnames[0], self._pnames[-1]):
            m, pn = self._pmods[n]
            if m._parameters[pn].data_ptr() != base + F32 * self._poff[n]:
                return False
        return True

    def _ensure_flat(self):
        if not self._flat_intact():  # e.g. parameters replaced by user code: re-flatten current values
            dev = self._flat_store.device
            flat = torch.zeros(self._n_params, dtype=torch.float32, device=dev)
            for n in self._pnames:
                m, pn = self._pmods[n]
                o = self._poff[n]
                flat[o:o + m._parameters[pn].numel()].copy_(m._parameters[pn].detach().reshape(-1))
            self._rebind(flat, self._bflat, self._iflat)

    def _apply(self, fn, recurse=True):
        flat = fn(self._flat_store.detach())
        if flat.dtype != torch.float32:
            raise RuntimeError("ViT-CNN MI355X path computes in fp32 master weights; dtype casts are not supported")
        bflat, iflat = fn(self._bflat), fn(self._iflat)
        if flat.data_ptr() == self._flat_store.data_ptr() and bflat.data_ptr() == self._bflat.data_ptr() and \
                iflat.data_ptr() == self._iflat.data_ptr():
            # .to(the device it is on): nothing moves, and the workspaces -- which captured hipGraphs of
            # the step (vitcnn_amd.step.TrainStepper) write into -- must stay alive
            return self
        self._rebind(flat, bflat, iflat)
        return self

    def set_precision(self, precision: str):
        """Arithmetic of the dense contractions (BASELINE config 2): "fp32" (the parity mode, exact fp32
        MFMA) or "bf16" (every GEMM's operands rounded to bf16 as they are staged, fp32 accumulation;
        master weights, AdamW, the scan state, LayerNorm / BatchNorm / TokenLearner statistics and
        all elementwise work stay fp32)."""
        self.precision = _check_precision(precision)
        return self

    @property
    def flat_params(self) -> torch.Tensor:
        """The single fp32 parameter tensor; after backward its .grad holds every gradient."""
        return self._flat_store

    @property
    def n_active_params(self) -> int:
        """Leading elements of flat_params that receive gradients (the rest are the unused
        hsiMamba.tokenlearner / ln3 parameters the reference never calls)."""
        return self._n_active

    def flat_buffers(self):
        """(fp32 running statistics, int64 num_batches_tracked) — every buffer of the model lives
        in one of these two tensors (one broadcast each for data-parallel buffer sync)."""
        return self._bflat, self._iflat

    def _state_layout(self):
        """(key, buffer kind, offset, shape, numel) in state_dict() order, and state_dict's metadata"""
        lay = getattr(self, "_sd_layout", None)
        if lay is None:
            sd = nn.Module.state_dict(self)
            rows = []
            for k, v in sd.items():
                kind = "p" if k in self._poff else ("b" if k in self._boff else "i")
                off = (self._poff if kind == "p" else self._boff if kind == "b" else self._ioff)[k]
                rows.append((k, kind, off, tuple(v.shape), v.numel()))
            lay = (rows, getattr(sd, "_metadata", None))
            object.__setattr__(self, "_sd_layout", lay)
        return lay

    def snapshot_state_dict(self, device=None):
        """state_dict() -- same keys, order, shapes and metadata -- whose values are views of ONE copy of
        each flat buffer (three device copies instead of 1704 tensor copies): train()'s best-state copy
        (model_utils.py:1017 deep-copies the state_dict every improving epoch) and save_model (one
        device-to-host transfer).  `device`: where the copy goes (default: the model's device)."""
        from collections import OrderedDict
        rows, meta = self._state_layout()
        src = {}
        for kind, t in (("p", self._flat_store.detach()), ("b", self._bflat), ("i", self._iflat)):
            src[kind] = t.clone() if device is None else t.to(device, copy=True)
        out = OrderedDict((k, src[kind][o:o + n].view(shape)) for k, kind, o, shape, n in rows)
        if meta is not None:
            out._metadata = meta
        return out

    def zero_grad(self, set_to_none: bool = True):
        super().zero_grad(set_to_none=set_to_none)
        if set_to_none:
            self._flat_store.grad = None
        elif self._flat_store.grad is not None:
            self._flat_store.grad.zero_()

    # ------------------------------------------------------------------ device caches
    def _ptrs(self):
        base = self._flat_store.data_ptr()
        if self._ptr_cache is None or self._ptr_cache[0] != base:
            bb, ib = self._bflat.data_ptr(), self._iflat.data_ptr()
            p = {n: base + F32 * o for n, o in self._poff.items()}
            b = {n: bb + F32 * o for n, o in self._boff.items()}
            self._ptr_cache = (base, p, b, ib)
        return self._ptr_cache

    def _device_tables(self, device):
        key = str(device)
        t = self._dev_cache.get(key)
        if t is None:
            t = {}
            for H in (self.patch, self.patch - 2):
                orders = scan_orders(H)
                inv = [[0] * len(o) for o in orders]
                for k, o in enumerate(orders):
                    for pos, tok in enumerate(o):
                        inv[k][tok] = pos
                t[("order", H)] = torch.tensor(orders, dtype=torch.int32, device=device).contiguous()
                t[("inv", H)] = torch.tensor(inv, dtype=torch.int32, device=device).contiguous()
            t["tracked"] = torch.tensor(self._tracked, dtype=torch.int32, device=device)
            t["gaps"] = torch.tensor(self._gaps, dtype=torch.int32, device=device)
            self._dev_cache[key] = t
        return t

    def _workspace(self, device, B, mode):
        key = (str(device), int(B), mode)
        ws = self._ws.get(key)
        if ws is None:
            ws = _Workspace(device)
            self._ws[key] = ws
        return ws

    def _scratch(self, device, B):
        need = self._scratch_floats(B)
        key = "scratch"
        t = self._dev_cache.get(str(device), {}).get(key)
        if t is None or t.numel() < need:
            if t is not None:
                self._bind_gen += 1   # the old scratch is freed: graphs captured with it are stale
            t = torch.empty(need, dtype=torch.float32, device=device)
            self._device_tables(device)[key] = t
        return t

    def _side_lanes(self, device):
        """Side streams of the step's branch-level concurrency, each with its own scratch (split-K
        slabs, reduction partials) so concurrent kernels never share a workspace.  The hsiMamba
        scan (the only large scratch user) always runs on the caller's stream."""
        tab = self._device_tables(device)
        lanes = tab.get("lanes")
        if lanes is None:
            lanes = [(torch.cuda.Stream(device), torch.empty(SIDE_SCRATCH, dtype=torch.float32, device=device))
                     for _ in range(N_SIDE)]
            tab["lanes"] = lanes
        return lanes

    def _gemm_group_buf(self, device, lane):
        """host memory of one grouped-GEMM state per lane (vc_gemm_group_*: the library keeps none)"""
        tab = self._device_tables(device)
        bufs = tab.get("gemm_groups")
        if bufs is None:
            bufs = [ctypes.create_string_buffer(GEMM_GROUP_BYTES) for _ in range(N_SIDE + 1)]
            tab["gemm_groups"] = bufs
        return ctypes.addressof(bufs[lane])

    def _tile_counters(self, device):
        """one zeroed split-K arrival-counter array per lane (vc_gemm_ex; kernels leave them zero)"""
        tab = self._device_tables(device)
        c = tab.get("tile_counters")
        if c is None:
            c = [torch.zeros(N_COUNTERS, dtype=torch.int32, device=device) for _ in range(N_SIDE + 1)]
            tab["tile_counters"] = c
        return c

    def _scratch_floats(self, B):
        need = 1 << 22
        for blk in (self.hsi1, self.hsi2):
            L = blk.img * blk.img
            D = blk.embed // 2
            nseq = NDIR * B
            nchunk = -(-D // 16)
            need = max(need, nchunk * nseq * L * 32 + nseq * D * 16 + nseq * D + nseq * nchunk + (1 << 20))
        return int(need)

    # ------------------------------------------------------------------ nn.Module API
    def forward(self, hsi: torch.Tensor, lidar: torch.Tensor) -> torch.Tensor:
        if hsi.device.type != "cuda":
            raise RuntimeError("ViT-CNN MI355X path: inputs must be on a ROCm (cuda) device; no CPU fallback")
        if hsi.dim() != 4 or hsi.shape[1] != self.c1 or hsi.shape[2] != self.patch or hsi.shape[3] != self.patch:
            raise RuntimeError(f"expected hsi [B, {self.c1}, {self.patch}, {self.patch}], got {list(hsi.shape)}")
        if lidar.dim() != 4 or lidar.shape[0] != hsi.shape[0] or lidar.shape[1] != self.c2 or \
                lidar.shape[2] != self.patch or lidar.shape[3] != self.patch:
            raise RuntimeError(f"expected lidar [B, {self.c2}, {self.patch}, {self.patch}], got {list(lidar.shape)}")
        self._ensure_flat()
        if self._flat_store.device != hsi.device:
            raise RuntimeError("model and inputs are on different devices")
        hsi = hsi.detach().to(torch.float32).contiguous()
        lidar = lidar.detach().to(torch.float32).contiguous()
        needs_grad = torch.is_grad_enabled() and self._flat_store.requires_grad
        return _VitCnnFunction.apply(self, hsi, lidar, self._flat_store, needs_grad)


class _VitCnnFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model, hsi, lidar, flat, needs_grad):
        prog = _Program(model, hsi.device, hsi.shape[0], model.training, "grad" if needs_grad else "nograd")
        logits = prog.forward(hsi, lidar)
        ctx.prog = prog
        ctx.gen = prog.ws.generation
        ctx.model = model
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        prog = ctx.prog
        if prog.ws.generation != ctx.gen:
            raise RuntimeError("ViT-CNN MI355X path: another training forward of the same batch size overwrote "
                               "the saved activations before this backward; call backward before the next forward")
        # The autograd engine runs this on its device thread.  Forking side streams from that thread
        # inside a hipGraph capture (opened on the user's thread) breaks capture_end on this ROCm
        # release, so a captured autograd backward runs on one stream; `fused_train_step`
        # (step.py) captures the multi-stream backward from the caller's thread instead.
        grad = prog.backward(dlogits.detach().to(torch.float32).contiguous(),
                             lanes=not torch.cuda.is_current_stream_capturing())
        return None, None, None, grad, None


class _Program:
    """The forward / backward launch sequence of one training step (channels-last activations)."""

    def __init__(self, model: Multimodality_Mamba, device, B, train, mode):
        self.m = model
        self.L = lib() if _TRACER is None else _TRACER.wrap(lib(), self)
        self.B = int(B)
        self.train = 1 if train else 0
        self.ws = model._workspace(device, B, ("train" if train else "eval", mode))
        self.ws_grad = mode == "grad"
        self.tab = model._device_tables(device)
        scr = model._scratch(device, B)
        lanes = model._side_lanes(device)
        self.streams = [torch.cuda.current_stream(device)] + [st for st, _ in lanes]
        if _LANE_MAP:   # logical lane -> stream (lanes sharing a stream run in issue order)
            self.streams = [self.streams[_LANE_MAP[i]] for i in range(len(self.streams))]
        self._raw = [st.cuda_stream for st in self.streams]
        self._scr = [(scr.data_ptr(), scr.numel())] + [(t.data_ptr(), t.numel()) for _, t in lanes]
        self._cnt = [t.data_ptr() for t in model._tile_counters(device)]
        self.gemm_flags = GEMM_BF16 if model.precision == "bf16" else 0
        # 3x3 convs as implicit GEMMs (fp32 only, opt-in); bf16 operands use im2col + the bf16 vc_gemm
        self.implicit_conv = not self.gemm_flags and _IMPLICIT_CONV
        self.scan_fused = _SCAN_FUSED
        self.row_chain = _ROW_CHAIN
        self.cur = 0
        self._gemm_i = 0
        self._ev_i = 0
        self._ev_lane = {}
        self.lanes_on = _LANES
        self.wgrad_tail = None
        self.pending_wgrads = []
        self.wgrad_tail1 = None
        self.pending_wgrads1 = []
        self._grouping = None      # the open GEMM group's state (host address) while gemm_group() collects
        self._group_lane = 0
        _, self.P, self.BUF, self.I64 = model._ptrs()
        self.device = device

    # ---------------------------------------------------------------- lanes (stream-level concurrency)
    # Lane 0 is the caller's stream; independent branches of the network run on side lanes that
    # fork from / join back to it through events (captured as graph edges under hipGraph capture).
    @property
    def s(self):
        return self._raw[self.cur]

    @property
    def scr_p(self):
        return self._scr[self.cur][0]

    @property
    def scr_n(self):
        return self._scr[self.cur][1]

    def _event(self):
        """next event of the model's per-device pool.  Events are reused step after step instead of
        created and destroyed: an event destroyed while a hipGraph capture is still open leaves the
        capture referring to a dead object."""
        pool = self.m._device_tables(self.device).setdefault("events", [])
        if self._ev_i == len(pool):
            pool.append(torch.cuda.Event())
        e = pool[self._ev_i]
        self._ev_i += 1
        return e

    def site_flags(self, ta, M, N, K, exact=False):
        """one GEMM site of the program: its index (the _GEMM_SITES census, the _BF16_EXACT list) and the
        precision flags the policy gives it (the model's bf16 bit unless exact / excluded / below _BF16_MIN_K).
        Every GEMM entry point the program calls goes through here, so site indices stay stable"""
        i = self._gemm_i
        self._gemm_i += 1
        if _GEMM_SITES is not None:
            f = sys._getframe(2)
            f = f.f_back if f.f_code.co_name.startswith("mm_") else f
            _GEMM_SITES.append((i, f.f_code.co_name, f.f_lineno, M, N, K, exact))
        if self.gemm_flags and not exact and i not in _BF16_EXACT and K >= _BF16_MIN_K and not (_BF16_MIN_K and ta):
            return self.gemm_flags
        return 0

    def gemm(self, *args, exact=False, ws=None):
        """vc_gemm_ex on the current lane with its scratch and split-K tile counters; args are
        vc_gemm's up to bias_grad (flags at index 21 get the model's precision bit unless `exact`);
        ws = (pointer, floats): a caller-owned slab buffer instead of the lane's scratch"""
        fl = self.site_flags(args[0], args[2], args[3], args[4], exact)
        if fl:
            args = args[:21] + (args[21] | fl,) + args[22:]
        wp, wn = ws if ws is not None else (self.scr_p, self.scr_n)
        if self._grouping is not None and self._group_lane == self.cur:
            self.L.vc_gemm_group_add(self._grouping, *args, wp, wn, self._cnt[self.cur], N_COUNTERS)
        else:
            self.L.vc_gemm_ex(*args, wp, wn, self._cnt[self.cur], N_COUNTERS, self.s)

    @contextlib.contextmanager
    def gemm_group(self):
        """the fp32 GEMMs issued inside (on the current lane; they must be independent of each other)
        launch as one grouped grid + one grouped split-K reduce (vc_gemm_group_begin / _add / _end over
        the lane's caller-owned group state)"""
        if not _GROUP or self._grouping is not None:   # nested: the outer group collects
            yield
            return
        grp = self.m._gemm_group_buf(self.device, self.cur)
        self.L.vc_gemm_group_begin(grp, self.s)
        self._grouping, self._group_lane = grp, self.cur
        try:
            yield
        finally:
            self._grouping = None
            self.L.vc_gemm_group_end(grp)

    def mark(self):
        """event recorded on the current lane"""
        e = self._event()
        e.record(self.streams[self.cur])
        self._ev_lane[id(e)] = self.cur
        if _TRACER is not None:
            _TRACER.mark(e, self.cur)
        return e

    def wait(self, *events):
        """The current lane waits for the given events.  Capture rules this ROCm release needs
        (tools/graph_probe*.py): a side lane is forked by waiting on a lane-0 event before it waits
        on another side lane's event, and a lane never waits on its own event (a no-op anyway)."""
        for e in events:
            src = self._ev_lane.get(id(e))
            if src is not None and self.streams[src] is self.streams[self.cur]:
                continue
            self.streams[self.cur].wait_event(e)
            if _TRACER is not None:
                _TRACER.wait(e, self.cur)

    @contextlib.contextmanager
    def lane(self, i, *after):
        prev = self.cur
        self.cur = i if self.lanes_on else 0
        self.wait(*after)
        try:
            yield
        finally:
            self.cur = prev

    def join_lanes(self):
        """lane 0 waits for everything issued on the side lanes"""
        assert self.cur == 0
        for i in range(1, len(self.streams)):
            if any(self.streams[i] is self.streams[j] for j in range(i)):
                continue   # a stream shared with an earlier lane (VITCNN_LANE_MAP)
            e = self._event()
            e.record(self.streams[i])
            self.streams[0].wait_event(e)
            if _TRACER is not None:
                _TRACER.mark(e, i)
                _TRACER.wait(e, 0)

    # ---------------------------------------------------------------- gemm wrappers
    def mm_nt(self, M, N, K, A, lda, W, ldw, C, ldc, bias=0, alpha=1.0, beta=0.0, add=0, add_ld=0, add_mod=0,
              relu=0, exact=False):
        """C[M,N] = alpha * A[M,K] W[N,K]^T + beta*C + bias + addend"""
        self.gemm(0, 1, M, N, K, alpha, A, lda, 0, W, ldw, 0, beta, C, ldc, 0, 1, bias or None, add or None,
                  add_ld, add_mod, relu, None, exact=exact)

    def mm_nn(self, M, N, K, A, lda, Bm, ldb, C, ldc, alpha=1.0, beta=0.0, relu_mask=0):
        """C[M,N] = alpha * A[M,K] B[K,N] + beta*C; relu_mask (a [M,N] layer output, ld N): the result
        is zeroed where relu_mask <= 0 (the ReLU backward through that output, in the GEMM epilogue)"""
        self.gemm(0, 0, M, N, K, alpha, A, lda, 0, Bm, ldb, 0, beta, C, ldc, 0, 1, None, relu_mask or None,
                  N if relu_mask else 0, 0, GEMM_MASK if relu_mask else 0, None)

    def mm_tn(self, M, N, K, A, lda, Bm, ldb, C, ldc, alpha=1.0, beta=0.0, bias_grad=0, flags=0, ws=None):
        """C[M,N] = alpha * A^T B, A stored [K, M] (weight gradients: M,N small, K = rows);
        bias_grad[M] (optional) = alpha * column sums of A, fused into the same GEMM"""
        self.gemm(1, 0, M, N, K, alpha, A, lda, 0, Bm, ldb, 0, beta, C, ldc, 0, 1, None, None, 0, 0, flags,
                  bias_grad or None, ws=ws)

    def colsum(self, R, C, X, ldx, out, beta=0.0):
        self.L.vc_colsum_ex(R, C, X, ldx, out, beta, self.scr_p, self.scr_n, self._cnt[self.cur], N_COUNTERS, self.s)

    # ---------------------------------------------------------------- building blocks (forward)
    def bn_stats(self, pfx, X, ldx, M, C, tag):
        ws = self.ws
        mean, inv = ws.f(tag + ".bm", C), ws.f(tag + ".bi", C)
        self.L.vc_bn_stats_ex(self.train, M, C, X, ldx, BN_EPS, BN_MOM, mean, inv, self.BUF[pfx + ".running_mean"],
                              self.BUF[pfx + ".running_var"], self.scr_p, self.scr_n,
                              self._cnt[self.cur] if _BN_TICKETS else None, N_COUNTERS, self.s)
        return mean, inv

    def layernorm(self, pfx, X, R, C, tag):
        ws = self.ws
        Y, mu, rs = ws.f(tag, R * C), ws.f(tag + ".m", R), ws.f(tag + ".r", R)
        self.L.vc_layernorm_fwd(R, C, X, C, self.P[pfx + ".weight"], self.P[pfx + ".bias"], LN_EPS, Y, C, mu, rs,
                                self.s)
        return Y

    def conv_bn_relu3(self, pfx, X, H, Cin, Cout):
        """ms_conv_bn_relu: BN(X) -> conv3x3 valid (+bias) -> ReLU: vc_im2col3x3 (BN affine fused) +
        vc_gemm, or the implicit GEMM vc_conv3x3_fwd (VITCNN_IMPLICIT_CONV=1, fp32)."""
        B, S = self.B, (H - 2) * (H - 2)
        if self.train and not self.implicit_conv:
            # statistics partials + (final reduction, BN apply, im2col) in one launch: vc_bn_im2col3x3
            tag, ws = pfx + ".bn", self.ws
            col = ws.f(pfx + ".col", B * S * 9 * Cin)
            self.L.vc_bn_im2col3x3(B, H, H, Cin, X, BN_EPS, BN_MOM, ws.f(tag + ".bm", Cin), ws.f(tag + ".bi", Cin),
                                   self.BUF[tag + ".running_mean"], self.BUF[tag + ".running_var"],
                                   self.P[tag + ".weight"], self.P[tag + ".bias"], col, self.scr_p, self.scr_n, self.s)
            out = ws.f(pfx + ".out", B * S * Cout)
            self.mm_nt(B * S, Cout, 9 * Cin, col, 9 * Cin, self.P[pfx + ".conv.weight"], 9 * Cin, out, Cout,
                       bias=self.P[pfx + ".conv.bias"], relu=1)
            return out
        mean, inv = self.bn_stats(pfx + ".bn", X, Cin, B * H * H, Cin, pfx + ".bn")
        if self.implicit_conv:
            out = self.ws.f(pfx + ".out", B * S * Cout)
            self.L.vc_conv3x3_fwd(B, H, H, Cin, Cout, 0, X, Cin, mean, inv, self.P[pfx + ".bn.weight"],
                                  self.P[pfx + ".bn.bias"], self.P[pfx + ".conv.weight"], self.P[pfx + ".conv.bias"], 1,
                                  out, Cout, self.scr_p, self.scr_n, self.s)
            return out
        col = self.ws.f(pfx + ".col", B * S * 9 * Cin)
        self.L.vc_im2col3x3(B, H, H, Cin, X, mean, inv, self.P[pfx + ".bn.weight"], self.P[pfx + ".bn.bias"], col,
                            self.s)
        out = self.ws.f(pfx + ".out", B * S * Cout)
        self.mm_nt(B * S, Cout, 9 * Cin, col, 9 * Cin, self.P[pfx + ".conv.weight"], 9 * Cin, out, Cout,
                   bias=self.P[pfx + ".conv.bias"], relu=1)
        return out

    def conv1x1_bn_relu(self, seq, X, M, Cin, Cout):
        """Sequential(Conv2d 1x1, BatchNorm2d, ReLU) (FusionLayer of GLfusionBlock / fusionBlock)."""
        pre = self.ws.f(seq + ".pre", M * Cout)
        tag, ws = seq + ".1", self.ws
        mean, inv = ws.f(tag + ".bm", Cout), ws.f(tag + ".bi", Cout)
        out = ws.f(seq + ".out", M * Cout)
        W, bias = self.P[seq + ".0.weight"], self.P[seq + ".0.bias"]
        if self.train and _GEMM_BNSTATS and Cin % 4 == 0 and X % 16 == 0 and W % 16 == 0:
            # the BatchNorm statistics pass folded into the GEMM's epilogue (partials per 64-row tile, shift = the
            # conv bias), then one statistics + apply + ReLU launch: 2 launches instead of 3
            P_ = -(-M // 64)
            cs = ws.get(seq + ".cs", 2 * P_ * Cout, torch.float64).data_ptr()
            fl = self.site_flags(0, M, Cout, Cin)
            self.L.vc_gemm_colstats(M, Cout, Cin, X, Cin, W, Cin, bias, pre, Cout, fl, cs, self.s)
            self.L.vc_bn_apply_partials(M, Cout, pre, Cout, P_, cs, bias, BN_EPS, BN_MOM, mean, inv,
                                        self.BUF[tag + ".running_mean"], self.BUF[tag + ".running_var"],
                                        self.P[tag + ".weight"], self.P[tag + ".bias"], 1, out, Cout, self.s)
            return out
        self.mm_nt(M, Cout, Cin, X, Cin, W, Cin, pre, Cout, bias=bias)
        # statistics partials + the channel-tiled apply that reduces them (two launches), include/vitcnn.h
        self.L.vc_bn_forward_ex(self.train, M, Cout, pre, Cout, BN_EPS, BN_MOM, mean, inv,
                                self.BUF[tag + ".running_mean"], self.BUF[tag + ".running_var"],
                                self.P[tag + ".weight"], self.P[tag + ".bias"], 1, out, Cout, self.scr_p, self.scr_n,
                                self._cnt[self.cur], N_COUNTERS, self.s)
        return out

    def fusion(self, pfx, X1, C1, X2, C2, M, Cout):
        cat = self.ws.f(pfx + ".cat", M * (C1 + C2))
        self.L.vc_cat2_fwd(M, C1, C2, X1, C1, X2, C2, 1 if C1 == C2 else 0, cat, self.s)
        return self.conv1x1_bn_relu(pfx + ".FusionLayer", cat, M, C1 + C2, Cout)

    def tl_ws(self, pfx, L_, S):
        """the TokenLearner call site's fp64 scratch (moment / gradient partials, include/vitcnn.h)"""
        return self.ws.get(pfx + ".tlw", (self.L.vc_tl_ws_floats(self.B, L_, S) + 1) // 2, torch.float64).data_ptr()

    def token_learner(self, pfx, X, L_, C, S):
        """TokenLearner(S) forward (Mutimodality_Mamba7.py:51-64): the pooled channel max / mean per pixel, then
        the tokens' BN(1) statistics, attention maps and pooled tokens Z [B, S, C] in one launch"""
        B, ws = self.B, self.ws
        rows = B * L_
        mx, amx, avg = ws.f(pfx + ".mx", rows), ws.get(pfx + ".amx", rows, torch.int32).data_ptr(), ws.f(pfx + ".avg",
                                                                                                           rows)
        tlw = self.tl_ws(pfx, L_, S)
        self.L.vc_tl_pixel_stats(rows, C, X, C, mx, amx, avg, tlw, self.s)
        st = ws.get(pfx + ".st", 2 * S + 8, torch.float64).data_ptr()
        Z = ws.f(pfx + ".Z", B * S * C)
        # the attention maps, kept for the backward's pooling product (training with grad only)
        amap = ws.f(pfx + ".a", B * S * L_) if self.ws_grad else None
        self.L.vc_tl_fwd(self.train, B, L_, C, S, X, C, mx, avg, self.P[pfx + ".tokenizers.0.conv.0.weight"],
                         self.BUF[pfx + ".tokenizers.0.conv.1.running_mean"], BN_EPS, BN_MOM, tlw, st, amap, Z, self.s)
        return Z

    def block(self, blk, pfx, X, H):
        B, ws, P = self.B, self.ws, self.P
        Cin, Cout, E = blk.cin, blk.cout, blk.embed
        D, R = E // 2, math.ceil(E / 16)
        XW = R + 32
        L_, Hs = H * H, H - 2
        S, Ci, Pk = Hs * Hs, Cout // 2, (Hs // 2) * (Hs // 2)
        rows = B * L_
        gv, mx = pfx + ".global_view", pfx + ".global_view.layers.0"
        order, inv = self.tab[("order", H)].data_ptr(), self.tab[("inv", H)].data_ptr()
        M = B * S
        if _GLOBAL_FIRST:
            # lanes 1 / 2 fork here, but their launches are captured after lane 0's global view: the graph's
            # executor hands the kernels to the hardware queues in capture order (section 14)
            e0 = self.mark()
            Fg = self.global_view(blk, pfx, X, H)
            FM, e_fm = self.block_local_branch(blk, pfx, X, H, e0)
            self.wait(e_fm)
            return self.fusion(pfx + ".fusion", Fg, Cout, FM, Cout, M, Cout)
        FM, e_fm = self.block_local_branch(blk, pfx, X, H)
        Fg = self.global_view(blk, pfx, X, H)
        self.wait(e_fm)
        # --- fusionBlock(global, fused) with ChannelExchange
        return self.fusion(pfx + ".fusion", Fg, Cout, FM, Cout, M, Cout)

    def global_view(self, blk, pfx, X, H):
        """hsiMamba global view -> change_dim -> TokenLearner -> ln3 (lane 0); returns Fg"""
        B, ws, P = self.B, self.ws, self.P
        Cin, Cout, E = blk.cin, blk.cout, blk.embed
        D, R = E // 2, math.ceil(E / 16)
        XW = R + 32
        L_, Hs = H * H, H - 2
        S = Hs * Hs
        rows = B * L_
        gv, mx = pfx + ".global_view", pfx + ".global_view.layers.0"
        order, inv = self.tab[("order", H)].data_ptr(), self.tab[("inv", H)].data_ptr()
        if self._tap_dgrad(blk):
            # the local conv's weight, tap-major, for its data gradient in the backward (lane 0 has slack here)
            self.L.vc_conv3x3_pack(Cout, Cin, 0, P[pfx + ".local_feature.conv.weight"],
                                   ws.f(pfx + ".local_feature.wt", Cout * 9 * ((Cin + 3) // 4 * 4)), 0.0, self.s)
        # --- hsiMamba global view (Mutimodality_Mamba7.py:419-701, :983-1017), on lane 0
        T = ws.f(pfx + ".T", rows * E)
        XZ = ws.f(pfx + ".XZ", rows * 2 * D)
        chain = self._chain_ok(blk)
        if chain:
            # patch_embed + pos_embed -> pre_norm -> in_proj in one launch (T, Xn and its statistics kept)
            tag = pfx + ".Xn"
            self.L.vc_rowchain_front(rows, Cin, E, 2 * D, X, P[gv + ".patch_embed.projection.weight"],
                                     P[gv + ".pos_embed"], L_, T, P[gv + ".pre_norm.weight"], P[gv + ".pre_norm.bias"],
                                     LN_EPS, ws.f(tag, rows * E), ws.f(tag + ".m", rows), ws.f(tag + ".r", rows),
                                     P[mx + ".in_proj.weight"], XZ, self.s)
        else:
            self.mm_nt(rows, E, Cin, X, Cin, P[gv + ".patch_embed.projection.weight"], Cin, T, E,
                       add=P[gv + ".pos_embed"], add_ld=E, add_mod=L_)
            Xn = self.layernorm(gv + ".pre_norm", T, rows, E, pfx + ".Xn")
            self.mm_nt(rows, 2 * D, E, Xn, E, P[mx + ".in_proj.weight"], E, XZ, 2 * D)
        U = ws.f(pfx + ".U", NDIR * rows * D)
        XD = ws.f(pfx + ".XD", NDIR * rows * XW)
        Y = ws.f(pfx + ".Y", NDIR * rows * D)
        # segment checkpoints of the scan state, kept for the backward (training with grad only)
        CKP = ws.f(pfx + ".CKP", self.L.vc_mamba_scan_ckpt_floats(B, L_, D, NDIR)) if self.ws_grad else None
        if self.scan_fused:
            # direction conv + x_proj + scan as one launch (U and XD written for the backward)
            self.L.vc_mamba_scan_fwd_fused(B, L_, D, R, NDIR, XZ, order, P[mx + ".conv1d.weight"],
                                           P[mx + ".conv1d.bias"], P[mx + ".x_proj.weight"],
                                           P[mx + ".dt_proj.weight"], P[mx + ".dt_proj.bias"], P[mx + ".A_log"],
                                           P[mx + ".D"], U, XD, Y, CKP, self.s)
        else:
            self.L.vc_mamba_dirconv_fwd(B, L_, D, NDIR, order, XZ, P[mx + ".conv1d.weight"],
                                        P[mx + ".conv1d.bias"], U, self.s)
            self.mm_nt(NDIR * rows, XW, D, U, D, P[mx + ".x_proj.weight"], D, XD, XW)
            self.L.vc_mamba_scan_fwd(B, L_, D, R, NDIR, U, XD, order, P[mx + ".dt_proj.weight"],
                                     P[mx + ".dt_proj.bias"], P[mx + ".A_log"], P[mx + ".D"], Y, CKP, self.s)
        YP, YS = ws.f(pfx + ".YP", rows * D), ws.f(pfx + ".YS", rows * D)
        T2 = ws.f(pfx + ".T2", rows * E)
        CD = ws.f(pfx + ".CD", rows * Cout)
        if chain:
            # combine -> out_proj (+ residual) -> ln1 -> change_dim in one launch
            tag = pfx + ".G"
            self.L.vc_rowchain_back(B, L_, D, NDIR, inv, P[gv + ".weights"], Y, XZ, YP, YS, E,
                                    P[mx + ".out_proj.weight"], T, T2, P[gv + ".ln1.weight"], P[gv + ".ln1.bias"],
                                    LN_EPS, ws.f(tag, rows * E), ws.f(tag + ".m", rows), ws.f(tag + ".r", rows), Cout,
                                    P[pfx + ".change_dim.weight"], P[pfx + ".change_dim.bias"], CD, self.s)
        else:
            self.L.vc_mamba_combine_fwd(B, L_, D, NDIR, inv, P[gv + ".weights"], Y, XZ, YP, YS, self.s)
            self.mm_nt(rows, E, D, YS, D, P[mx + ".out_proj.weight"], D, T2, E, add=T, add_ld=E, add_mod=rows)
            G = self.layernorm(gv + ".ln1", T2, rows, E, pfx + ".G")
            # --- global feature: change_dim -> TokenLearner -> ln3
            self.mm_nt(rows, Cout, E, G, E, P[pfx + ".change_dim.weight"], E, CD, Cout,
                       bias=P[pfx + ".change_dim.bias"])
        Zg = self.token_learner(pfx + ".global_feature", CD, L_, Cout, S)
        return self.layernorm(pfx + ".ln3", Zg, B * S, Cout, pfx + ".Fg")

    def block_local_branch(self, blk, pfx, X, H, e0=None):
        """local feature (lane 1) || channel feature (lane 2), then the GLfusionBlock on lane 1, forked from lane 0 at
        e0 (now if None); returns (FM, event on lane 1 after FM)."""
        B, ws, P = self.B, self.ws, self.P
        Cin, Cout = blk.cin, blk.cout
        L_, Hs = H * H, H - 2
        S, Ci, Pk = Hs * Hs, Cout // 2, (Hs // 2) * (Hs // 2)
        rows = B * L_
        e0 = self.mark() if e0 is None else e0
        # --- local feature: BN -> conv3x3 -> ReLU
        with self.lane(1, e0):
            Fl = self.conv_bn_relu3(pfx + ".local_feature", X, H, Cin, Cout)
        # --- channel feature: conv1x1 -> TokenLearner -> ln4
        with self.lane(2, e0):
            CF = ws.f(pfx + ".CF", rows * Cout)
            self.mm_nt(rows, Cout, Cin, X, Cin, P[pfx + ".channel_feature.weight"], Cin, CF, Cout,
                       bias=P[pfx + ".channel_feature.bias"])
            Zc = self.token_learner(pfx + ".channel_token", CF, L_, Cout, S)
            Fc = self.layernorm(pfx + ".ln4", Zc, B * S, Cout, pfx + ".Fc")
            if _PG_LANE2 and self.lanes_on:
                # the NonLocal phi | g projection of Fc on this lane, beside lane 1's local conv (_PG_LANE2)
                nl = pfx + ".FusionLayer.cross_attention"
                self.mm_nt(B * S, 2 * Ci, Cout, Fc, Cout, P[nl + ".phi.0.weight"], Cout, ws.f(pfx + ".PG", B * S * 2 * Ci),
                           2 * Ci, bias=P[nl + ".phi.0.bias"])
            e_fc = self.mark()
        with self.lane(1, e_fc):
            FM = self.glfusion(pfx, Fl, Fc, Cout, S, Ci, Pk, Hs)
            return FM, self.mark()

    def glfusion(self, pfx, Fl, Fc, Cout, S, Ci, Pk, Hs):
        """GLfusionBlock(x1 = channel, x2 = local): non-local cross attention (:140-159, :1107-1117)"""
        B, ws, P = self.B, self.ws, self.P
        nl = pfx + ".FusionLayer.cross_attention"
        M = B * S
        TH = ws.f(pfx + ".TH", M * Ci)
        PG = ws.f(pfx + ".PG", M * 2 * Ci)
        with self.gemm_group():
            self.mm_nt(M, Ci, Cout, Fl, Cout, P[nl + ".theta.weight"], Cout, TH, Ci, bias=P[nl + ".theta.bias"])
            if not (_PG_LANE2 and self.lanes_on):
                # phi | g as one product over their stacked weights / biases (_build_flat keeps them adjacent)
                self.mm_nt(M, 2 * Ci, Cout, Fc, Cout, P[nl + ".phi.0.weight"], Cout, PG, 2 * Ci,
                           bias=P[nl + ".phi.0.bias"])
        PP = ws.f(pfx + ".PP", B * Pk * 2 * Ci)
        PA = ws.get(pfx + ".PA", B * Pk * 2 * Ci, torch.uint8).data_ptr()
        ATT, O = ws.f(pfx + ".ATT", M * Pk), ws.f(pfx + ".O", M * Ci)
        if _GLF_FUSED:   # 2x2 max pool folded into the attention forward (pooled + taps kept for the backward)
            self.L.vc_nonlocal_attn_pool_fwd(B, S, Pk, Ci, Hs, TH, PG, 2 * Ci, PP, PA, ATT, O, self.s)
        else:
            self.L.vc_maxpool2_fwd(B, Hs, Hs, 2 * Ci, PG, 2 * Ci, PP, PA, self.s)
            self.L.vc_nonlocal_attn_fwd(B, S, Pk, Ci, TH, PP, ATT, O, self.s)
        WP = ws.f(pfx + ".WP", M * Cout)
        # the W projection stays fp32 in the bf16 mode: the train-mode BatchNorm after it sees a batch
        # spread small against the mean, so bf16 operands here alone move the logits by 3.3e-2 of their
        # scale (tools/bf16_sites.py: 5.8e-2 -> 2.5e-2 deviation, argmax 61/64 -> 64/64); a K = 128 GEMM
        self.mm_nt(M, Cout, Ci, O, Ci, P[nl + ".W.0.weight"], Ci, WP, Cout, bias=P[nl + ".W.0.bias"], exact=True)
        CAT1 = ws.f(pfx + ".CAT1", M * 2 * Cout)
        if self.train:   # BN(W y) statistics finished inside the combine launch
            tag = pfx + ".W1"
            self.L.vc_bn_glf_combine(M, Cout, WP, BN_EPS, BN_MOM, ws.f(tag + ".bm", Cout), ws.f(tag + ".bi", Cout),
                                     self.BUF[nl + ".W.1.running_mean"], self.BUF[nl + ".W.1.running_var"],
                                     P[nl + ".W.1.weight"], P[nl + ".W.1.bias"], Fc, Fl, CAT1, self.scr_p, self.scr_n,
                                     self.s)
        else:
            wm, wi = self.bn_stats(nl + ".W.1", WP, Cout, M, Cout, pfx + ".W1")
            self.L.vc_glf_combine_fwd(M, Cout, WP, wm, wi, P[nl + ".W.1.weight"], P[nl + ".W.1.bias"], Fc, Fl, CAT1,
                                      self.s)
        return self.conv1x1_bn_relu(pfx + ".FusionLayer.FusionLayer", CAT1, M, 2 * Cout, Cout)

    def forward(self, hsi, lidar):
        m, B, ws = self.m, self.B, self.ws
        ws.generation += 1
        Pp = m.patch
        X0 = ws.f("x0", B * Pp * Pp * m.c1)
        S1, S2 = (Pp - 2) ** 2, (Pp - 4) ** 2
        e_in = self.mark()
        # LiDAR branch on lane 3 (independent of the HSI blocks until fusion1 / fusion2)
        with self.lane(3, e_in):
            if m.c2 == 1:
                ws.t["lidar_in"] = lidar  # keep alive for the backward
                LX = lidar.data_ptr()
            else:
                LX = ws.f("lx0", B * Pp * Pp * m.c2)
                self.L.vc_nchw_to_nhwc(B, m.c2, Pp * Pp, lidar.data_ptr(), LX, self.s)
            L1 = self.conv_bn_relu3("lidar1", LX, Pp, m.c2, 16)
            L2 = self.conv_bn_relu3("lidar2", L1, Pp - 2, 16, 32)
            if self.train:   # every BatchNorm's num_batches_tracked += 1 (off lane 0's chain: nothing reads it)
                tr = self.tab["tracked"]
                self.L.vc_index_add_i64(tr.numel(), tr.data_ptr(), self.I64, 1, self.s)
        self.L.vc_nchw_to_nhwc(B, m.c1, Pp * Pp, hsi.data_ptr(), X0, self.s)
        ws.t["hsi_in"] = hsi
        self.X0, self.LX = X0, LX
        H1 = self.block(m.hsi1, "hsi1", X0, Pp)
        e_h1 = self.mark()
        with self.lane(3, e_h1):
            F1 = self.fusion("fusion1", H1, m.hsi1.cout, L1, 16, B * S1, 128)
            e_f1 = self.mark()
        H2 = self.block(m.hsi2, "hsi2", H1, Pp - 2)
        self.wait(e_f1)
        F2 = self.fusion("fusion2", H2, m.hsi2.cout, L2, 32, B * S2, 128)
        self.join_lanes()
        logits = torch.empty(B, m.ncls, dtype=torch.float32, device=self.device)
        feat = ws.f("feat", B * 128)
        self.L.vc_head_fwd(B, S1, S2, 128, m.ncls, F1, F2, self.P["classifier.weight"], self.P["classifier.bias"],
                           feat, logits.data_ptr(), self.s)
        self.H1, self.H2, self.L1, self.L2, self.F1, self.F2, self.feat = H1, H2, L1, L2, F1, F2, feat
        return logits

    # ---------------------------------------------------------------- backward
    def bn_bwd(self, pfx, tag, dY, lddy, X, ldx, relu_out, M, C, dX, lddx, beta_dx):
        ws = self.ws
        if relu_out and _BN_RELU_AFFINE:
            # the ReLU decisions recomputed from X and the affine (vc_bn_bwd_relu_ex: same bits, one read less)
            self.L.vc_bn_bwd_relu_ex(self.train, M, C, dY, lddy, X, ldx, ws.f(tag + ".bm", C), ws.f(tag + ".bi", C),
                                     self.P[pfx + ".weight"], self.P[pfx + ".bias"], dX or None, lddx, beta_dx,
                                     self.G[pfx + ".weight"], self.G[pfx + ".bias"], 0.0, self.scr_p, self.scr_n,
                                     self._cnt[self.cur] if (dX or _BN_TICKETS) else None, N_COUNTERS, self.s)
            return
        self.L.vc_bn_bwd_ex(self.train, M, C, dY, lddy, X, ldx, relu_out or None, C, ws.f(tag + ".bm", C),
                            ws.f(tag + ".bi", C), self.P[pfx + ".weight"], dX or None, lddx, beta_dx,
                            self.G[pfx + ".weight"], self.G[pfx + ".bias"], 0.0, self.scr_p, self.scr_n,
                            self._cnt[self.cur] if (dX or _BN_TICKETS) else None, N_COUNTERS, self.s)

    def ln_bwd(self, pfx, tag, dY, X, R, C, dX, beta_dx, res=0, defer=False):
        """dX = beta_dx * dX + LN grad, or res + LN grad (res: a residual gradient in another buffer).
        defer (lane 0): dX now, the weight / bias gradient reduction queued for the weight-gradient
        lane (its partials kept in a buffer of their own)"""
        ws = self.ws
        if self._deferring(defer):
            part_n = 1024 * 2 * C   # >= the kernel's partial rows, so the same split as vc_layernorm_bwd
            part = ws.f(tag + ".lnpart", part_n)
            self.L.vc_layernorm_bwd_dx(R, C, dY, C, X, C, self.P[pfx + ".weight"], ws.f(tag + ".m", R),
                                       ws.f(tag + ".r", R), res or None, C, dX, C, beta_dx, part, part_n, self.s)
            gw, gb = self.G[pfx + ".weight"], self.G[pfx + ".bias"]
            self.pending_wgrads.append(
                lambda: self.L.vc_layernorm_bwd_params(R, C, part, part_n, gw, gb, 0.0, self.s))
            return
        if res:
            self.L.vc_layernorm_bwd_res(R, C, dY, C, X, C, self.P[pfx + ".weight"], ws.f(tag + ".m", R),
                                        ws.f(tag + ".r", R), res, C, dX, C, self.G[pfx + ".weight"],
                                        self.G[pfx + ".bias"], 0.0, self.scr_p, self.scr_n, self.s)
            return
        self.L.vc_layernorm_bwd(R, C, dY, C, X, C, self.P[pfx + ".weight"], ws.f(tag + ".m", R), ws.f(tag + ".r", R),
                                dX, C, beta_dx, self.G[pfx + ".weight"], self.G[pfx + ".bias"], 0.0, self.scr_p,
                                self.scr_n, self.s)

    def linear_bwd(self, wname, bname, dY, M, N, K, X, ldx, dX, beta_dx, lddy=None, defer=False, relu_mask=0):
        """Y[M,N] = X[M,K] W[N,K]^T + b:  dW = dY^T X, db = colsum(dY), dX (+)= dY W (then masked by
        relu_mask > 0 if given: see mm_nn).

        defer (lane 0 only): the weight gradient is queued (self.defer_wgrad) and issued on the
        weight-gradient lane at the next flush_wgrads(), so the data gradient -- the only part the rest
        of the backward waits for -- follows at once on lane 0.  The caller guarantees that nothing
        writes dY or X again in this backward (they are read whenever the weight-gradient lane gets
        there, up to the final join)."""
        lddy = lddy or N
        with self.gemm_group():
            self.defer_wgrad(defer, N, K, M, dY, lddy, X, ldx, self.G[wname], K, self.G[bname] if bname else 0)
            if dX:
                self.mm_nn(M, K, N, dY, lddy, self.P[wname], K, dX, K, beta=beta_dx, relu_mask=relu_mask)

    def _deferring(self, defer):
        return defer and _DEFER_WGRAD and self.lanes_on and (self.cur == 0 or (self.cur == 1 and _DEFER_WGRAD1))

    def defer_wgrad(self, defer, M, N, K, A, lda, Bm, ldb, C, ldc, bias_grad=0):
        """C[M,N] = A^T B (a weight gradient, mm_tn), now or -- defer on lane 0 with lanes on -- at the next
        flush_wgrads().  (Round 5 also queued lane 1's split-K reductions for the weight-gradient lane: 1.74 ->
        2.0-2.1 ms, profiles/r05_ab_defer_reduce.log; removed with its ABI in round 6.)"""
        if self._deferring(defer):
            (self.pending_wgrads if self.cur == 0 else self.pending_wgrads1).append(
                lambda: self.mm_tn(M, N, K, A, lda, Bm, ldb, C, ldc, bias_grad=bias_grad))
            return
        self.mm_tn(M, N, K, A, lda, Bm, ldb, C, ldc, bias_grad=bias_grad)

    def flush_wgrads(self):
        """issue the queued parameter-gradient work (weight-gradient GEMMs, grouped; LayerNorm and scan
        parameter reductions) on the weight-gradient lane, forked once from lane 0 here; wgrad_tail =
        that lane's event after them"""
        if not self.pending_wgrads:
            return
        e = self.mark()
        with self.lane(WGRAD_LANE, e):
            with self.gemm_group():
                for fn in self.pending_wgrads:
                    fn()
            self.wgrad_tail = self.mark()
        self.pending_wgrads = []

    def flush_wgrads1(self):
        """lane 1's queued weight gradients (the GLfusion / local / channel chains' 1x1 and 3x3 convs) on
        WGRAD1_LANE, forked from lane 1 at the end of its block chain: lane 1 keeps only the data gradients"""
        if not self.pending_wgrads1:
            return
        e = self.mark()
        with self.lane(WGRAD1_LANE, e):
            with self.gemm_group():
                for fn in self.pending_wgrads1:
                    fn()
            self.wgrad_tail1 = self.mark()
        self.pending_wgrads1 = []

    def wgrad_events(self):
        """the weight-gradient lanes' latest events, as a list (empty if nothing was deferred)"""
        return [e for e in (self.wgrad_tail, self.wgrad_tail1) if e is not None]

    def conv1x1_bn_relu_bwd(self, seq, X, M, Cin, Cout, dOut, dX, beta_dx, defer=False):
        ws = self.ws
        pre, out = ws.f(seq + ".pre", M * Cout), ws.f(seq + ".out", M * Cout)
        dpre = ws.f(seq + ".dpre", M * Cout)
        self.bn_bwd(seq + ".1", seq + ".1", dOut, Cout, pre, Cout, out, M, Cout, dpre, Cout, 0.0)
        self.linear_bwd(seq + ".0.weight", seq + ".0.bias", dpre, M, Cout, Cin, X, Cin, dX, beta_dx, defer=defer)

    def fusion_bwd(self, pfx, X1, C1, X2, C2, M, Cout, dOut, dX1, beta1, dX2, beta2, defer=False):
        ws = self.ws
        cat = ws.f(pfx + ".cat", M * (C1 + C2))
        dcat = ws.f(pfx + ".dcat", M * (C1 + C2))
        self.conv1x1_bn_relu_bwd(pfx + ".FusionLayer", cat, M, C1 + C2, Cout, dOut, dcat, 0.0, defer=defer)
        self.L.vc_cat2_bwd(M, C1, C2, dcat, 1 if C1 == C2 else 0, dX1 or None, C1, beta1, dX2 or None, C2, beta2,
                           self.s)

    def _tap_dgrad(self, blk):
        return _TAP_DGRAD and self.ws_grad and not self.implicit_conv and blk.cin % 4 == 0

    def conv_bn_relu3_bwd(self, pfx, X, H, Cin, Cout, dOut, dX, beta_dx, tap=False, masked=False, defer=False):
        """tap: the data gradient by vc_conv3x3_tap_dgrad over the tap-major weight block() packed;
        masked: dOut has been through the ReLU backward already (its producer's GEMM epilogue)"""
        B, ws = self.B, self.ws
        S = (H - 2) * (H - 2)
        if masked:
            dpre = dOut
        else:
            out = ws.f(pfx + ".out", B * S * Cout)
            dpre = ws.f(pfx + ".dpre", B * S * Cout)
            self.L.vc_relu_bwd(B * S * Cout, dOut, out, dpre, self.s)
        dxbn = ws.f(pfx + ".dxbn", B * H * H * Cin)
        if self.implicit_conv:
            tag = pfx + ".bn"
            self.L.vc_conv3x3_wgrad(B, H, H, Cin, Cout, 0, X, Cin, ws.f(tag + ".bm", Cin), ws.f(tag + ".bi", Cin),
                                    self.P[tag + ".weight"], self.P[tag + ".bias"], dpre, Cout, 0.0,
                                    self.G[pfx + ".conv.weight"], self.G[pfx + ".conv.bias"], self.scr_p, self.scr_n,
                                    self.s)
            self.L.vc_conv3x3_dgrad(B, H, H, Cin, Cout, 0, dpre, Cout, self.P[pfx + ".conv.weight"], 0.0, dxbn, Cin,
                                    self.scr_p, self.scr_n, self.s)
        elif tap:
            col = ws.f(pfx + ".col", B * S * 9 * Cin)
            self.linear_bwd(pfx + ".conv.weight", pfx + ".conv.bias", dpre, B * S, Cout, 9 * Cin, col, 9 * Cin, 0, 0.0)
            self.L.vc_conv3x3_tap_dgrad(B, H, H, Cin, Cout, 0, dpre, Cout,
                                        ws.f(pfx + ".wt", Cout * 9 * ((Cin + 3) // 4 * 4)), 0.0, dxbn, Cin,
                                        self.scr_p, self.scr_n, self.s)
        else:
            col = ws.f(pfx + ".col", B * S * 9 * Cin)
            dcol = ws.f(pfx + ".dcol", B * S * 9 * Cin)
            self.linear_bwd(pfx + ".conv.weight", pfx + ".conv.bias", dpre, B * S, Cout, 9 * Cin, col, 9 * Cin, dcol,
                            0.0, defer=defer)
            self.L.vc_col2im3x3(B, H, H, Cin, dcol, dxbn, self.s)
        self.bn_bwd(pfx + ".bn", pfx + ".bn", dxbn, Cin, X, Cin, 0, B * H * H, Cin, dX, Cin, beta_dx)

    def token_learner_bwd(self, pfx, X, L_, C, S, dZ, dX):
        """dX (overwritten) = gradient of the TokenLearner input; the tokenizers' parameter gradients"""
        B, ws = self.B, self.ws
        rows = B * L_
        st = ws.get(pfx + ".st", 2 * S + 8, torch.float64).data_ptr()
        self.L.vc_tl_bwd(self.train, B, L_, C, S, X, C, ws.f(pfx + ".mx", rows), ws.f(pfx + ".avg", rows),
                         ws.get(pfx + ".amx", rows, torch.int32).data_ptr(), self.P[pfx + ".tokenizers.0.conv.0.weight"],
                         st, ws.f(pfx + ".a", B * S * L_), dZ, self.tl_ws(pfx, L_, S), dX, C,
                         self.G[pfx + ".tokenizers.0.conv.0.weight"], self.s)

    def block_bwd(self, blk, pfx, X, H, dOut, dX, dx_ready):
        """dX (accumulated, beta=1) = gradient w.r.t. the block input, or None to skip input grads;
        dx_ready = event after which dX holds its initial value (None: already ordered on lane 0).
        Lane 0 runs the global (hsiMamba) chain, lane 1 the GLfusion/non-local, local-conv and channel
        chains; the accumulations into dX are ordered local -> channel (lane 1) -> global (lane 0).
        Side lanes only ever wait on lane-0 events and lane 0 joins them (a star): the one cross-
        stream topology this ROCm release's graph capture handles in a backward (tools/graph_probe.py)."""
        B, ws, P, G = self.B, self.ws, self.P, self.G
        Cin, Cout, E = blk.cin, blk.cout, blk.embed
        D, R = E // 2, math.ceil(E / 16)
        XW = R + 32
        L_, Hs = H * H, H - 2
        S, Ci, Pk = Hs * Hs, Cout // 2, (Hs // 2) * (Hs // 2)
        rows, M = B * L_, B * S
        gv, mx = pfx + ".global_view", pfx + ".global_view.layers.0"
        nl = pfx + ".FusionLayer.cross_attention"
        order, inv = self.tab[("order", H)].data_ptr(), self.tab[("inv", H)].data_ptr()
        f = ws.f
        Fg, Fl, Fc = f(pfx + ".Fg", M * Cout), f(pfx + ".local_feature.out", M * Cout), f(pfx + ".Fc", M * Cout)
        FMo = f(pfx + ".FusionLayer.FusionLayer.out", M * Cout)
        # fusionBlock(Fg, FM)
        dFg, dFM = f(pfx + ".dFg", M * Cout), f(pfx + ".dFM", M * Cout)
        self.fusion_bwd(pfx + ".fusion", Fg, Cout, FMo, Cout, M, Cout, dOut, dFg, 0.0, dFM, 0.0, defer=True)
        if dX and dx_ready is not None:
            self.wait(dx_ready)  # lane 1 accumulates into dX: order it after dX's producer
        e0 = self.mark()
        with self.lane(1, e0):
            # GLfusionBlock FusionLayer + non-local branch (lane 1) -> dFc, dFl
            CAT1, dCAT1 = f(pfx + ".CAT1", M * 2 * Cout), f(pfx + ".dCAT1", M * 2 * Cout)
            self.conv1x1_bn_relu_bwd(pfx + ".FusionLayer.FusionLayer", CAT1, M, 2 * Cout, Cout, dFM, dCAT1, 0.0,
                                     defer=True)
            dFc, dFl = f(pfx + ".dFc", M * Cout), f(pfx + ".dFl", M * Cout)
            if _GLF_FUSED:
                self.L.vc_add2_2d_dup(M, Cout, dCAT1, 2 * Cout, dCAT1 + F32 * Cout, 2 * Cout, dFc, Cout, dFl, Cout,
                                      self.s)
            else:
                self.L.vc_add2_2d(M, Cout, dCAT1, 2 * Cout, dCAT1 + F32 * Cout, 2 * Cout, dFc, Cout, 0.0, self.s)
                self.L.vc_add2_2d(M, Cout, dFc, Cout, 0, 0, dFl, Cout, 0.0, self.s)
            # localf = BN(W o) + Fc + Fl  ->  non-local branch
            WP, dWP = f(pfx + ".WP", M * Cout), f(pfx + ".dWP", M * Cout)
            self.bn_bwd(nl + ".W.1", pfx + ".W1", dCAT1, 2 * Cout, WP, Cout, 0, M, Cout, dWP, Cout, 0.0)
            O, dO = f(pfx + ".O", M * Ci), f(pfx + ".dO", M * Ci)
            self.linear_bwd(nl + ".W.0.weight", nl + ".W.0.bias", dWP, M, Cout, Ci, O, Ci, dO, 0.0, defer=True)
            TH, PP, ATT = f(pfx + ".TH", M * Ci), f(pfx + ".PP", B * Pk * 2 * Ci), f(pfx + ".ATT", M * Pk)
            dTH, dPP = f(pfx + ".dTH", M * Ci), f(pfx + ".dPP", B * Pk * 2 * Ci)
            dPG = f(pfx + ".dPG", M * 2 * Ci)
            PA = ws.get(pfx + ".PA", B * Pk * 2 * Ci, torch.uint8).data_ptr()
            if _GLF_FUSED:   # attention backward with the 2x2 max-pool backward folded in (dPP: fallback only)
                self.L.vc_nonlocal_attn_pool_bwd(B, S, Pk, Ci, Hs, TH, PP, ATT, dO, PA, dTH, dPP, dPG, self.s)
            else:
                self.L.vc_nonlocal_attn_bwd(B, S, Pk, Ci, TH, PP, ATT, dO, dTH, dPP, self.s)
                self.L.vc_maxpool2_bwd(B, Hs, Hs, 2 * Ci, dPP, PA, dPG, 2 * Ci, self.s)
            # phi | g (stacked, one weight + one data gradient) and theta: one grouped launch
            with self.gemm_group():
                self.linear_bwd(nl + ".phi.0.weight", nl + ".phi.0.bias", dPG, M, 2 * Ci, Cout, Fc, Cout, dFc, 1.0,
                                defer=True)
                # dFl's last contribution; its epilogue applies the local conv's ReLU backward (mask Fl)
                self.linear_bwd(nl + ".theta.weight", nl + ".theta.bias", dTH, M, Ci, Cout, Fl, Cout, dFl, 1.0,
                                relu_mask=Fl, defer=True)
            side = self.lanes_on and _CH_LANE != 1
            e_pg = self.mark() if side else None
            # local feature: BN -> conv3x3 -> ReLU backward (first accumulation into dX)
            self.conv_bn_relu3_bwd(pfx + ".local_feature", X, H, Cin, Cout, dFl, dX or 0, 1.0, tap=self._tap_dgrad(blk),
                                   masked=True, defer=True)
            e_loc = self.mark() if side else None
        # channel feature: ln4 -> TokenLearner -> conv1x1, after the local chain on lane 1 (or, measurement
        # switch _CH_LANE, on a lane of its own beside it: see _CH_ORDERED)
        with (self.lane(_CH_LANE, e0, e_pg) if side else self.lane(1)):
            Zc, dZc = f(pfx + ".channel_token.Z", M * Cout), f(pfx + ".dZc", M * Cout)
            self.ln_bwd(pfx + ".ln4", pfx + ".Fc", dFc, Zc, M, Cout, dZc, 0.0)
            CF, dCF = f(pfx + ".CF", rows * Cout), f(pfx + ".dCF", rows * Cout)
            self.token_learner_bwd(pfx + ".channel_token", CF, L_, Cout, S, dZc, dCF)
            if side and dX and _CH_ORDERED:
                self.wait(e_loc)   # the dX accumulations in program order: local, then channel
            with self.gemm_group():
                self.linear_bwd(pfx + ".channel_feature.weight", pfx + ".channel_feature.bias", dCF, rows, Cout,
                                Cin, X, Cin, 0, 0.0, defer=True)
                if dX:
                    self.mm_nn(rows, Cin, Cout, dCF, Cout, self.P[pfx + ".channel_feature.weight"], Cin, dX, Cin,
                               beta=1.0)
            e_ch = (self.mark(), e_loc) if side else (self.mark(),)
            self.flush_wgrads1()   # lane 1's weight gradients, beside lane 0's chain
        # global feature: ln3 -> TokenLearner -> change_dim
        Zg, dZg = f(pfx + ".global_feature.Z", M * Cout), f(pfx + ".dZg", M * Cout)
        self.ln_bwd(pfx + ".ln3", pfx + ".Fg", dFg, Zg, M, Cout, dZg, 0.0, defer=True)
        CD, dCD = f(pfx + ".CD", rows * Cout), f(pfx + ".dCD", rows * Cout)
        self.token_learner_bwd(pfx + ".global_feature", CD, L_, Cout, S, dZg, dCD)
        Gm, dG = f(pfx + ".G", rows * E), f(pfx + ".dG", rows * E)
        # hsiMamba: ln1 -> out_proj -> scan/combine -> x_proj/dt_proj -> conv -> in_proj -> pre_norm -> patch_embed
        T2, dT = f(pfx + ".T2", rows * E), f(pfx + ".dT", rows * E)
        YS, dYS = f(pfx + ".YS", rows * D), f(pfx + ".dYS", rows * D)
        U, XD, XZ = f(pfx + ".U", NDIR * rows * D), f(pfx + ".XD", NDIR * rows * XW), f(pfx + ".XZ", rows * 2 * D)
        Y, YP = f(pfx + ".Y", NDIR * rows * D), f(pfx + ".YP", rows * D)
        dU, dDTL = f(pfx + ".dU", NDIR * rows * D), f(pfx + ".dDTL", NDIR * rows * D)
        dXD, dXZ, dYP = f(pfx + ".dXD", NDIR * rows * XW), f(pfx + ".dXZ", rows * 2 * D), f(pfx + ".dYP", rows * D)
        if self._chain_ok(blk):
            # change_dim / ln1 / out_proj data gradients + the SiLU(z) gate backward in one launch; the
            # weight gradients and ln1's parameter reduction queued for the weight-gradient lane
            part = f(pfx + ".ln1part", self.L.vc_rowchain_ln_part_floats(rows, E))
            self.L.vc_rowchain_back_bwd(rows, Cout, E, D, dCD, P[pfx + ".change_dim.weight"], T2, f(pfx + ".G.m", rows),
                                        f(pfx + ".G.r", rows), P[gv + ".ln1.weight"], dT, part,
                                        P[mx + ".out_proj.weight"], XZ, YP, dYP, dXZ, self.s)
            self.defer_wgrad(True, Cout, E, rows, dCD, Cout, Gm, E, G[pfx + ".change_dim.weight"], E,
                             G[pfx + ".change_dim.bias"])
            self._ln_params(gv + ".ln1", rows, E, part)
            self.defer_wgrad(True, E, D, rows, dT, E, YS, D, G[mx + ".out_proj.weight"], D)
        else:
            self.linear_bwd(pfx + ".change_dim.weight", pfx + ".change_dim.bias", dCD, rows, Cout, E, Gm, E, dG, 0.0,
                            defer=True)
            self.ln_bwd(gv + ".ln1", pfx + ".G", dG, T2, rows, E, dT, 0.0, defer=True)
            # (the pre_norm backward below writes the residual sum to dTt, so dT stays as this reads it)
            self.linear_bwd(mx + ".out_proj.weight", None, dT, rows, E, D, YS, D, dYS, 0.0, defer=True)
            # SiLU(z) gate (token-wise): dyp and the z half of dxz
            self.L.vc_mamba_gate_bwd(B, L_, D, XZ, YP, dYS, dYP, dXZ, self.s)
        self.flush_wgrads()   # fusion, change_dim, out_proj: alongside the scan backward
        CKPb = f(pfx + ".CKP", self.L.vc_mamba_scan_ckpt_floats(B, L_, D, NDIR))
        if self.scan_fused:
            self._scan_bwd_fused(pfx, gv, mx, B, L_, D, R, XW, order, inv, CKPb)
            return self._block_bwd_tail(blk, pfx, gv, mx, B, L_, E, Cin, rows, X, dX, dT, e_ch)
        if self._deferring(True):
            # the per-sequence dA_log / D / gate partials stay in a buffer of their own; their
            # reductions go with the next weight-gradient flush
            nseq = NDIR * B
            spn = nseq * D * 16 + nseq * D + nseq
            sp = f(pfx + ".scanpart", spn)
            self.L.vc_mamba_scan_bwd(B, L_, D, R, NDIR, U, XD, order, P[mx + ".dt_proj.weight"],
                                     P[mx + ".dt_proj.bias"], P[mx + ".A_log"], P[mx + ".D"], P[gv + ".weights"], Y,
                                     dYP, CKPb, dU, dDTL, dXD, None, None, None, sp, spn, self.s)
            gl, ga, gd, gg = P[gv + ".weights"], G[mx + ".A_log"], G[mx + ".D"], G[gv + ".weights"]
            self.pending_wgrads.append(
                lambda: self.L.vc_mamba_scan_bwd_params(B, D, NDIR, gl, sp, ga, gd, gg, self.scr_p, self.scr_n,
                                                        self.s))
        else:
            self.L.vc_mamba_scan_bwd(B, L_, D, R, NDIR, U, XD, order, P[mx + ".dt_proj.weight"],
                                     P[mx + ".dt_proj.bias"], P[mx + ".A_log"], P[mx + ".D"], P[gv + ".weights"], Y,
                                     dYP, CKPb, dU, dDTL, dXD, G[mx + ".A_log"], G[mx + ".D"], G[gv + ".weights"],
                                     self.scr_p, self.scr_n, self.s)
        nr = NDIR * rows
        # dt_proj: dt_lin = xdbl[:, :R] W_dt^T + b_dt
        # (the weight gradient reads dDTL and XD's dt-rank columns; the data gradient writes dXD's)
        self.defer_wgrad(True, D, R, nr, dDTL, D, XD, XW, G[mx + ".dt_proj.weight"], R, G[mx + ".dt_proj.bias"])
        self.mm_nn(nr, R, D, dDTL, D, P[mx + ".dt_proj.weight"], R, dXD, XW)
        # x_proj: xdbl = u W_x^T
        self.linear_bwd(mx + ".x_proj.weight", None, dXD, nr, XW, D, U, D, dU, 1.0, defer=True)
        self.L.vc_mamba_dirconv_bwd(B, L_, D, NDIR, order, inv, XZ, P[mx + ".conv1d.weight"], P[mx + ".conv1d.bias"],
                                    dU, dXZ, G[mx + ".conv1d.weight"], G[mx + ".conv1d.bias"], self.scr_p,
                                    self.scr_n, self.s)
        self._block_bwd_tail(blk, pfx, gv, mx, B, L_, E, Cin, rows, X, dX, dT, e_ch)

    def _scan_bwd_fused(self, pfx, gv, mx, B, L_, D, R, XW, order, inv, CKPb):
        """scan backward + dt_proj / x_proj data gradients + conv1d / SiLU backward in one launch
        (vc_mamba_scan_bwd_fused), the direction gather into dxz, and the parameter gradients (dt_proj,
        x_proj, conv1d, A_log / D / gate) queued for the weight-gradient lane"""
        P, G, f = self.P, self.G, self.ws.f
        rows = B * L_
        nr, nseq = NDIR * rows, NDIR * B
        U, XD, XZ = f(pfx + ".U", nr * D), f(pfx + ".XD", nr * XW), f(pfx + ".XZ", rows * 2 * D)
        Y, dYP = f(pfx + ".Y", nr * D), f(pfx + ".dYP", rows * D)
        dU, dDTL, dXD, dXZ = f(pfx + ".dU", nr * D), f(pfx + ".dDTL", nr * D), f(pfx + ".dXD", nr * XW), f(
            pfx + ".dXZ", rows * 2 * D)
        CP = f(pfx + ".convpart", nseq * 5 * D)
        defer = self._deferring(True)
        spn = nseq * D * 16 + nseq * D + nseq
        sp = f(pfx + ".scanpart", spn)
        gl, ga, gd, gg = P[gv + ".weights"], G[mx + ".A_log"], G[mx + ".D"], G[gv + ".weights"]
        self.L.vc_mamba_scan_bwd_fused(B, L_, D, R, NDIR, U, XD, order, XZ, P[mx + ".conv1d.weight"],
                                       P[mx + ".conv1d.bias"], P[mx + ".x_proj.weight"], P[mx + ".dt_proj.weight"],
                                       P[mx + ".dt_proj.bias"], P[mx + ".A_log"], P[mx + ".D"], gl, Y, dYP, CKPb, dU,
                                       dDTL, dXD, CP, None, None, None, sp, spn, self.s)
        cw, cb = G[mx + ".conv1d.weight"], G[mx + ".conv1d.bias"]
        # A_log, D, gate and conv1d parameter gradients: one reduction launch (the same order deferred or not), on the
        # weight-gradient lane when deferring (round 6; _ONE_PARAM_REDUCE = False: the round-5 launches)
        if _ONE_PARAM_REDUCE:
            params = lambda: self.L.vc_mamba_bwd_params(B, D, NDIR, gl, sp, CP, ga, gd, gg, cw, cb, self.s)  # noqa: E731
        else:
            def params():
                self.L.vc_mamba_scan_bwd_params(B, D, NDIR, gl, sp, ga, gd, gg, self.scr_p, self.scr_n, self.s)
                self.L.vc_mamba_conv_params(B, D, NDIR, CP, cw, cb, self.s)
        if defer:
            self.pending_wgrads.append(params)
        else:
            params()
        self.L.vc_mamba_dirconv_bwd_gather(B, L_, D, NDIR, inv, P[mx + ".conv1d.weight"], dU, dXZ, self.s)
        # parameter gradients: dt_proj (dDTL, XD's dt-rank columns), x_proj (dXD, U), conv1d (partials)
        self.defer_wgrad(True, D, R, nr, dDTL, D, XD, XW, G[mx + ".dt_proj.weight"], R, G[mx + ".dt_proj.bias"])
        self.defer_wgrad(True, XW, D, nr, dXD, XW, U, D, G[mx + ".x_proj.weight"], D)

    def _chain_ok(self, blk):
        """the row-chain launches apply to this block's widths (rowchain.hip limits)"""
        E = blk.embed
        return (self.row_chain and blk.cin <= 256 and blk.cin % 4 == 0 and E <= 256 and E % 4 == 0
                and (E // 2) % 4 == 0 and blk.cout <= 256)

    def _ln_params(self, pfx, rows, E, part):
        """a LayerNorm's weight / bias gradients from a backward chain's partials: queued for the
        weight-gradient lane (or now, without lanes)"""
        gw, gb = self.G[pfx + ".weight"], self.G[pfx + ".bias"]
        fn = lambda: self.L.vc_rowchain_ln_params(rows, E, part, gw, gb, 0.0, self.s)  # noqa: E731
        if self._deferring(True):
            self.pending_wgrads.append(fn)
        else:
            fn()

    def _block_bwd_tail(self, blk, pfx, gv, mx, B, L_, E, Cin, rows, X, dX, dT, e_ch):
        """in_proj -> pre_norm -> patch_embed backward of a GlobalLocal block"""
        ws, P, G, f = self.ws, self.P, self.G, self.ws.f
        D = E // 2
        dXZ = f(pfx + ".dXZ", rows * 2 * D)
        Xn, dXn = f(pfx + ".Xn", rows * E), f(pfx + ".dXn", rows * E)
        T, dTt = f(pfx + ".T", rows * E), f(pfx + ".dTt", rows * E)
        if self._chain_ok(blk):
            # in_proj / pre_norm (+ the residual dT) / patch_embed data gradients in one launch, after the
            # other branches' accumulations into dX (lane 1 is done long before lane 0 gets here)
            self.defer_wgrad(True, 2 * D, E, rows, dXZ, 2 * D, Xn, E, G[mx + ".in_proj.weight"], E)
            self.flush_wgrads()   # dt_proj, x_proj, conv1d, in_proj
            if dX:
                self.wait(*e_ch)
            part = f(pfx + ".prepart", self.L.vc_rowchain_ln_part_floats(rows, E))
            self.L.vc_rowchain_front_bwd(rows, 2 * D, E, Cin, dXZ, P[mx + ".in_proj.weight"], T, f(pfx + ".Xn.m", rows),
                                         f(pfx + ".Xn.r", rows), P[gv + ".pre_norm.weight"], dT, dTt, part,
                                         P[gv + ".patch_embed.projection.weight"], dX or None, 1.0, None, self.s)
            self._ln_params(gv + ".pre_norm", rows, E, part)
        else:
            self.linear_bwd(mx + ".in_proj.weight", None, dXZ, rows, 2 * D, E, Xn, E, dXn, 0.0, defer=True)
            self.flush_wgrads()   # dt_proj, x_proj, conv1d, in_proj
            self.ln_bwd(gv + ".pre_norm", pfx + ".Xn", dXn, T, rows, E, dTt, 0.0, res=dT, defer=True)   # dT + LN grad
            if dX:
                self.wait(*e_ch)
                self.mm_nn(rows, Cin, E, dTt, E, P[gv + ".patch_embed.projection.weight"], Cin, dX, Cin, beta=1.0)
        # pos_embed and patch_embed weight gradients: off the critical path
        e = self.mark()
        with self.lane(WGRAD_LANE if _DEFER_WGRAD else 0, e):
            self.colsum(B, L_ * E, dTt, L_ * E, G[gv + ".pos_embed"])
            self.mm_tn(E, Cin, rows, dTt, E, X, Cin, G[gv + ".patch_embed.projection.weight"], Cin)
            if self.lanes_on and _DEFER_WGRAD:
                self.wgrad_tail = self.mark()

    def bucket_ready(self, hook, name, *side_events):
        """Gradient bucket `name` is complete once lane 0 reaches this point and the given side-lane
        events have fired: hand `hook` (data parallelism, parallel.GradExchange) one lane-0 event plus
        the side events to order its collective after."""
        if hook is None:
            return
        assert self.cur == 0
        hook(name, [self.mark()] + list(side_events))

    def backward(self, dlogits, lanes=True, bucket_hook=None, out=None):
        """bucket_hook(name, events): called as each gradient bucket of parallel.GradExchange.BUCKETS
        ("tail": LiDAR + fusion + classifier, "hsi2", "hsi1" — head side first) is complete."""
        m, B, ws = self.m, self.B, self.ws
        self.lanes_on = lanes and _LANES and _LANES_BWD
        grad = out if out is not None else torch.empty(m._n_params, dtype=torch.float32, device=self.device)
        if m._n_params > m._n_active or m._gaps:
            # parameters the reference forward never uses get no gradient, and the alignment gaps stay zero
            # (off lane 0's chain: nothing reads these entries before the final join)
            with self.lane(3, self.mark()):
                self.L.vc_fill(m._n_params - m._n_active, grad.data_ptr() + F32 * m._n_active, 0.0, self.s)
                gaps = self.tab["gaps"]
                self.L.vc_fill_index(gaps.numel(), gaps.data_ptr(), grad.data_ptr(), 0.0, self.s)
        gb = grad.data_ptr()
        self.G = {n: gb + F32 * o for n, o in m._poff.items()}
        Pp = m.patch
        S1, S2 = (Pp - 2) ** 2, (Pp - 4) ** 2
        C1o, C2o = m.hsi1.cout, m.hsi2.cout
        dF1, dF2 = ws.f("dF1", B * S1 * 128), ws.f("dF2", B * S2 * 128)
        self.L.vc_head_bwd(B, S1, S2, 128, m.ncls, dlogits.data_ptr(), self.P["classifier.weight"], self.feat, dF1,
                           dF2, self.G["classifier.weight"], self.G["classifier.bias"], self.s)
        dH1, dH2 = ws.f("dH1", B * S1 * C1o), ws.f("dH2", B * S2 * C2o)
        dL1, dL2 = ws.f("dL1", B * S1 * 16), ws.f("dL2", B * S2 * 32)
        self.wgrad_tail = self.wgrad_tail1 = None
        self.fusion_bwd("fusion2", self.H2, C2o, self.L2, 32, B * S2, 128, dF2, dH2, 0.0, dL2, 0.0, defer=True)
        e_f2 = self.mark()
        with self.lane(3, e_f2):  # fusion1 + LiDAR branch on lane 3
            self.fusion_bwd("fusion1", self.H1, C1o, self.L1, 16, B * S1, 128, dF1, dH1, 0.0, dL1, 0.0)
            e_f1 = self.mark()
            self.conv_bn_relu3_bwd("lidar2", self.L1, Pp - 2, 16, 32, dL2, dL1, 1.0)
            self.conv_bn_relu3_bwd("lidar1", self.LX, Pp, m.c2, 16, dL1, 0, 0.0)
            e_l3 = self.mark()
        # classifier + fusion2 (lane 0 so far) and fusion1 + LiDAR (lane 3): the "tail" bucket
        if bucket_hook is not None:
            self.flush_wgrads()   # fusion2's weight gradient belongs to the tail bucket
        self.bucket_ready(bucket_hook, "tail", e_l3, *self.wgrad_events())
        self.block_bwd(m.hsi2, "hsi2", self.H1, Pp - 2, dH2, dH1, e_f1)
        # block_bwd joined its lane-1 chain before dH1; its deferred weight gradients end at wgrad_tail
        if bucket_hook is not None:
            self.flush_wgrads()   # hsi2's pre_norm parameter reduction is still queued
        self.bucket_ready(bucket_hook, "hsi2", *self.wgrad_events())
        self.block_bwd(m.hsi1, "hsi1", self.X0, Pp, dH1, None, None)
        self.flush_wgrads()
        self.join_lanes()
        self.bucket_ready(bucket_hook, "hsi1")
        return grad
