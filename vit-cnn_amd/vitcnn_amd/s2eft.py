"""S2EFT comparison model (config 5) on the MI355X path.

Reference: `model/compare_method/S2EFT.py` (class `ViT` :110-162, `Transformer` :76-108,
`Attention` :34-74, `FeedForward` :21-32), built by `model_utils.py:400-423`
(image_size 7, near_band 3, num_patches = n_bands, dim 64, depth 5, heads 4, mlp_dim 8,
dim_head 16, mode 'CAF', Adam lr 5e-4).

The module keeps the reference's parameter tree, so `state_dict()` has the reference's key names
and `.pth` files interchange.  Forward and backward are one hand-written program of HIP kernels
(`csrc/s2eft.hip` + `vc_gemm` + `vc_layernorm_*`) over token rows [B, T, D] (T = N + 1); the
parameters live in one flat fp32 buffer whose `.grad` the backward fills (the fused optimizer of
`optim.py` then updates it in one pass; Adam = `AdamW(weight_decay=0)`).

Dropout (p = 0.1 in `get_model`) is applied in training at the reference's four sites (emb_dropout
:151, to_out :43, FeedForward :26 and :28) by a counter-based hash mask (`vc_dropout_fwd`, seeded
from torch's CPU generator each forward, so `torch.manual_seed` reproduces a run; a hipGraph replay
repeats the captured masks).  The `mask` argument is unsupported (the reference's mask path
references an un-imported `F`, :58, and raises too).
"""
from __future__ import annotations

import ctypes
from functools import partial

import torch
import torch.nn as nn

from ._lib import lib
from .flat import F32, FlatParams

LN_EPS = 1e-5  # nn.LayerNorm default (PreNorm :13-19, mlp_head :125-128)


# ---------------------------------------------------------------- parameter tree (reference names)
class Residual(nn.Module):
    def __init__(self, fn):
        super().__init__()
        self.fn = fn


class PreNorm(nn.Module):
    def __init__(self, dim, fn):
        super().__init__()
        self.norm = nn.LayerNorm(dim)
        self.fn = fn


class FeedForward(nn.Module):
    def __init__(self, dim, hidden_dim, dropout=0.0):
        super().__init__()
        self.net = nn.Sequential(nn.Linear(dim, hidden_dim), nn.GELU(), nn.Dropout(dropout),
                                 nn.Linear(hidden_dim, dim), nn.Dropout(dropout))


class Attention(nn.Module):
    def __init__(self, dim, heads, dim_head, dropout):
        super().__init__()
        inner = dim_head * heads
        self.heads = heads
        self.scale = dim_head ** -0.5
        self.to_qkv = nn.Linear(dim, inner * 3, bias=False)
        self.to_out = nn.Sequential(nn.Linear(inner, dim), nn.Dropout(dropout))


class Transformer(nn.Module):
    def __init__(self, dim, depth, heads, dim_head, mlp_head, dropout, num_channel, mode):
        super().__init__()
        self.layers = nn.ModuleList([])
        for _ in range(depth):
            self.layers.append(nn.ModuleList([
                Residual(PreNorm(dim, Attention(dim, heads=heads, dim_head=dim_head, dropout=dropout))),
                Residual(PreNorm(dim, FeedForward(dim, mlp_head, dropout=dropout)))]))
        self.mode = mode
        self.skipcat = nn.ModuleList([])
        for _ in range(depth - 2):
            self.skipcat.append(nn.Conv2d(num_channel + 1, num_channel + 1, [1, 2], 1, 0))


class ViT(FlatParams, nn.Module):
    """Same constructor as the reference `ViT` (S2EFT.py:110-131); forward(x [B, N, C]) -> logits."""

    def __init__(self, image_size, near_band, num_patches, num_classes, dim, depth, heads, mlp_dim, pool="cls",
                 channels=1, dim_head=16, dropout=0.0, emb_dropout=0.0, mode="ViT"):
        super().__init__()
        if dim_head != 16:
            raise ValueError("S2EFT MI355X path: the attention kernel is written for dim_head 16 (the reference's)")
        if mode not in ("ViT", "CAF"):
            raise ValueError(f"unknown transformer mode {mode!r}")
        patch_dim = image_size ** 2 * near_band
        # creation order = the reference's, so the default initialisation draws the same numbers
        self.conv2d = nn.Conv1d(in_channels=2, out_channels=1, kernel_size=7, stride=1, padding=3)
        self.pos_embedding = nn.Parameter(torch.randn(1, num_patches + 2, dim))
        self.patch_to_embedding = nn.Linear(patch_dim, dim)
        self.cls_token = nn.Parameter(torch.randn(1, 1, dim))
        self.dropout = nn.Dropout(emb_dropout)
        self.transformer = Transformer(dim, depth, heads, dim_head, mlp_dim, dropout, num_patches + 1, mode)
        self.pool = pool
        self.mlp_head = nn.Sequential(nn.LayerNorm(dim), nn.Linear(dim, num_classes))
        # tokens in: num_patches + 1 (HSI bands + the LiDAR band), so that T = N + 1 matches the skipcat
        # Conv2d(num_patches + 2) channels and pos_embedding's num_patches + 2 rows (S2EFT.py:88, :117)
        self.N, self.C, self.D, self.depth, self.heads = num_patches + 1, patch_dim, dim, depth, heads
        self.hidden, self.ncls, self.mode = mlp_dim, num_classes, mode
        self.p_drop, self.p_emb = float(dropout), float(emb_dropout)
        self._build_flat()

    # ------------------------------------------------------------ forward
    def forward(self, x: torch.Tensor, mask=None) -> torch.Tensor:
        if mask is not None:
            raise NotImplementedError("S2EFT mask path is not supported (the reference's raises NameError, :58)")
        if x.device.type != "cuda":
            raise RuntimeError("S2EFT MI355X path: input must be on a ROCm (cuda) device; no CPU fallback")
        if x.dim() != 3 or x.shape[1] != self.N or x.shape[2] != self.C:
            raise RuntimeError(f"expected x [B, {self.N}, {self.C}], got {list(x.shape)}")
        self._ensure_flat()
        if self._flat_store.device != x.device:
            raise RuntimeError("model and input are on different devices")
        x = x.detach().to(torch.float32).contiguous()
        needs_grad = torch.is_grad_enabled() and self._flat_store.requires_grad
        return _S2EFTFunction.apply(self, x, self._flat_store, needs_grad)


class _S2EFTFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model, x, flat, needs_grad):
        prog = _Program(model, x)
        logits = prog.forward()
        ctx.prog = prog if needs_grad else None
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        if ctx.prog is None:
            raise RuntimeError("S2EFT: backward through a forward run without grad")
        grad = ctx.prog.backward(dlogits.detach().to(torch.float32).contiguous())
        ctx.prog = None
        return None, None, grad, None


# the backward's parameter gradients (round 6): 0 = each on the chain where its inputs are made; 1 = each on a side
# stream as soon as its inputs exist (one fork per product); 2 = a layer's parameter gradients queued and forked to
# the side stream once, at the layer's end; 3 = queued and issued on the chain at the layer's end, the layer's
# weight-gradient GEMMs as ONE grouped launch + one grouped split-K reduce (vc_gemm_group_*).  Every GEMM's plan
# depends on its shape and workspace only, and each stream runs its launches in one order: bit-identical results
# in every mode (tests/test_s2eft.py).  Measured (tools/s2eft_step.py, 200 replays x 2, profiles/
# r06_ab_s2eft_side_stream.log): 0: 1.28-1.32 ms, 1: 1.50 ms, 2: 1.35-1.36 ms, 3: 1.173-1.176 ms (default)
_SIDE_STREAM = 3
GEMM_GROUP_BYTES = 16384   # VC_GEMM_GROUP_BYTES (include/vitcnn.h)


class _Program:
    """One forward (saving what the backward reads) and its hand-written backward."""

    SCRATCH = 1 << 22

    def __init__(self, m: ViT, x: torch.Tensor):
        self.m, self.x, self.L = m, x, lib()
        self.dev = x.device
        self.s = torch.cuda.current_stream(self.dev).cuda_stream
        self.B = x.shape[0]
        self.T = m.N + 1
        base = m._flat_store.data_ptr()
        self.P = {n: base + F32 * o for n, o in m._poff.items()}
        self.scr = self.new(self.SCRATCH)
        self.keep = []
        self.pd = m.p_drop if m.training else 0.0
        self.pe = m.p_emb if m.training else 0.0
        self.seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if (self.pd > 0 or self.pe > 0) else 0
        if self.seed:
            # data parallelism: every rank seeds torch alike (main.py), so mix the rank in — the
            # replicas must not apply the same keep masks to their different shards
            from .parallel import rank
            self.seed = (self.seed + 0x9E3779B97F4A7C15 * rank()) % (1 << 62)
        self.masks = {}
        self._group = None

    def drop(self, site, x, add, y, n, p):
        """y = add + dropout_p(x) (add may be None); the keep mask is saved under `site`"""
        mk = torch.empty(n, dtype=torch.uint8, device=self.dev)
        self.L.vc_dropout_fwd(n, x.data_ptr(), add.data_ptr() if add is not None else None, y.data_ptr(),
                              mk.data_ptr(), p, (self.seed + 1000003 * len(self.masks)) % (1 << 63), self.s)
        self.masks[site] = mk

    def new(self, *shape):
        return torch.empty(*shape, dtype=torch.float32, device=self.dev)

    def gemm(self, tA, tB, M, N, K, A, lda, sA, Bm, ldb, sB, beta, C, ldc, sC, batch=1, bias=None, add=None,
             add_ld=0, add_mod=0, bias_grad=None, alpha=1.0, side=None):
        """vc_gemm on the program's stream with its scratch, or (side = (stream handle, scratch pointer)) on the
        backward's weight-gradient stream"""
        st, scr = side if side is not None else (self.s, self.scr.data_ptr())
        if self._group is not None:   # recorded into the open group (launched at vc_gemm_group_end)
            self.L.vc_gemm_group_add(self._group, tA, tB, M, N, K, alpha, A, lda, sA, Bm, ldb, sB, beta, C, ldc, sC,
                                     batch, bias, add, add_ld, add_mod, 0, bias_grad, scr, self.SCRATCH, None, 0)
            return
        self.L.vc_gemm(tA, tB, M, N, K, alpha, A, lda, sA, Bm, ldb, sB, beta, C, ldc, sC, batch, bias, add, add_ld,
                       add_mod, 0, bias_grad, scr, self.SCRATCH, st)

    def ln(self, pfx, X, R, ldx):
        D = self.m.D
        Y, mu, rs = self.new(R, D), self.new(R), self.new(R)
        self.L.vc_layernorm_fwd(R, D, X, ldx, self.P[pfx + ".weight"], self.P[pfx + ".bias"], LN_EPS, Y.data_ptr(), D,
                                mu.data_ptr(), rs.data_ptr(), self.s)
        return Y, mu, rs

    def forward(self):
        m, L, B, T, N, C, D, Hh = self.m, self.L, self.B, self.T, self.m.N, self.m.C, self.m.D, self.m.heads
        R = B * T
        P = self.P
        xg, mask = self.new(B, N, C), self.new(B, N)
        L.vc_s2eft_gate_fwd(B, N, C, self.x.data_ptr(), P["conv2d.weight"], P["conv2d.bias"], 0.4, xg.data_ptr(),
                            mask.data_ptr(), self.s)
        X = self.new(B, T, D)
        L.vc_s2eft_cls_rows(B, T, D, P["cls_token"], P["pos_embedding"], X.data_ptr(), self.s)
        # rows 1..N of every sample: xg W^T + b + pos[1 + t]  (pos fused as the GEMM's row addend)
        self.gemm(0, 1, N, D, C, xg.data_ptr(), C, N * C, P["patch_to_embedding.weight"], C, 0, 0.0,
                  X.data_ptr() + F32 * D, D, T * D, batch=B, bias=P["patch_to_embedding.bias"],
                  add=P["pos_embedding"] + F32 * D, add_ld=D, add_mod=N)
        if self.pe > 0:
            self.drop("emb", X, None, X, R * D, self.pe)
        self.xg = xg
        self.saved = []
        xin = []
        for li in range(m.depth):
            pre = f"transformer.layers.{li}"
            st = {"xin": X}
            xin.append(X)
            if m.mode == "CAF" and li > 1:
                sk = f"transformer.skipcat.{li - 2}"
                Z, bm, Xs = self.new(B, 2 * T, D), self.new(T, D), self.new(B, T, D)
                L.vc_s2eft_skip_pack(B, T, D, X.data_ptr(), xin[li - 2].data_ptr(), P[sk + ".bias"], Z.data_ptr(),
                                     bm.data_ptr(), self.s)
                self.gemm(0, 0, T, D, 2 * T, P[sk + ".weight"], 2 * T, 0, Z.data_ptr(), D, 2 * T * D, 0.0,
                          Xs.data_ptr(), D, T * D, batch=B, add=bm.data_ptr(), add_ld=D, add_mod=T)
                st["Z"] = Z
                X = Xs
            st["xs"] = X
            # attention sub-block
            Y, mu, rs = self.ln(pre + ".0.fn.norm", X.data_ptr(), R, D)
            qkv = self.new(R, 3 * Hh * 16)
            self.gemm(0, 1, R, 3 * Hh * 16, D, Y.data_ptr(), D, 0, P[pre + ".0.fn.fn.to_qkv.weight"], D, 0, 0.0,
                      qkv.data_ptr(), 3 * Hh * 16, 0)
            O, lse = self.new(R, Hh * 16), self.new(B, Hh, T)
            L.vc_s2eft_attn_fwd(B, T, Hh, qkv.data_ptr(), 16 ** -0.5, O.data_ptr(), lse.data_ptr(), self.s)
            X2 = self.new(B, T, D)
            if self.pd > 0:
                A2 = self.new(R, D)
                self.gemm(0, 1, R, D, Hh * 16, O.data_ptr(), Hh * 16, 0, P[pre + ".0.fn.fn.to_out.0.weight"], Hh * 16,
                          0, 0.0, A2.data_ptr(), D, 0, bias=P[pre + ".0.fn.fn.to_out.0.bias"])
                self.drop(f"{li}.attn", A2, X, X2, R * D, self.pd)
            else:
                self.gemm(0, 1, R, D, Hh * 16, O.data_ptr(), Hh * 16, 0, P[pre + ".0.fn.fn.to_out.0.weight"], Hh * 16,
                          0, 0.0, X2.data_ptr(), D, 0, bias=P[pre + ".0.fn.fn.to_out.0.bias"], add=X.data_ptr(),
                          add_ld=D)
            # feed-forward sub-block
            Y2, mu2, rs2 = self.ln(pre + ".1.fn.norm", X2.data_ptr(), R, D)
            Hd = self.new(R, m.hidden)
            self.gemm(0, 1, R, m.hidden, D, Y2.data_ptr(), D, 0, P[pre + ".1.fn.fn.net.0.weight"], D, 0, 0.0,
                      Hd.data_ptr(), m.hidden, 0, bias=P[pre + ".1.fn.fn.net.0.bias"])
            G = self.new(R, m.hidden)
            L.vc_gelu_fwd(R * m.hidden, Hd.data_ptr(), G.data_ptr(), self.s)
            if self.pd > 0:
                self.drop(f"{li}.ff1", G, None, G, R * m.hidden, self.pd)
            X3 = self.new(B, T, D)
            if self.pd > 0:
                F2 = self.new(R, D)
                self.gemm(0, 1, R, D, m.hidden, G.data_ptr(), m.hidden, 0, P[pre + ".1.fn.fn.net.3.weight"], m.hidden,
                          0, 0.0, F2.data_ptr(), D, 0, bias=P[pre + ".1.fn.fn.net.3.bias"])
                self.drop(f"{li}.ff2", F2, X2, X3, R * D, self.pd)
            else:
                self.gemm(0, 1, R, D, m.hidden, G.data_ptr(), m.hidden, 0, P[pre + ".1.fn.fn.net.3.weight"], m.hidden,
                          0, 0.0, X3.data_ptr(), D, 0, bias=P[pre + ".1.fn.fn.net.3.bias"], add=X2.data_ptr(),
                          add_ld=D)
            st.update(Y=Y, mu=mu, rs=rs, qkv=qkv, O=O, lse=lse, X2=X2, Y2=Y2, mu2=mu2, rs2=rs2, Hd=Hd, G=G)
            self.saved.append(st)
            X = X3
        self.Xout = X
        # head on the cls rows (ld T*D)
        Yc, muc, rsc = self.ln("mlp_head.0", X.data_ptr(), B, T * D)
        logits = self.new(B, m.ncls)
        self.gemm(0, 1, B, m.ncls, D, Yc.data_ptr(), D, 0, P["mlp_head.1.weight"], D, 0, 0.0, logits.data_ptr(),
                  m.ncls, 0, bias=P["mlp_head.1.bias"])
        self.head = (Yc, muc, rsc)
        return logits

    def backward(self, dlogits):
        """The hand-written backward.  The data-gradient chain (dX through the layers) runs on the program's
        stream; every weight / bias gradient (the weight-gradient GEMMs with their split-K reduces, the LayerNorm
        parameter reductions, the skipcat and embedding column sums) goes through `side()`, which by default
        (_SIDE_STREAM 3) queues it to the layer's end, where the layer's weight-gradient GEMMs launch as ONE grouped
        grid + one grouped split-K reduce (10 launches -> 2 per layer); it can also run each at once on the chain (0)
        or on a side stream forked from the chain and joined before the gradient is returned (1, 2: measured slower,
        the cross-stream edges cost more than the overlap gains).  The chain never
        writes a buffer the parameter gradients read (the LayerNorm backward writes the residual sum to a new
        buffer: vc_layernorm_bwd_dx with res), and every buffer they read stays referenced until the join.
        Per-launch arithmetic and per-stream order do not depend on the mode: the same bits."""
        m, L, B, T, N, C, D, Hh = self.m, self.L, self.B, self.T, self.m.N, self.m.C, self.m.D, self.m.heads
        R = B * T
        P = self.P
        main = torch.cuda.current_stream(self.dev)
        side_stream = self._side_stream() if _SIDE_STREAM in (1, 2) else main
        scr2 = self.new(self.SCRATCH) if side_stream is not main else self.scr
        sd = (side_stream.cuda_stream, scr2.data_ptr())
        keep, pending = [scr2], []

        def flush():   # the side stream continues after everything issued on the chain so far, runs the queue
            if side_stream is not main:
                ev = torch.cuda.Event()
                ev.record(main)
                side_stream.wait_event(ev)
            if _SIDE_STREAM == 3:   # the queued GEMMs (independent products) as one grouped launch, then the rest
                gemms = [fn for fn in pending if getattr(fn, "func", None) == self.gemm]
                if gemms:
                    self._group = self._group_buf()
                    L.vc_gemm_group_begin(self._group, self.s)
                    try:
                        for fn in gemms:
                            fn()
                    finally:
                        grp, self._group = self._group, None
                        L.vc_gemm_group_end(grp)
                pending[:] = [fn for fn in pending if getattr(fn, "func", None) != self.gemm]
            for fn in pending:
                fn()
            pending.clear()

        def side(bufs, *calls):
            """parameter-gradient work (calls with their arguments bound), reading `bufs`: on the chain now
            (_SIDE_STREAM 0), on the side stream now (1), queued for the layer's end (2, 3)"""
            keep.extend(bufs)
            pending.extend(calls)
            if _SIDE_STREAM not in (2, 3):
                flush()

        grad = self.new(m._n_params)
        L.vc_fill(m._n_params, grad.data_ptr(), 0.0, self.s)
        gb = grad.data_ptr()
        G = {n: gb + F32 * o for n, o in m._poff.items()}
        scr, ns = self.scr.data_ptr(), self.SCRATCH
        part_n = 1024 * 2 * D   # LayerNorm parameter partials (>= the kernel's partial rows: vc_layernorm_bwd's split)

        def ln_bwd(pfx, dY, X, mu, rs, res, rows):
            """dx = res + LN grad into a new buffer (chain); the weight / bias reduction on the side stream"""
            out, part = self.new(rows, D), self.new(part_n)
            L.vc_layernorm_bwd_dx(rows, D, dY.data_ptr(), D, X, D, P[pfx + ".weight"], mu.data_ptr(), rs.data_ptr(),
                                  res, D, out.data_ptr(), D, 0.0, part.data_ptr(), part_n, self.s)
            side((part,), partial(L.vc_layernorm_bwd_params, rows, D, part.data_ptr(), part_n, G[pfx + ".weight"],
                                  G[pfx + ".bias"], 0.0, sd[0]))
            return out

        # head
        Yc, muc, rsc = self.head
        side((dlogits,), partial(self.gemm, 1, 0, m.ncls, D, B, dlogits.data_ptr(), m.ncls, 0, Yc.data_ptr(), D, 0, 0.0,
                                 G["mlp_head.1.weight"], D, 0, bias_grad=G["mlp_head.1.bias"], side=sd))
        dYc = self.new(B, D)
        self.gemm(0, 0, B, D, m.ncls, dlogits.data_ptr(), m.ncls, 0, P["mlp_head.1.weight"], D, 0, 0.0, dYc.data_ptr(),
                  D, 0)
        dX = self.new(B, T, D)
        L.vc_fill(R * D, dX.data_ptr(), 0.0, self.s)
        L.vc_layernorm_bwd(B, D, dYc.data_ptr(), D, self.Xout.data_ptr(), T * D, P["mlp_head.0.weight"], muc.data_ptr(),
                           rsc.data_ptr(), dX.data_ptr(), T * D, 0.0, G["mlp_head.0.weight"], G["mlp_head.0.bias"], 0.0,
                           scr, ns, self.s)
        dlast = {}
        for li in reversed(range(m.depth)):
            pre = f"transformer.layers.{li}"
            st = self.saved[li]
            # feed-forward: X3 = X2 + W2 gelu(W1 LN(X2) + b1) + b2 ; dX holds dX3, then dX2 (a new buffer)
            dG = self.new(R, m.hidden)
            dF2 = dX
            if self.pd > 0:
                dF2 = self.new(R, D)
                L.vc_dropout_bwd(R * D, dX.data_ptr(), self.masks[f"{li}.ff2"].data_ptr(), self.pd, dF2.data_ptr(),
                                 self.s)
            side((dF2,), partial(self.gemm, 1, 0, D, m.hidden, R, dF2.data_ptr(), D, 0, st["G"].data_ptr(), m.hidden, 0,
                                 0.0, G[pre + ".1.fn.fn.net.3.weight"], m.hidden, 0,
                                 bias_grad=G[pre + ".1.fn.fn.net.3.bias"], side=sd))
            self.gemm(0, 0, R, m.hidden, D, dF2.data_ptr(), D, 0, P[pre + ".1.fn.fn.net.3.weight"], m.hidden, 0, 0.0,
                      dG.data_ptr(), m.hidden, 0)
            if self.pd > 0:
                L.vc_dropout_bwd(R * m.hidden, dG.data_ptr(), self.masks[f"{li}.ff1"].data_ptr(), self.pd,
                                 dG.data_ptr(), self.s)
            dH = self.new(R, m.hidden)
            L.vc_gelu_bwd(R * m.hidden, dG.data_ptr(), st["Hd"].data_ptr(), dH.data_ptr(), self.s)
            side((dH,), partial(self.gemm, 1, 0, m.hidden, D, R, dH.data_ptr(), m.hidden, 0, st["Y2"].data_ptr(), D, 0,
                                0.0, G[pre + ".1.fn.fn.net.0.weight"], D, 0, bias_grad=G[pre + ".1.fn.fn.net.0.bias"],
                                side=sd))
            dY2 = self.new(R, D)
            self.gemm(0, 0, R, D, m.hidden, dH.data_ptr(), m.hidden, 0, P[pre + ".1.fn.fn.net.0.weight"], D, 0, 0.0,
                      dY2.data_ptr(), D, 0)
            dX = ln_bwd(pre + ".1.fn.norm", dY2, st["X2"].data_ptr(), st["mu2"], st["rs2"], dX.data_ptr(), R)
            # attention: X2 = Xs + Wo attn(Wqkv LN(Xs)) + bo ; dX holds dX2, then dXs (a new buffer)
            E = Hh * 16
            dA2 = dX
            if self.pd > 0:
                dA2 = self.new(R, D)
                L.vc_dropout_bwd(R * D, dX.data_ptr(), self.masks[f"{li}.attn"].data_ptr(), self.pd, dA2.data_ptr(),
                                 self.s)
            side((dA2,), partial(self.gemm, 1, 0, D, E, R, dA2.data_ptr(), D, 0, st["O"].data_ptr(), E, 0, 0.0,
                                 G[pre + ".0.fn.fn.to_out.0.weight"], E, 0, bias_grad=G[pre + ".0.fn.fn.to_out.0.bias"],
                                 side=sd))
            dO = self.new(R, E)
            self.gemm(0, 0, R, E, D, dA2.data_ptr(), D, 0, P[pre + ".0.fn.fn.to_out.0.weight"], E, 0, 0.0,
                      dO.data_ptr(), E, 0)
            dqkv = self.new(R, 3 * E)
            L.vc_s2eft_attn_bwd(B, T, Hh, st["qkv"].data_ptr(), st["O"].data_ptr(), dO.data_ptr(), st["lse"].data_ptr(),
                                16 ** -0.5, dqkv.data_ptr(), self.s)
            side((dqkv,), partial(self.gemm, 1, 0, 3 * E, D, R, dqkv.data_ptr(), 3 * E, 0, st["Y"].data_ptr(), D, 0, 0.0,
                                  G[pre + ".0.fn.fn.to_qkv.weight"], D, 0, side=sd))
            dY = self.new(R, D)
            self.gemm(0, 0, R, D, 3 * E, dqkv.data_ptr(), 3 * E, 0, P[pre + ".0.fn.fn.to_qkv.weight"], D, 0, 0.0,
                      dY.data_ptr(), D, 0)
            dX = ln_bwd(pre + ".0.fn.norm", dY, st["xs"].data_ptr(), st["mu"], st["rs"], dX.data_ptr(), R)
            # skipcat: Xs[b] = Wm Z[b] + bias  (Wm = weight viewed [T, 2T]); its weight / bias gradients on the side
            if "Z" in st:
                sk = f"transformer.skipcat.{li - 2}"
                dWb = self.new(B, T * 2 * T)
                side((dX, dWb),
                     partial(self.gemm, 0, 1, T, 2 * T, D, dX.data_ptr(), D, T * D, st["Z"].data_ptr(), D, 2 * T * D, 0.0,
                             dWb.data_ptr(), 2 * T, T * 2 * T, batch=B, side=sd),
                     partial(L.vc_colsum, B, T * 2 * T, dWb.data_ptr(), T * 2 * T, G[sk + ".weight"], 0.0, sd[1], ns,
                             sd[0]),
                     partial(L.vc_s2eft_skip_bias_grad, B, T, D, dX.data_ptr(), G[sk + ".bias"], sd[0]))
                dZ = self.new(B, 2 * T, D)
                self.gemm(1, 0, 2 * T, D, T, P[sk + ".weight"], 2 * T, 0, dX.data_ptr(), D, T * D, 0.0, dZ.data_ptr(),
                          D, 2 * T * D, batch=B)
                dlast[li - 2] = self.new(B, T, D)   # written once, by this unpack (layer li - 2's skip gradient)
                dXin = self.new(B, T, D)
                # this layer's input is also last_output[li] of layer li + 2: its gradient folded in here
                L.vc_s2eft_skip_unpack(B, T, D, dZ.data_ptr(), dXin.data_ptr(), 0,
                                       dlast[li].data_ptr() if li in dlast else None, dlast[li - 2].data_ptr(), self.s)
                dX = dXin
            elif li in dlast:  # this layer's input is also last_output[li] of layer li + 2
                L.vc_add2_2d(R, D, dX.data_ptr(), D, dlast[li].data_ptr(), D, dX.data_ptr(), D, 0.0, self.s)
            flush()   # _SIDE_STREAM 2: the layer's parameter gradients, one fork
        # embedding: X0 = dropout(cat(cls, xg W^T + b) + pos)
        if self.pe > 0:
            L.vc_dropout_bwd(R * D, dX.data_ptr(), self.masks["emb"].data_ptr(), self.pe, dX.data_ptr(), self.s)
        dE = self.new(B * N, D)
        L.vc_s2eft_strip_cls(B, N, D, dX.data_ptr(), dE.data_ptr(), self.s)
        side((dX, dE),
             partial(L.vc_colsum, B, T * D, dX.data_ptr(), T * D, G["pos_embedding"], 0.0, sd[1], ns, sd[0]),
             partial(L.vc_colsum, B, D, dX.data_ptr(), T * D, G["cls_token"], 0.0, sd[1], ns, sd[0]),
             partial(self.gemm, 1, 0, D, C, B * N, dE.data_ptr(), D, 0, self.xg.data_ptr(), C, 0, 0.0,
                     G["patch_to_embedding.weight"], C, 0, bias_grad=G["patch_to_embedding.bias"], side=sd))
        flush()
        # join: the gradient is complete when the side stream is; its buffers may go back to the allocator after it
        if side_stream is not main:
            ev = torch.cuda.Event()
            ev.record(side_stream)
            main.wait_event(ev)
        keep.clear()
        return grad

    def _group_buf(self):
        """host memory of the backward's grouped-GEMM state (vc_gemm_group_*: the library keeps none)"""
        buf = self.m.__dict__.get("_vc_group_buf")
        if buf is None:
            buf = ctypes.create_string_buffer(GEMM_GROUP_BYTES)
            self.m.__dict__["_vc_group_buf"] = buf
        return ctypes.addressof(buf)

    def _side_stream(self):
        """the backward's weight-gradient stream: one per model and device"""
        streams = self.m.__dict__.setdefault("_vc_side_streams", {})
        key = str(self.dev)
        if key not in streams:
            streams[key] = torch.cuda.Stream(self.dev)
        return streams[key]
