"""FusAtNet comparison model (config 5) on the MI355X path.

Reference: `model/compare_method/FusAtNet.py` (`FusAtNet` :168-186), built by `model_utils.py:109-118`
(patch 11, Adam lr 1e-3).  The module keeps the reference's parameter tree and state_dict names.
Forward (train-mode BatchNorm with running-stat updates, or eval-mode) is a program of HIP kernels
over channels-last [B, H, W, C] rows: every 3x3 conv is the tap-major implicit GEMM
`vc_conv3x3_tap_fwd` (conv_tap.hip: operand rows gathered from the channels-last map as float4 runs,
k = tap * C + c, weights repacked tap-major once per step by `vc_conv3x3_pack`, bias fused; no im2col
matrix; all tap-major packs in one `vc_conv3x3_pack_many` launch per step), train-mode BatchNorm + ReLU
`vc_bn_forward_ex` (partial statistics + a fused final/apply launch), residual adds `vc_add2_2d`, pools
`vc_maxpool2_fwd` / `vc_pool_scale`, products `vc_mul2_2d`, the concatenation is written in place.
(The module constant `_TAP_CONV = False` restores the rounds 1-2 formulation, `vc_im2col3x3_pad` +
`vc_gemm`, for measurements.)

Backward: the reference's own autograd raises (the in-place `x += identity` on a saved ReLU output,
:44, :61).  This path defines the out-of-place semantics (`b = relu(bn2(conv2(a)))
+ a`) and runs a hand-written backward over a tape of the forward's ops (conv: `vc_conv3x3_tap_wgrad_oihw`,
the weight gradient stored in the torch layout with the bias gradient fused, through the LDS-DMA
pipelined `conv_pipe` where C and O are multiples of 4; `vc_conv3x3_tap_dgrad` over the tap-major
weights; `vc_bn_bwd_relu_ex`, the ReLU decisions recomputed from the BN input and affine; maxpool,
pooled-scale and product backwards; every gradient buffer written by its first writer with beta 0 instead
of zero-filled); the parameter gradients land in one flat gradient
(`flat_params.grad`) for the fused Adam (vitcnn_amd.optim.AdamW, weight_decay 0).
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn as nn

from ._lib import lib
from .flat import F32, FlatParams
from .model import _IMPLICIT_CONV, N_COUNTERS

# 3x3 convs: the tap-major implicit GEMM (vc_conv3x3_tap_*, conv_tap.hip); False restores the im2col +
# vc_gemm formulation of rounds 1-2 (a module constant: tools/knobs.py sets it from VITCNN_FUSAT_IM2COL=1)
_TAP_CONV = True
# the LiDAR input (C2 bands, 1 at config 5) laid out in rows padded to 4 floats with zero columns, so its 3x3 convs
# take the pipelined conv (conv_tap.hip conv_pipe_ok: 16-B rows) instead of conv_tap
_PAD_LIDAR = True

BN_EPS, BN_MOMENTUM = 1e-5, 0.1
_COUNTER_BUFS = {}


def _counters(dev, stream):
    """one zeroed arrival-counter array per (device, stream) (split-K in-launch combine, BN
    reductions): kernels of one stream run in order and each leaves its counters zero"""
    key = (dev.type, dev.index, stream)
    if key not in _COUNTER_BUFS:
        _COUNTER_BUFS[key] = torch.zeros(N_COUNTERS, dtype=torch.int32, device=dev)
    return _COUNTER_BUFS[key].data_ptr()


class ConvUnit(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, kernel_size=3, padding=1, bias=True)
        self.bn = nn.BatchNorm2d(cout)
        self.activation = nn.ReLU()


class ConvUnit_NP(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, kernel_size=3, bias=True)
        self.bn = nn.BatchNorm2d(cout)
        self.activation = nn.ReLU()


class Residual_Unit1(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, kernel_size=3, padding=1, bias=True)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, kernel_size=3, padding=1, bias=True)
        self.bn2 = nn.BatchNorm2d(cout)
        self.activation = nn.ReLU()
        self.max_pool = nn.MaxPool2d(kernel_size=2, stride=2)


class Residual_Unit2(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, kernel_size=3, padding=1, bias=True)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, kernel_size=3, padding=1, bias=True)
        self.bn2 = nn.BatchNorm2d(cout)
        self.activation = nn.ReLU()


class _SixConv(nn.Module):
    """Hyper_Feature_Extractor / Modality_Feature_Extractor (:64-83, :103-122)"""

    def __init__(self, cin, cout=1024):
        super().__init__()
        self.conv1 = ConvUnit(cin, 256)
        self.conv2 = ConvUnit(256, 256)
        self.conv3 = ConvUnit(256, 256)
        self.conv4 = ConvUnit(256, 256)
        self.conv5 = ConvUnit(256, 256)
        self.conv6 = ConvUnit(256, cout)


class Hyper_Feature_Extractor(_SixConv):
    pass


class Modality_Feature_Extractor(_SixConv):
    pass


class Spectral_Attention_Module(nn.Module):
    def __init__(self, cin, cout=1024):
        super().__init__()
        self.res1 = Residual_Unit1(cin, 256)
        self.res2 = Residual_Unit1(256, 256)
        self.conv1 = ConvUnit(256, 256)
        self.conv2 = ConvUnit(256, cout)
        self.max_pool = nn.MaxPool2d(kernel_size=2, stride=2)
        self.avg_pool = nn.AdaptiveAvgPool2d(1)


class _ResAttention(nn.Module):
    """Spatial_Attention_module / Modality_Attention_Module (:103-117, :124-138)"""

    def __init__(self, cin, cout=1024):
        super().__init__()
        self.res1 = Residual_Unit2(cin, 128)
        self.res2 = Residual_Unit2(128, 256)
        self.conv1 = ConvUnit(256, 256)
        self.conv2 = ConvUnit(256, cout)


class Spatial_Attention_module(_ResAttention):
    pass


class Modality_Attention_Module(_ResAttention):
    pass


class Classification_Module(nn.Module):
    def __init__(self, cin, num_classes):
        super().__init__()
        self.conv1 = ConvUnit_NP(cin, 256)
        self.conv2 = ConvUnit_NP(256, 256)
        self.conv3 = ConvUnit_NP(256, 256)
        self.conv4 = ConvUnit_NP(256, 256)
        self.conv5 = ConvUnit_NP(256, 1024)
        self.conv6 = nn.Conv2d(1024, num_classes, kernel_size=1, bias=True)


class FusAtNet(FlatParams, nn.Module):
    """Same constructor as the reference (FusAtNet.py:168-176); forward(x1 [B,C1,P,P], x2 [B,C2,P,P]).
    Parameters live in one flat buffer (vitcnn_amd.flat): the backward writes one flat gradient, which
    the fused optimizer (vitcnn_amd.optim.AdamW with weight_decay=0: the reference's Adam,
    model_utils.py:109-118) updates in one pass."""

    def __init__(self, input_channels, input_channels2, num_classes):
        super().__init__()
        self.hfe = Hyper_Feature_Extractor(input_channels, 1024)
        self.spectral_am = Spectral_Attention_Module(input_channels, 1024)
        self.spatial_am = Spatial_Attention_module(input_channels2, 1024)
        self.mfe = Modality_Feature_Extractor(1024 * 2 + input_channels + input_channels2, 1024)
        self.mam = Modality_Attention_Module(1024 * 2 + input_channels + input_channels2, 1024)
        self.cm = Classification_Module(1024, num_classes)
        self.c1, self.c2, self.ncls = input_channels, input_channels2, num_classes
        self._build_flat()

    def forward(self, x1: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
        if x1.device.type != "cuda":
            raise RuntimeError("FusAtNet MI355X path: inputs must be on a ROCm (cuda) device; no CPU fallback")
        if x1.dim() != 4 or x1.shape[1] != self.c1 or x1.shape[2] != x1.shape[3]:
            raise RuntimeError(f"expected x1 [B, {self.c1}, P, P], got {list(x1.shape)}")
        if x2.dim() != 4 or x2.shape[0] != x1.shape[0] or x2.shape[1] != self.c2 or x2.shape[2:] != x1.shape[2:]:
            raise RuntimeError(f"expected x2 [B, {self.c2}, P, P] matching x1, got {list(x2.shape)}")
        if x1.shape[2] < 11:
            raise RuntimeError("FusAtNet needs patch >= 11 (five valid 3x3 convs + two 2x2 pools)")
        x1 = x1.detach().float().contiguous()
        x2 = x2.detach().float().contiguous()
        self._ensure_flat()
        if self._flat_store.device != x1.device:
            raise RuntimeError("model and inputs are on different devices")
        if torch.is_grad_enabled() and self._flat_store.requires_grad:
            return _FusAtNetFunction.apply(self, x1, x2, self._flat_store)
        with torch.no_grad():
            return _Program(self, x1, x2, False).run()


class _FusAtNetFunction(torch.autograd.Function):
    """Backward with out-of-place residual semantics (`b = relu(bn2(conv2(a))) + a`): the gradient the
    reference's code would have if its in-place `x += identity` (FusAtNet.py:44, :61) were written
    out of place -- the reference's own autograd raises there."""

    @staticmethod
    def forward(ctx, model, x1, x2, flat):
        prog = _Program(model, x1, x2, True)
        logits = prog.run()
        ctx.prog = prog
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        grad = ctx.prog.backward(dlogits.detach().float().contiguous())
        ctx.prog = None
        return None, None, None, grad


class _Program:
    # split-K slabs of the tap-major conv GEMMs: ~50 MB at B = 64 (sized from the batch, not a
    # fixed 256 MiB), cached per (device, batch) on the model so a forward allocates nothing
    SCRATCH_PER_SAMPLE = 1 << 18      # floats (1 MiB) per sample: 64 MiB at B = 64

    def __init__(self, m: FusAtNet, x1, x2, grad: bool):
        self.m, self.L, self.dev = m, lib(), x1.device
        self.s = torch.cuda.current_stream(self.dev).cuda_stream
        self.B, self.P = x1.shape[0], x1.shape[2]
        self.x1, self.x2 = x1, x2
        self.SCRATCH = max(1 << 22, self.B * self.SCRATCH_PER_SAMPLE)
        key = (str(self.dev), self.SCRATCH)
        cache = m.__dict__.setdefault("_vc_scratch", {})
        if key not in cache:
            cache.clear()
            cache[key] = torch.empty(self.SCRATCH, dtype=torch.float32, device=self.dev)
        self.scr = cache[key]
        self.cnt = _counters(self.dev, self.s)
        self.train = m.training
        self.grad = grad
        self.tape = []        # backward closures, run in reverse
        self.g = {}           # id(activation) -> gradient buffer (grad_of: zero-filled on creation;
                              # acc: left to its first writer, which writes it whole with beta 0)
        self.keep = {}        # id -> activation (keeps ids unique while the tape lives)
        self.no_grad_ids = set()

    def new(self, *shape):
        return torch.empty(*shape, dtype=torch.float32, device=self.dev)

    def grad_of(self, t):
        k = id(t)
        if k not in self.g:
            buf = self.new(t.numel())
            self.L.vc_fill(t.numel(), buf.data_ptr(), 0.0, self.s)
            self.g[k] = buf
        return self.g[k]

    def acc(self, t):
        """(gradient buffer of t, beta) for a writer that covers all of t's gradient: beta 0 on the first
        write (no zero fill), 1 once the buffer holds a contribution"""
        k = id(t)
        if k in self.g:
            return self.g[k], 1.0
        buf = self.new(t.numel())
        self.g[k] = buf
        return buf, 0.0

    def record(self, fn, *acts):
        if self.grad:
            for a in acts:
                self.keep[id(a)] = a
            self.tape.append(fn)

    def add_into(self, dst, src, M, C, ld_dst=None, beta=1.0):
        self.L.vc_add2_2d(M, C, src.data_ptr(), C, None, 0, dst.data_ptr(), ld_dst or C, beta, self.s)

    def acc_into(self, t, src, M, C):
        """t's gradient (+)= src (dense M x C)"""
        g, beta = self.acc(t)
        self.add_into(g, src, M, C, beta=beta)

    def nhwc(self, x, ld=None):
        """x [B, C, H, W] -> channels-last rows of ld >= C floats (columns C .. ld - 1 zero)"""
        B, C, H, W = x.shape
        ld = ld or C
        y = self.new(B, H, W, ld)
        if ld == C:
            self.L.vc_nchw_to_nhwc(B, C, H * W, x.data_ptr(), y.data_ptr(), self.s)
        else:
            self.L.vc_nchw_to_nhwc_pad(B, C, H * W, x.data_ptr(), y.data_ptr(), ld, self.s)
        self.no_grad_ids.add(id(y))
        return y

    def gemm(self, tA, tB, M, N, K, A, lda, Bm, ldb, beta, C, ldc, bias=None, bias_grad=None):
        self.L.vc_gemm_ex(tA, tB, M, N, K, 1.0, A, lda, 0, Bm, ldb, 0, beta, C, ldc, 0, 1, bias, None, 0, 0, 0,
                          bias_grad, self.scr.data_ptr(), self.SCRATCH, self.cnt, N_COUNTERS, self.s)

    def conv3(self, x, ldx, H, C, conv, pad):
        """x [B,H,W,C] rows (ld ldx) -> conv3x3 + bias, [B,OH,OH,O] contiguous.

        Default: the tap-major implicit GEMM (vc_conv3x3_tap_fwd / _wgrad / _dgrad): operand tiles are
        gathered input rows, so neither an im2col matrix (611 MB for the 2193-channel concat) nor a
        col2im pass exists; the weights are repacked tap-major per step (vc_conv3x3_pack, in the
        captured graph) and the tap-major weight gradient unpacked into the flat gradient.
        VITCNN_FUSAT_IM2COL=1: vc_im2col3x3_pad + vc_gemm (rounds 1-2); VITCNN_IMPLICIT_CONV=1 with it:
        the element-gather implicit GEMM vc_conv3x3_*."""
        B, O = self.B, conv.out_channels
        OH = H + 2 * pad - 2
        M, K = B * OH * OH, C * 9
        L, scr = self.L, self.scr.data_ptr()
        y = self.new(B, OH, OH, O)
        wt = None
        if _TAP_CONV:
            wt = self.wts.get(id(conv))   # tap-major weight (rows padded to 4), read again by dgrad
            if wt is None:
                wt = self.new(O * 9 * ((C + 3) // 4 * 4))
                L.vc_conv3x3_pack(O, C, 0, conv.weight.data_ptr(), wt.data_ptr(), 0.0, self.s)
            L.vc_conv3x3_tap_fwd(B, H, H, C, O, pad, x.data_ptr(), ldx, wt.data_ptr(), conv.bias.data_ptr(),
                                 y.data_ptr(), O, scr, self.SCRATCH, self.s)
        elif _IMPLICIT_CONV:
            L.vc_conv3x3_fwd(B, H, H, C, O, pad, x.data_ptr(), ldx, None, None, None, None, conv.weight.data_ptr(),
                             conv.bias.data_ptr(), 0, y.data_ptr(), O, scr, self.SCRATCH, self.s)
        else:
            col = self.new(M, K)
            L.vc_im2col3x3_pad(B, H, H, C, pad, x.data_ptr(), ldx, col.data_ptr(), self.s)
            self.gemm(0, 1, M, O, K, col.data_ptr(), K, conv.weight.data_ptr(), K, 0.0, y.data_ptr(), O,
                      bias=conv.bias.data_ptr())
            del col

        def bwd():
            dy = self.grad_of(y)
            if _TAP_CONV:   # weight gradient in the torch layout and the bias gradient, by the wgrad launch
                L.vc_conv3x3_tap_wgrad_oihw(B, H, H, C, O, pad, x.data_ptr(), ldx, dy.data_ptr(), O,
                                            self.pgrad(conv.weight), self.pgrad(conv.bias), scr, self.SCRATCH, self.s)
                if id(x) not in self.no_grad_ids:   # every row's C columns written (ldx padding never read)
                    gx, beta = self.acc(x)
                    L.vc_conv3x3_tap_dgrad(B, H, H, C, O, pad, dy.data_ptr(), O, wt.data_ptr(), beta, gx.data_ptr(),
                                           ldx, scr, self.SCRATCH, self.s)
                return
            if _IMPLICIT_CONV:
                L.vc_conv3x3_wgrad(B, H, H, C, O, pad, x.data_ptr(), ldx, None, None, None, None, dy.data_ptr(), O,
                                   0.0, self.pgrad(conv.weight), self.pgrad(conv.bias), scr, self.SCRATCH, self.s)
                if id(x) not in self.no_grad_ids:
                    L.vc_conv3x3_dgrad(B, H, H, C, O, pad, dy.data_ptr(), O, conv.weight.data_ptr(), 1.0,
                                       self.grad_of(x).data_ptr(), ldx, scr, self.SCRATCH, self.s)
                return
            colr = self.new(M, K)   # recomputed: cheaper than keeping every im2col matrix
            L.vc_im2col3x3_pad(B, H, H, C, pad, x.data_ptr(), ldx, colr.data_ptr(), self.s)
            self.gemm(1, 0, O, K, M, dy.data_ptr(), O, colr.data_ptr(), K, 0.0, self.pgrad(conv.weight), K,
                      bias_grad=self.pgrad(conv.bias))
            if id(x) in self.no_grad_ids:
                return
            dcol = colr
            self.gemm(0, 0, M, K, O, dy.data_ptr(), O, conv.weight.data_ptr(), K, 0.0, dcol.data_ptr(), K)
            L.vc_col2im3x3_pad(B, H, H, C, pad, dcol.data_ptr(), self.grad_of(x).data_ptr(), ldx, 1, self.s)

        self.record(bwd, x, y) if wt is None else self.record(bwd, x, y, wt)
        return y, OH

    def bn_relu(self, y, M, C, bn, relu=1):
        mean, invstd = self.new(C), self.new(C)
        if self.train:
            self.nbt.append(bn.num_batches_tracked)   # incremented together at the end of run()
        z = self.new(*y.shape) if self.grad else y
        # train: statistics partials + the channel-tiled apply that reduces them (two launches)
        self.L.vc_bn_forward_ex(1 if self.train else 0, M, C, y.data_ptr(), C, bn.eps,
                                bn.momentum if bn.momentum is not None else BN_MOMENTUM, mean.data_ptr(),
                                invstd.data_ptr(), bn.running_mean.data_ptr(), bn.running_var.data_ptr(),
                                bn.weight.data_ptr(), bn.bias.data_ptr(), relu, z.data_ptr(), C, self.scr.data_ptr(),
                                self.SCRATCH, self.cnt, N_COUNTERS, self.s)

        def bwd():
            gy, beta = self.acc(y)
            if relu:   # the ReLU decisions recomputed from y and the affine: z is not read again
                self.L.vc_bn_bwd_relu_ex(1 if self.train else 0, M, C, self.grad_of(z).data_ptr(), C, y.data_ptr(), C,
                                         mean.data_ptr(), invstd.data_ptr(), bn.weight.data_ptr(),
                                         bn.bias.data_ptr(), gy.data_ptr(), C, beta, self.pgrad(bn.weight),
                                         self.pgrad(bn.bias), 0.0, self.scr.data_ptr(), self.SCRATCH, self.cnt,
                                         N_COUNTERS, self.s)
                return
            self.L.vc_bn_bwd_ex(1 if self.train else 0, M, C, self.grad_of(z).data_ptr(), C, y.data_ptr(), C,
                                None, C, mean.data_ptr(), invstd.data_ptr(),
                                bn.weight.data_ptr(), gy.data_ptr(), C, beta, self.pgrad(bn.weight),
                                self.pgrad(bn.bias), 0.0, self.scr.data_ptr(), self.SCRATCH, self.cnt, N_COUNTERS,
                                self.s)

        self.record(bwd, y, z)
        return z

    def pgrad(self, p):
        """address of p's slice of the flat gradient (every parameter is written once, beta 0)"""
        return self.gflat.data_ptr() + F32 * self.poff[id(p)]

    def unit(self, x, ldx, H, C, u, pad=1):
        y, OH = self.conv3(x, ldx, H, C, u.conv, pad)
        return self.bn_relu(y, self.B * OH * OH, u.conv.out_channels, u.bn), OH

    def residual(self, x, ldx, H, C, r, pool):
        a, _ = self.conv3(x, ldx, H, C, r.conv1, 1)
        O = r.conv1.out_channels
        M = self.B * H * H
        a = self.bn_relu(a, M, O, r.bn1)
        b, _ = self.conv3(a, O, H, O, r.conv2, 1)
        b = self.bn_relu(b, M, O, r.bn2)
        out = self.new(*b.shape) if self.grad else b
        self.L.vc_add2_2d(M, O, b.data_ptr(), O, a.data_ptr(), O, out.data_ptr(), O, 0.0, self.s)  # x += identity

        def bwd():
            d = self.grad_of(out)
            self.acc_into(b, d, M, O)
            self.acc_into(a, d, M, O)

        self.record(bwd, a, b, out)
        if not pool:
            return out, H
        return self.maxpool(out, H, O), H // 2

    def maxpool(self, x, H, C):
        y = self.new(self.B, H // 2, H // 2, C)
        arg = torch.empty(y.numel(), dtype=torch.uint8, device=self.dev)
        self.L.vc_maxpool2_fwd(self.B, H, H, C, x.data_ptr(), C, y.data_ptr(), arg.data_ptr(), self.s)

        def bwd():
            gx, beta = self.acc(x)
            # the pool backward writes every input element: straight into x's gradient on its first write
            tmp = gx if beta == 0.0 else self.new(x.numel())
            self.L.vc_maxpool2_bwd(self.B, H, H, C, self.grad_of(y).data_ptr(), arg.data_ptr(), tmp.data_ptr(), C,
                                   self.s)
            if beta != 0.0:
                self.add_into(gx, tmp, self.B * H * H, C)

        self.record(bwd, x, y, arg)
        return y

    def mul(self, a, b, M, C, out, ldo, dout_of):
        """out (ld ldo) = a * b; dout_of() gives (gradient pointer, ld) of out at backward time"""
        self.L.vc_mul2_2d(M, C, a.data_ptr(), C, b.data_ptr(), C, out, ldo, self.s)

        def bwd():
            dptr, ld = dout_of()
            tmp = None
            for t, other in ((a, b), (b, a)):   # dt (+)= dout * other; first write straight into dt
                g, beta = self.acc(t)
                if beta == 0.0:
                    self.L.vc_mul2_2d(M, C, dptr, ld, other.data_ptr(), C, g.data_ptr(), C, self.s)
                else:
                    tmp = tmp if tmp is not None else self.new(M * C)
                    self.L.vc_mul2_2d(M, C, dptr, ld, other.data_ptr(), C, tmp.data_ptr(), C, self.s)
                    self.add_into(g, tmp, M, C)

        self.record(bwd, a, b)

    def six(self, x, ldx, H, C, mod):
        for u in (mod.conv1, mod.conv2, mod.conv3, mod.conv4, mod.conv5, mod.conv6):
            x, _ = self.unit(x, ldx, H, C, u)
            C = ldx = u.conv.out_channels
        return x

    def res_attention(self, x, ldx, H, C, mod):
        x, _ = self.residual(x, ldx, H, C, mod.res1, False)
        x, _ = self.residual(x, 128, H, 128, mod.res2, False)
        x, _ = self.unit(x, 256, H, 256, mod.conv1)
        x, _ = self.unit(x, 256, H, 256, mod.conv2)
        return x

    def pack_all(self):
        """every 3x3 conv's tap-major weights in one arena, packed by one launch (vc_conv3x3_pack_many)"""
        self.wts = {}
        if not _TAP_CONV:
            return
        convs = [c for c in self.m.modules() if isinstance(c, nn.Conv2d) and tuple(c.kernel_size) == (3, 3)]
        sizes = [c.out_channels * 9 * ((c.in_channels + 3) // 4 * 4) for c in convs]
        arena = self.new(sum(sizes))
        self.keep[id(arena)] = arena
        n = len(convs)
        shapes = (ctypes.c_int * (2 * n))(*[v for c in convs for v in (c.out_channels, c.in_channels)])
        src = (ctypes.c_void_p * n)(*[c.weight.data_ptr() for c in convs])
        dst = (ctypes.c_void_p * n)()
        off = 0
        for i, (c, k) in enumerate(zip(convs, sizes)):
            self.wts[id(c)] = arena[off:off + k]
            dst[i] = arena.data_ptr() + F32 * off
            off += k
        self.L.vc_conv3x3_pack_many(n, ctypes.addressof(shapes), ctypes.addressof(src), ctypes.addressof(dst),
                                    self.s)

    def run(self):
        self.nbt = []
        out = self._run()
        if self.nbt:   # every executed BatchNorm's num_batches_tracked += 1: one multi-tensor launch
            torch._foreach_add_(self.nbt, 1)
        return out

    def _run(self):
        m, L, B, P = self.m, self.L, self.B, self.P
        self.pack_all()
        c1, c2 = m.c1, m.c2
        ld2 = (c2 + 3) // 4 * 4 if _PAD_LIDAR else c2
        x1, x2 = self.nhwc(self.x1), self.nhwc(self.x2, ld2)
        HW = P * P
        M = B * HW
        Fhs = self.six(x1, c1, P, c1, m.hfe)                                  # [B,P,P,1024]
        # spectral attention: two pooled residual units, two units, maxpool, global average
        sa = m.spectral_am
        t, H = self.residual(x1, c1, P, c1, sa.res1, True)
        t, H = self.residual(t, 256, H, 256, sa.res2, True)
        t, _ = self.unit(t, 256, H, 256, sa.conv1)
        t, _ = self.unit(t, 256, H, 256, sa.conv2)
        t = self.maxpool(t, H, 1024)
        Hp = H // 2
        Ct = c1 + c2 + 2048
        Cp = (Ct + 3) // 4 * 4    # row stride of the concat: 16-B aligned rows (float4 gathers in conv_tap)
        cat = self.new(B, P, P, Cp)                                           # cat([x1, x2, Ms, Mt], 1)
        self.cat = cat
        # the row padding (Ct .. Cp) zeroed: the pipelined conv's last 16-B chunk of a row reads it against the packed
        # weights' zero padding (conv_tap.hip conv_pipe_ok), so the 2193-channel convs run on conv_pipe
        L.vc_fill_2d(M, Cp - Ct, cat.data_ptr() + F32 * Ct, Cp, 0.0, self.s)
        L.vc_add2_2d(M, c1, x1.data_ptr(), c1, None, 0, cat.data_ptr(), Cp, 0.0, self.s)
        L.vc_add2_2d(M, c2, x2.data_ptr(), ld2, None, 0, cat.data_ptr() + F32 * c1, Cp, 0.0, self.s)
        offs = F32 * (c1 + c2)
        L.vc_pool_scale(B, HW, Hp * Hp, 1024, t.data_ptr(), Fhs.data_ptr(), 1024, cat.data_ptr() + offs, Cp,
                        self.s)                                               # Ms

        def ms_bwd():
            dpooled = self.grad_of(t)
            L.vc_pool_scale_bwd(B, HW, Hp * Hp, 1024, t.data_ptr(), Fhs.data_ptr(), 1024,
                                self.grad_of(cat).data_ptr() + offs, Cp, self.grad_of(Fhs).data_ptr(), 1024,
                                dpooled.data_ptr(), self.s)

        self.record(ms_bwd, t, Fhs, cat)
        Sp = self.res_attention(x2, ld2, P, c2, m.spatial_am)
        offt = F32 * (c1 + c2 + 1024)
        self.mul(Sp, Fhs, M, 1024, cat.data_ptr() + offt, Cp,
                 lambda: (self.grad_of(cat).data_ptr() + offt, Cp))           # Mt
        Fm = self.six(cat, Cp, P, Ct, m.mfe)
        Am = self.res_attention(cat, Cp, P, Ct, m.mam)
        Fss = self.new(B, P, P, 1024) if self.grad else Fm
        self.mul(Fm, Am, M, 1024, Fss.data_ptr(), 1024, lambda: (self.grad_of(Fss).data_ptr(), 1024))
        self.keep[id(Fss)] = Fss
        x, H, C = Fss, P, 1024
        for u in (m.cm.conv1, m.cm.conv2, m.cm.conv3, m.cm.conv4, m.cm.conv5):
            x, H = self.unit(x, C, H, C, u, pad=0)
            C = u.conv.out_channels
        Mo = B * H * H
        logits = self.new(Mo, m.ncls)
        conv6 = m.cm.conv6
        self.gemm(0, 1, Mo, m.ncls, C, x.data_ptr(), C, conv6.weight.data_ptr(), C, 0.0, logits.data_ptr(), m.ncls,
                  bias=conv6.bias.data_ptr())
        self.head = (x, Mo, C)
        if H == 1:
            return logits.view(B, m.ncls).squeeze()                          # torch.squeeze (:165)
        return logits.view(B, H, H, m.ncls).permute(0, 3, 1, 2).squeeze()

    def backward(self, dlogits):
        """the flat gradient of every parameter (zero where the forward does not reach)"""
        m = self.m
        x, Mo, C = self.head
        if dlogits.numel() != Mo * m.ncls or Mo != self.B:
            raise RuntimeError("FusAtNet backward: the classifier output must be 1x1 (patch 11)")
        named = dict(m.named_parameters())
        self.poff = {id(named[n]): o for n, o in m._poff.items()}
        self.gflat = self.new(m._n_params)
        self.L.vc_fill(m._n_params, self.gflat.data_ptr(), 0.0, self.s)
        conv6 = m.cm.conv6
        self.gemm(1, 0, m.ncls, C, Mo, dlogits.data_ptr(), m.ncls, x.data_ptr(), C, 0.0, self.pgrad(conv6.weight), C,
                  bias_grad=self.pgrad(conv6.bias))
        gx, beta = self.acc(x)
        self.gemm(0, 0, Mo, C, m.ncls, dlogits.data_ptr(), m.ncls, conv6.weight.data_ptr(), C, beta, gx.data_ptr(), C)
        for fn in reversed(self.tape):
            fn()
        self.tape, self.g, self.keep = [], {}, {}
        return self.gflat
