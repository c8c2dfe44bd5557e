"""Implicit-GEMM 3x3 convolution (csrc/conv_gemm.hip) against torch float64 on the same inputs:
forward with the fused BatchNorm affine / bias / ReLU, the weight + bias gradient, and the data
gradient, for the ViT-CNN (valid, BN-fused) and FusAtNet (padding 1 / 0) shapes plus ragged ones."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"

SHAPES = [
    # B, H, C, O, pad, bn
    (4, 9, 144, 256, 0, True),     # hsi1.local_feature (B reduced)
    (3, 7, 256, 144, 0, True),     # hsi2.local_feature
    (5, 9, 1, 16, 0, True),        # lidar1
    (2, 11, 33, 20, 1, False),     # FusAtNet ConvUnit, ragged channels
    (2, 7, 5, 7, 0, False),        # ragged everything (no float4 path)
    (64, 9, 144, 256, 0, True),    # full hsi1 batch: split-K wgrad
]


def _lib():
    from vitcnn_amd._lib import lib
    return lib()


def _ref(x, w, b, pad, bn):
    """x NHWC float64 -> y NHWC (pre-activation), with the BN affine applied first"""
    if bn is not None:
        mean, inv, g, beta = bn
        x = (x - mean) * (inv * g) + beta
    y = F.conv2d(x.permute(0, 3, 1, 2), w, b, padding=pad)
    return y.permute(0, 2, 3, 1), x


@pytest.mark.parametrize("B,H,C,O,pad,use_bn", SHAPES)
def test_conv3x3_fwd_wgrad_dgrad(B, H, C, O, pad, use_bn):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    L = _lib()
    g = torch.Generator().manual_seed(B * 1000 + H * 100 + C + O)
    x = torch.rand(B, H, H, C, generator=g, dtype=torch.float64)
    w = (torch.rand(O, C, 3, 3, generator=g, dtype=torch.float64) - 0.5) * 0.2
    b = torch.rand(O, generator=g, dtype=torch.float64) - 0.5
    bn = None
    if use_bn:
        bn = (torch.rand(C, generator=g, dtype=torch.float64), torch.rand(C, generator=g, dtype=torch.float64) + 0.5,
              torch.rand(C, generator=g, dtype=torch.float64) + 0.5, torch.rand(C, generator=g, dtype=torch.float64))
    OH = H + 2 * pad - 2
    dy = torch.rand(B, OH, OH, O, generator=g, dtype=torch.float64) - 0.5
    xr = x.clone().requires_grad_(True)
    yref, xbn = _ref(xr, w, b, pad, bn)
    # gradients w.r.t. the (post-BN) conv input, the weight and the bias
    xbn_l = xbn.detach().clone().requires_grad_(True)
    wl, bl = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    y2 = F.conv2d(xbn_l.permute(0, 3, 1, 2), wl, bl, padding=pad).permute(0, 2, 3, 1)
    y2.backward(dy)

    f = lambda t: t.float().contiguous().to(DEV)  # noqa: E731
    xd, wd, bd, dyd = f(x), f(w.reshape(O, 9 * C)), f(b), f(dy)
    bnd = [f(t) for t in bn] if bn is not None else [None] * 4
    bp = [t.data_ptr() if t is not None else None for t in bnd]
    ws = torch.empty(1 << 24, device=DEV)
    s = torch.cuda.current_stream().cuda_stream
    y = torch.empty(B, OH, OH, O, device=DEV)
    L.vc_conv3x3_fwd(B, H, H, C, O, pad, xd.data_ptr(), C, *bp, wd.data_ptr(), bd.data_ptr(), 1, y.data_ptr(), O,
                     ws.data_ptr(), ws.numel(), s)
    dw = torch.full((O, 9 * C), 7.0, device=DEV)
    db = torch.full((O,), 3.0, device=DEV)
    L.vc_conv3x3_wgrad(B, H, H, C, O, pad, xd.data_ptr(), C, *bp, dyd.data_ptr(), O, 1.0, dw.data_ptr(),
                       db.data_ptr(), ws.data_ptr(), ws.numel(), s)
    dx = torch.full((B, H, H, C), 2.0, device=DEV)
    L.vc_conv3x3_dgrad(B, H, H, C, O, pad, dyd.data_ptr(), O, wd.data_ptr(), 1.0, dx.data_ptr(), C, ws.data_ptr(),
                       ws.numel(), s)
    torch.cuda.synchronize()

    def rel(got, ref):
        return float((got.double().cpu() - ref).abs().max() / ref.abs().max().clamp_min(1e-30))

    assert rel(y, yref.detach().clamp_min(0)) < 1e-5
    assert rel(dw - 7.0, wl.grad.reshape(O, 9 * C)) < 1e-5
    assert rel(db - 3.0, bl.grad) < 1e-5
    assert rel(dx - 2.0, xbn_l.grad) < 1e-5


def test_conv3x3_rejects_bad_shapes():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    L = _lib()
    with pytest.raises(RuntimeError):
        L.vc_conv3x3_fwd(1, 2, 2, 4, 4, 0, None, 4, None, None, None, None, None, None, 0, None, 4, None, 0, 0)
    with pytest.raises(RuntimeError):
        L.vc_conv3x3_dgrad(1, 9, 9, 4, 4, 2, None, 4, None, 0.0, None, 4, None, 0, 0)
