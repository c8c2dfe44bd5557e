"""The tap-major implicit-GEMM 3x3 conv (conv_tap.hip) against a float64 PyTorch conv of the same op:
forward (+ bias), weight gradient, data gradient (with accumulation), padding 0 / 1, channel counts
that are not multiples of 4 (FusAtNet's 2193-channel concat, its 1-band LiDAR input), a padded row
stride, and small grids that take the split-K path."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


@pytest.mark.parametrize("B,H,C,O,pad,ldx", [
    (2, 11, 37, 50, 1, 37),        # ragged channels, scalar loads
    (3, 7, 144, 256, 0, 144),      # valid conv (classifier module shapes)
    (2, 11, 2193, 130, 1, 2196),   # the concat: C % 4 != 0, padded row stride
    (4, 11, 1, 16, 1, 1),          # the 1-band LiDAR input
    (2, 5, 512, 64, 1, 512),       # one output tile, long K: split-K path
    (64, 11, 256, 256, 1, 256),    # a full FusAtNet layer at B = 64
])
def test_conv_tap_fwd_wgrad_dgrad(B, H, C, O, pad, ldx):
    _need_gpu()
    from vitcnn_amd._lib import lib
    L = lib()
    g = torch.Generator().manual_seed(B * 1000 + C + O)
    x = torch.randn(B, H, H, C, generator=g)
    w = torch.randn(O, C, 3, 3, generator=g) / (3 * C) ** 0.5
    bias = torch.randn(O, generator=g)
    OH = H + 2 * pad - 2
    dy = torch.randn(B, OH, OH, O, generator=g)
    dx0 = torch.randn(B, H, H, C, generator=g)
    # float64 reference (NCHW)
    x64, w64, dy64 = x.double().permute(0, 3, 1, 2), w.double(), dy.double().permute(0, 3, 1, 2)
    x64.requires_grad_(True)
    w64.requires_grad_(True)
    y64 = F.conv2d(x64, w64, bias.double(), padding=pad)
    y64.backward(dy64)
    y_ref = y64.detach().permute(0, 2, 3, 1)
    dw_ref = w64.grad
    dx_ref = x64.grad.permute(0, 2, 3, 1) + dx0.double()
    # device: x with row stride ldx (padding columns filled with garbage the kernel must not read)
    xd = torch.full((B * H * H, ldx), float("nan"), device=DEV)
    xd[:, :C] = x.reshape(-1, C).to(DEV)
    wd, bd, dyd = w.to(DEV).contiguous(), bias.to(DEV), dy.reshape(-1, O).to(DEV).contiguous()
    s = torch.cuda.current_stream().cuda_stream
    ws = torch.empty(1 << 24, device=DEV)
    wt = torch.empty(O * 9 * C, device=DEV)
    w2 = torch.empty(O * 9 * C, device=DEV)
    L.vc_conv3x3_pack(O, C, 0, wd.data_ptr(), wt.data_ptr(), 0.0, s)
    L.vc_conv3x3_pack(O, C, 1, wd.data_ptr(), w2.data_ptr(), 0.0, s)
    y = torch.empty(B * OH * OH, O, device=DEV)
    L.vc_conv3x3_tap_fwd(B, H, H, C, O, pad, xd.data_ptr(), ldx, wt.data_ptr(), bd.data_ptr(), y.data_ptr(), O,
                         ws.data_ptr(), ws.numel(), s)
    dwt = torch.empty(O * 9 * C, device=DEV)
    L.vc_conv3x3_tap_wgrad(B, H, H, C, O, pad, xd.data_ptr(), ldx, dyd.data_ptr(), O, dwt.data_ptr(), ws.data_ptr(),
                           ws.numel(), s)
    dw = torch.full((O, C, 3, 3), 7.0, device=DEV)
    L.vc_conv3x3_pack(O, C, 2, dwt.data_ptr(), dw.data_ptr(), 0.0, s)
    dx = torch.full((B * H * H, ldx), float("nan"), device=DEV)
    dx[:, :C] = dx0.reshape(-1, C).to(DEV)
    L.vc_conv3x3_tap_dgrad(B, H, H, C, O, pad, dyd.data_ptr(), O, w2.data_ptr(), 1.0, dx.data_ptr(), ldx,
                           ws.data_ptr(), ws.numel(), s)
    torch.cuda.synchronize()
    tol = 2e-6 * (9 * max(C, O)) ** 0.5
    assert _rel(y.reshape(B, OH, OH, O), y_ref) < tol
    assert _rel(dw, dw_ref) < tol
    assert _rel(dx[:, :C].reshape(B, H, H, C), dx_ref) < tol
    assert torch.isnan(dx[:, C:]).all()          # the row padding is never written
