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


def _nrel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


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
    (4, 11, 256, 256, 1, 256),     # B = 4: tiny grids, deep split-K
    (4, 11, 2193, 256, 1, 2196),   # B = 4 concat conv: ~90 k-slices
    (4, 5, 1024, 256, 0, 1024),    # valid conv at a small spatial size
    (4, 3, 256, 128, 0, 256),      # 3x3 -> 1x1 output
    (4, 11, 144, 256, 1, 144),     # FusAtNet B = 4: the HSI branches' first conv
    (4, 11, 1024, 256, 0, 1024),   # FusAtNet B = 4: the classifier's first (valid) conv
    (4, 3, 256, 1024, 0, 256),     # FusAtNet B = 4: the classifier's last 3x3 conv
    (64, 11, 1024, 256, 0, 1024),  # FusAtNet B = 64: the classifier's convs
    (64, 5, 256, 256, 0, 256),
    (64, 3, 256, 1024, 0, 256),
])
@pytest.mark.parametrize("ws_log2", [0, 22, 24])
def test_conv_tap_fwd_wgrad_dgrad(B, H, C, O, pad, ldx, ws_log2):
    """ws_log2 = 0: no workspace (one k-slice per tile); 22 / 24: split-K slabs limited by a 16 MB /
    64 MB workspace (FusAtNet's scratch) -- every split must give the same answer to fp32 accuracy"""
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
    # device: x with row stride ldx (padding columns filled with garbage the kernel must not read).  With C % 4 != 0
    # and ldx % 4 == 0 the pipelined forward reads the padding up to C rounded to 4 against zero weights: the
    # contract (include/vitcnn.h) is finite values there, so finite garbage
    pad_val = 3.0 if (C % 4 and ldx % 4 == 0) else float("nan")
    xd = torch.full((B * H * H, ldx), pad_val, device=DEV)
    xd[:, :C] = x.reshape(-1, C).to(DEV)
    wd, bd, dyd = w.to(DEV).contiguous(), bias.to(DEV), dy.reshape(-1, O).to(DEV).contiguous()
    s = torch.cuda.current_stream().cuda_stream
    ws = torch.empty(1 << ws_log2, device=DEV) if ws_log2 else None
    wsp, wsn = (ws.data_ptr(), ws.numel()) if ws_log2 else (None, 0)
    Cw = (C + 3) // 4 * 4
    wt = torch.full((O * 9 * Cw,), 5.0, device=DEV)   # the pack must write the padding (as 0)
    w2 = torch.empty(O * 9 * C, device=DEV)
    L.vc_conv3x3_pack(O, C, 0, wd.data_ptr(), wt.data_ptr(), 0.0, s)
    L.vc_conv3x3_pack(O, C, 1, wd.data_ptr(), w2.data_ptr(), 0.0, s)
    w2_ref = w.permute(2, 3, 0, 1).reshape(9, O, C).contiguous()
    y = torch.empty(B * OH * OH, O, device=DEV)
    L.vc_conv3x3_tap_fwd(B, H, H, C, O, pad, xd.data_ptr(), ldx, wt.data_ptr(), bd.data_ptr(), y.data_ptr(), O,
                         wsp, wsn, s)
    dwt = torch.empty(O * 9 * C, device=DEV)
    L.vc_conv3x3_tap_wgrad(B, H, H, C, O, pad, xd.data_ptr(), ldx, dyd.data_ptr(), O, dwt.data_ptr(), wsp,
                           wsn, s)
    dw = torch.full((O, C, 3, 3), 7.0, device=DEV)
    L.vc_conv3x3_pack(O, C, 2, dwt.data_ptr(), dw.data_ptr(), 0.0, s)
    dx = torch.full((B * H * H, ldx), float("nan"), device=DEV)
    dx[:, :C] = dx0.reshape(-1, C).to(DEV)
    L.vc_conv3x3_tap_dgrad(B, H, H, C, O, pad, dyd.data_ptr(), O, wt.data_ptr(), 1.0, dx.data_ptr(), ldx,
                           wsp, wsn, s)
    torch.cuda.synchronize()
    assert torch.equal(w2.cpu().reshape(9, O, C), w2_ref)
    wt_ref = torch.zeros(O, 9, Cw)
    wt_ref[:, :, :C] = w.permute(0, 2, 3, 1).reshape(O, 9, C)
    assert torch.equal(wt.cpu().reshape(O, 9, Cw), wt_ref)
    tol = 2e-6 * (9 * max(C, O)) ** 0.5
    errs = (_rel(y.reshape(B, OH, OH, O), y_ref), _rel(dw, dw_ref), _rel(dx[:, :C].reshape(B, H, H, C), dx_ref),
            _nrel(y.reshape(B, OH, OH, O), y_ref), _nrel(dw, dw_ref), _nrel(dx[:, :C].reshape(B, H, H, C), dx_ref))
    print("errs", errs)
    assert max(errs[:3]) < tol, errs
    # norm-relative: fp32 accumulation over K <= 20k terms stays ~1e-6 of the norm
    assert max(errs[3:]) < 3e-6, errs
    assert torch.isnan(dx[:, C:]).all()          # the row padding is never written
    # the weight gradient stored straight into the torch layout: bit-identical to wgrad + pack mode 2
    dw2 = torch.full((O, C, 3, 3), 7.0, device=DEV)
    L.vc_conv3x3_tap_wgrad_oihw(B, H, H, C, O, pad, xd.data_ptr(), ldx, dyd.data_ptr(), O, dw2.data_ptr(), None,
                                wsp, wsn, s)
    torch.cuda.synchronize()
    assert torch.equal(dw2, dw)
    # ... and with the fused bias gradient: the weight gradient unchanged, db = column sums of dy
    dw3 = torch.full((O, C, 3, 3), 7.0, device=DEV)
    db = torch.full((O,), 9.0, device=DEV)
    L.vc_conv3x3_tap_wgrad_oihw(B, H, H, C, O, pad, xd.data_ptr(), ldx, dyd.data_ptr(), O, dw3.data_ptr(),
                                db.data_ptr(), wsp, wsn, s)
    torch.cuda.synchronize()
    assert torch.equal(dw3, dw)
    db_ref = dy64.sum(dim=(0, 2, 3))
    assert _rel(db, db_ref) < 2e-6 * (B * OH * OH) ** 0.5, _rel(db, db_ref)


@pytest.mark.gpu
def test_conv_pack_many_matches_single_packs():
    """vc_conv3x3_pack_many (one launch per 48 convs) == one vc_conv3x3_pack (mode 0) per conv, bit for bit,
    padding columns written 0; 50 convs so the second launch of the batch runs too"""
    _need_gpu()
    import ctypes
    from vitcnn_amd._lib import lib
    L = lib()
    g = torch.Generator().manual_seed(7)
    shapes = [(1 + (7 * i) % 37, 1 + (13 * i) % 29) for i in range(50)] + [(256, 2193), (16, 1)]
    ws = [torch.randn(O, C, 3, 3, generator=g).to(DEV) for O, C in shapes]
    sizes = [O * 9 * ((C + 3) // 4 * 4) for O, C in shapes]
    one = [torch.full((k,), 5.0, device=DEV) for k in sizes]
    many = [torch.full((k,), 5.0, device=DEV) for k in sizes]
    s = torch.cuda.current_stream().cuda_stream
    for (O, C), w, d in zip(shapes, ws, one):
        L.vc_conv3x3_pack(O, C, 0, w.data_ptr(), d.data_ptr(), 0.0, s)
    n = len(shapes)
    sh = (ctypes.c_int * (2 * n))(*[v for O, C in shapes for v in (O, C)])
    src = (ctypes.c_void_p * n)(*[w.data_ptr() for w in ws])
    dst = (ctypes.c_void_p * n)(*[d.data_ptr() for d in many])
    L.vc_conv3x3_pack_many(n, ctypes.addressof(sh), ctypes.addressof(src), ctypes.addressof(dst), s)
    torch.cuda.synchronize()
    for a, b in zip(one, many):
        assert torch.equal(a, b)
