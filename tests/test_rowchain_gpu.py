"""hsiMamba row chains (vc_rowchain_front / vc_rowchain_back, rowchain.hip) against the separate launches
they replace (vc_gemm + vc_layernorm_fwd + vc_gemm; vc_mamba_combine_fwd + vc_gemm + vc_layernorm_fwd +
vc_gemm) and a float64 evaluation: every output the backward reads, at both blocks' shapes, with a row
count that leaves a partial 32-row block."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vitcnn_amd._lib import lib
    return lib()


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))


def _ln64(x, w, b, eps):
    mu = x.mean(1, keepdim=True)
    var = ((x - mu) ** 2).mean(1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * w + b, mu.squeeze(1), 1 / torch.sqrt(var.squeeze(1) + eps)


@pytest.mark.parametrize("B,H,K0,E", [(3, 9, 144, 144), (5, 7, 256, 256), (64, 9, 144, 144)])
def test_rowchain_front(B, H, K0, E):
    lib = _lib()
    torch.manual_seed(1)
    L = H * H
    rows, N2 = B * L, E
    x = torch.rand(rows, K0, device=DEV)
    w1 = torch.randn(E, K0, device=DEV) / math.sqrt(K0)
    pos = 0.02 * torch.randn(L, E, device=DEV)
    lw, lb = 1 + 0.1 * torch.randn(E, device=DEV), 0.1 * torch.randn(E, device=DEV)
    w2 = torch.randn(N2, E, device=DEV) / math.sqrt(E)
    P = lambda t: t.data_ptr()  # noqa: E731
    s = torch.cuda.current_stream().cuda_stream
    T, Xn, O = (torch.empty(rows, n, device=DEV) for n in (E, E, N2))
    mu, rs = torch.empty(rows, device=DEV), torch.empty(rows, device=DEV)
    assert lib.vc_rowchain_front(rows, K0, E, N2, P(x), P(w1), P(pos), L, P(T), P(lw), P(lb), 1e-6, P(Xn), P(mu),
                                 P(rs), P(w2), P(O), s) == 0
    torch.cuda.synchronize()
    t64 = x.double() @ w1.double().t() + pos.double().repeat(B, 1)
    xn64, mu64, rs64 = _ln64(t64, lw.double(), lb.double(), 1e-6)
    o64 = xn64 @ w2.double().t()
    assert _rel(T, t64) < 1e-5
    assert _rel(mu, mu64) < 1e-4 and _rel(rs, rs64) < 1e-4
    assert _rel(Xn, xn64) < 1e-4
    assert _rel(O, o64) < 1e-4


@pytest.mark.parametrize("B,H,D,E,N2", [(3, 9, 72, 144, 256), (5, 7, 128, 256, 144), (64, 9, 72, 144, 256)])
def test_rowchain_back(B, H, D, E, N2):
    lib = _lib()
    torch.manual_seed(2)
    L, ndir = H * H, 10
    rows = B * L
    from vitcnn_amd.scan_orders import inverse, scan_orders
    inv = torch.tensor([inverse(o) for o in scan_orders(H)], dtype=torch.int32, device=DEV)
    glog = torch.randn(ndir, device=DEV)
    Y = torch.randn(ndir * rows, D, device=DEV)
    xz = torch.randn(rows, 2 * D, device=DEV)
    w1 = torch.randn(E, D, device=DEV) / math.sqrt(D)
    res = torch.randn(rows, E, device=DEV)
    lw, lb = 1 + 0.1 * torch.randn(E, device=DEV), 0.1 * torch.randn(E, device=DEV)
    w2, b2 = torch.randn(N2, E, device=DEV) / math.sqrt(E), 0.1 * torch.randn(N2, device=DEV)
    P = lambda t: t.data_ptr()  # noqa: E731
    s = torch.cuda.current_stream().cuda_stream
    YP, YS = torch.empty(rows, D, device=DEV), torch.empty(rows, D, device=DEV)
    T2, G, O = (torch.empty(rows, n, device=DEV) for n in (E, E, N2))
    mu, rs = torch.empty(rows, device=DEV), torch.empty(rows, device=DEV)
    assert lib.vc_rowchain_back(B, L, D, ndir, P(inv), P(glog), P(Y), P(xz), P(YP), P(YS), E, P(w1), P(res), P(T2),
                                P(lw), P(lb), 1e-6, P(G), P(mu), P(rs), N2, P(w2), P(b2), P(O), s) == 0
    YP2, YS2 = torch.empty_like(YP), torch.empty_like(YS)
    lib.vc_mamba_combine_fwd(B, L, D, ndir, P(inv), P(glog), P(Y), P(xz), P(YP2), P(YS2), s)
    torch.cuda.synchronize()
    assert torch.equal(YP, YP2) and torch.equal(YS, YS2)
    t64 = YS2.double() @ w1.double().t() + res.double()
    g64, mu64, rs64 = _ln64(t64, lw.double(), lb.double(), 1e-6)
    o64 = g64 @ w2.double().t() + b2.double()
    assert _rel(T2, t64) < 1e-5
    assert _rel(mu, mu64) < 1e-4 and _rel(rs, rs64) < 1e-4
    assert _rel(G, g64) < 1e-4
    assert _rel(O, o64) < 1e-4


def _ln_bwd64(dy, x, w, eps):
    mu = x.mean(1, keepdim=True)
    rs = 1 / torch.sqrt(((x - mu) ** 2).mean(1, keepdim=True) + eps)
    xh = (x - mu) * rs
    g = dy * w
    dx = rs * (g - g.mean(1, keepdim=True) - xh * (g * xh).mean(1, keepdim=True))
    return dx, (dy * xh).sum(0), dy.sum(0), mu.squeeze(1), rs.squeeze(1)


@pytest.mark.parametrize("B,H,Cout,E,D", [(3, 9, 256, 144, 72), (5, 7, 144, 256, 128), (64, 9, 256, 144, 72)])
def test_rowchain_back_bwd(B, H, Cout, E, D):
    """change_dim / ln1 / out_proj data gradients + gate backward + ln1 parameter gradients"""
    lib = _lib()
    torch.manual_seed(3)
    rows = B * H * H
    f64 = torch.float64
    dcd = torch.randn(rows, Cout, device=DEV)
    wcd = torch.randn(Cout, E, device=DEV) / math.sqrt(E)
    t2 = torch.randn(rows, E, device=DEV) + 0.5
    lw = 1 + 0.1 * torch.randn(E, device=DEV)
    wout = torch.randn(E, D, device=DEV) / math.sqrt(D)
    xz, yp = torch.randn(rows, 2 * D, device=DEV), torch.randn(rows, D, device=DEV)
    dg64 = dcd.double() @ wcd.double()
    dt64, dw64, db64, mu64, rs64 = _ln_bwd64(dg64, t2.double(), lw.double(), 1e-6)
    dys64 = dt64 @ wout.double()
    z = xz.double()[:, D:]
    sg = torch.sigmoid(z)
    dyp64 = dys64 * z * sg
    dz64 = dys64 * yp.double() * sg * (1 + z * (1 - sg))
    P = lambda t: t.data_ptr()  # noqa: E731
    s = torch.cuda.current_stream().cuda_stream
    mu, rs = mu64.float().contiguous(), rs64.float().contiguous()
    dT, dYP = torch.empty(rows, E, device=DEV), torch.empty(rows, D, device=DEV)
    dXZ = torch.full((rows, 2 * D), float("nan"), device=DEV)
    part = torch.empty(lib.vc_rowchain_ln_part_floats(rows, E), device=DEV)
    assert lib.vc_rowchain_back_bwd(rows, Cout, E, D, P(dcd), P(wcd), P(t2), P(mu), P(rs), P(lw), P(dT), P(part),
                                    P(wout), P(xz), P(yp), P(dYP), P(dXZ), s) == 0
    dw = torch.empty(2 * E, device=DEV)
    assert lib.vc_rowchain_ln_params(rows, E, P(part), P(dw), P(dw) + 4 * E, 0.0, s) == 0
    torch.cuda.synchronize()
    assert _rel(dT, dt64) < 1e-4
    assert _rel(dYP, dyp64) < 1e-4
    assert _rel(dXZ[:, D:], dz64) < 1e-4
    assert torch.isnan(dXZ[:, :D]).all()   # the x half is the scan backward's
    assert _rel(dw[:E], dw64) < 1e-4 and _rel(dw[E:], db64) < 1e-4


@pytest.mark.parametrize("B,H,E,Cin,with_dx,with_add", [(3, 9, 144, 144, False, False), (5, 7, 256, 256, True, False),
                                                        (64, 7, 256, 256, True, True), (64, 9, 144, 144, True, True)])
def test_rowchain_front_bwd(B, H, E, Cin, with_dx, with_add):
    """in_proj / pre_norm (+ residual) / patch_embed data gradients, dX accumulated; pre_norm parameters"""
    lib = _lib()
    torch.manual_seed(4)
    rows = B * H * H
    dxz = torch.randn(rows, E, device=DEV)
    win = torch.randn(E, E, device=DEV) / math.sqrt(E)
    t = torch.randn(rows, E, device=DEV) - 0.3
    lw = 1 + 0.1 * torch.randn(E, device=DEV)
    res = torch.randn(rows, E, device=DEV)
    wpe = torch.randn(E, Cin, device=DEV) / math.sqrt(Cin)
    dx0 = torch.randn(rows, Cin, device=DEV)
    dxn64 = dxz.double() @ win.double()
    dl64, dw64, db64, mu64, rs64 = _ln_bwd64(dxn64, t.double(), lw.double(), 1e-6)
    dtt64 = dl64 + res.double()
    dxa = torch.randn(rows, Cin, device=DEV)
    dx64 = dx0.double() + dtt64 @ wpe.double() + (dxa.double() if with_add else 0)
    P = lambda t_: t_.data_ptr()  # noqa: E731
    s = torch.cuda.current_stream().cuda_stream
    mu, rs = mu64.float().contiguous(), rs64.float().contiguous()
    dTt = torch.empty(rows, E, device=DEV)
    dX = dx0.clone()
    part = torch.empty(lib.vc_rowchain_ln_part_floats(rows, E), device=DEV)
    assert lib.vc_rowchain_front_bwd(rows, E, E, Cin, P(dxz), P(win), P(t), P(mu), P(rs), P(lw), P(res), P(dTt),
                                     P(part), P(wpe), P(dX) if with_dx else None, 1.0, P(dxa) if with_add else None,
                                     s) == 0
    dw, db = torch.empty(E, device=DEV), torch.empty(E, device=DEV)
    assert lib.vc_rowchain_ln_params(rows, E, P(part), P(dw), P(db), 0.0, s) == 0
    torch.cuda.synchronize()
    assert _rel(dTt, dtt64) < 1e-4
    assert _rel(dw, dw64) < 1e-4 and _rel(db, db64) < 1e-4
    if with_dx:
        assert _rel(dX, dx64) < 1e-4
    else:
        assert torch.equal(dX, dx0)
