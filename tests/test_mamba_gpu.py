"""Mamba mixer kernels (direction gather + conv1d, selective scan, gated combine) vs float64 autograd.

The reference semantics (transformers MambaMixer fallback, modeling_mamba.py:175-283, and the
10-direction gather/gate of Mutimodality_Mamba7.py:642-701) are written out in torch float64 on
the same inputs; the HIP kernels must match to fp32 accuracy (1e-4 relative to each tensor's max).
"""
import math
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vitcnn_amd._lib import lib
    return lib()


def _ref(xz, order, cw, cb, wx, wdt, bdt, alog, dsk, gate, B, L, D, R, ndir):
    """float64 reference of dirconv -> x_proj -> scan -> combine; returns ysum and the leaves."""
    N = 16
    xz = xz.clone().requires_grad_(True)
    leaves = [xz] + [t.clone().requires_grad_(True) for t in (cw, cb, wx, wdt, bdt, alog, dsk, gate)]
    xz_, cw_, cb_, wx_, wdt_, bdt_, alog_, dsk_, gate_ = leaves
    X = xz_.view(B, L, 2 * D)
    g = torch.softmax(gate_, 0)
    ys = 0
    for k in range(ndir):
        o = order[k]
        seq = X[:, o]                                         # [B, L, 2D]
        xs, z = seq[..., :D].transpose(1, 2), seq[..., D:]
        u = torch.nn.functional.conv1d(xs, cw_.view(D, 1, 4), cb_, padding=3, groups=D)[..., :L]
        u = torch.nn.functional.silu(u).transpose(1, 2)      # [B, L, D]
        xd = u @ wx_.t()
        dtl = xd[..., :R] @ wdt_.t() + bdt_
        dt = torch.nn.functional.softplus(dtl)
        A = -torch.exp(alog_)
        h = torch.zeros(B, D, N, dtype=xz.dtype)
        outs = []
        for t in range(L):
            h = torch.exp(A[None] * dt[:, t, :, None]) * h + dt[:, t, :, None] * xd[:, t, None, R:R + N] * u[:, t, :, None]
            outs.append((h * xd[:, t, None, R + N:]).sum(-1))
        y = (torch.stack(outs, 1) + u * dsk_) * torch.nn.functional.silu(z)
        ys = ys + g[k] * y[:, torch.argsort(o)]
    return ys, leaves


def _case(L, D, E):
    """seeded float64 inputs of one mixer shape, the float64 reference output / gradients, and their
    fp32 device copies"""
    torch.manual_seed(0)
    B, ndir, N = 2, 10, 16
    R = math.ceil(E / 16)
    XW = R + 2 * N
    from vitcnn_amd.scan_orders import scan_orders, inverse
    n = int(round(L ** 0.5))
    orders = scan_orders(n)
    order = torch.tensor(orders, dtype=torch.int64)
    f64 = torch.float64
    xz = torch.randn(B * L, 2 * D, dtype=f64)
    cw, cb = torch.randn(D, 4, dtype=f64) * 0.5, torch.randn(D, dtype=f64) * 0.1
    wx = torch.randn(XW, D, dtype=f64) / math.sqrt(D)
    wdt, bdt = torch.randn(D, R, dtype=f64) / math.sqrt(R), torch.randn(D, dtype=f64) * 0.5 - 3.0
    alog = torch.log(torch.arange(1, N + 1, dtype=f64)).repeat(D, 1) + 0.1 * torch.randn(D, N, dtype=f64)
    dsk, gate = 1 + 0.2 * torch.randn(D, dtype=f64), torch.randn(ndir, dtype=f64)
    dys = torch.randn(B * L, D, dtype=f64)
    ys_ref, leaves = _ref(xz, order, cw, cb, wx, wdt, bdt, alog, dsk, gate, B, L, D, R, ndir)
    (ys_ref.reshape(B * L, D) * dys).sum().backward()
    d = lambda t: t.to(torch.float32).contiguous().to(DEV)  # noqa: E731
    c = dict(B=B, ndir=ndir, N=N, R=R, XW=XW, ref=ys_ref.detach().reshape(B * L, D), leaves=leaves,
             o32=torch.tensor(orders, dtype=torch.int32, device=DEV),
             inv32=torch.tensor([inverse(o) for o in orders], dtype=torch.int32, device=DEV))
    for nm, t in (("xz", xz), ("cw", cw), ("cb", cb), ("wx", wx), ("wdt", wdt), ("bdt", bdt), ("alog", alog),
                  ("dsk", dsk), ("gate", gate), ("dys", dys)):
        c[nm] = d(t)
    return c


def _grad_errs(got, leaves):
    names = ["xz", "conv_w", "conv_b", "x_proj", "dt_w", "dt_b", "A_log", "D", "gate"]
    errs = {}
    for nm, g_, leaf in zip(names, got, leaves):
        r = leaf.grad.reshape(g_.shape)
        errs[nm] = float((g_.cpu().double() - r).abs().max() / r.abs().max())
    return errs


@pytest.mark.parametrize("L,D,E", [(81, 72, 144), (49, 72, 144), (121, 72, 144), (49, 128, 256), (25, 40, 80)])
def test_mamba_fused_vs_float64(L, D, E):
    """vc_mamba_scan_fwd_fused (direction conv + x_proj + scan in one launch) and vc_mamba_scan_bwd_fused
    (+ dt_proj / x_proj data gradients + conv1d backward) + the direction gather + the conv parameter
    reduction, against the same float64 reference as the separate kernels; U bit-identical to
    vc_mamba_dirconv_fwd, xdbl equal to the x_proj GEMM's to fp32 rounding."""
    lib = _lib()
    c = _case(L, D, E)
    B, ndir, N, R, XW = c["B"], c["ndir"], c["N"], c["R"], c["XW"]
    s = torch.cuda.current_stream().cuda_stream
    P = lambda t: t.data_ptr()  # noqa: E731
    rows = ndir * B * L
    U, XD, Y = torch.empty(rows, D, device=DEV), torch.empty(rows, XW, device=DEV), torch.empty(rows, D, device=DEV)
    CKP = torch.empty(lib.vc_mamba_scan_ckpt_floats(B, L, D, ndir), device=DEV)
    assert lib.vc_mamba_scan_fwd_fused(B, L, D, R, ndir, P(c["xz"]), P(c["o32"]), P(c["cw"]), P(c["cb"]), P(c["wx"]),
                                       P(c["wdt"]), P(c["bdt"]), P(c["alog"]), P(c["dsk"]), P(U), P(XD), P(Y), P(CKP),
                                       s) == 0
    YS, YP = torch.empty(B * L, D, device=DEV), torch.empty(B * L, D, device=DEV)
    lib.vc_mamba_combine_fwd(B, L, D, ndir, P(c["inv32"]), P(c["gate"]), P(Y), P(c["xz"]), P(YP), P(YS), s)
    U2, XD2 = torch.empty_like(U), torch.empty_like(XD)
    ws = torch.empty(1 << 24, device=DEV)
    lib.vc_mamba_dirconv_fwd(B, L, D, ndir, P(c["o32"]), P(c["xz"]), P(c["cw"]), P(c["cb"]), P(U2), s)
    lib.vc_gemm(0, 1, rows, XW, D, 1.0, P(U2), D, 0, P(c["wx"]), D, 0, 0.0, P(XD2), XW, 0, 1, None, None, 0, 0, 0,
                None, P(ws), ws.numel(), s)
    torch.cuda.synchronize()
    assert torch.equal(U, U2)
    assert float((XD - XD2).abs().max() / XD2.abs().max()) < 1e-6
    err = float((YS.cpu().double() - c["ref"]).abs().max() / c["ref"].abs().max())
    assert err < 1e-5, ("forward", err)

    dU, dDTL = (torch.full((rows, D), float("nan"), device=DEV) for _ in range(2))
    dXD = torch.full((rows, XW), float("nan"), device=DEV)
    CP = torch.full((ndir * B * 5 * D,), float("nan"), device=DEV)
    dXZ = torch.full((B * L, 2 * D), float("nan"), device=DEV)
    dYP = torch.empty(B * L, D, device=DEV)
    dA, dDs, dG = torch.empty(D, N, device=DEV), torch.empty(D, device=DEV), torch.empty(ndir, device=DEV)
    lib.vc_mamba_gate_bwd(B, L, D, P(c["xz"]), P(YP), P(c["dys"]), P(dYP), P(dXZ), s)
    assert lib.vc_mamba_scan_bwd_fused(B, L, D, R, ndir, P(U), P(XD), P(c["o32"]), P(c["xz"]), P(c["cw"]), P(c["cb"]),
                                       P(c["wx"]), P(c["wdt"]), P(c["bdt"]), P(c["alog"]), P(c["dsk"]), P(c["gate"]),
                                       P(Y), P(dYP), P(CKP), P(dU), P(dDTL), P(dXD), P(CP), P(dA), P(dDs), P(dG), P(ws),
                                       ws.numel(), s) == 0
    lib.vc_mamba_dirconv_bwd_gather(B, L, D, ndir, P(c["inv32"]), P(c["cw"]), P(dU), P(dXZ), s)
    dCW, dCB = torch.empty(D, 4, device=DEV), torch.empty(D, device=DEV)
    lib.vc_mamba_conv_params(B, D, ndir, P(CP), P(dCW), P(dCB), s)
    dWdt, dbdt, dWx = torch.empty(D, R, device=DEV), torch.empty(D, device=DEV), torch.empty(XW, D, device=DEV)
    lib.vc_gemm(1, 0, D, R, rows, 1.0, P(dDTL), D, 0, P(XD), XW, 0, 0.0, P(dWdt), R, 0, 1, None, None, 0, 0, 0,
                P(dbdt), P(ws), ws.numel(), s)
    lib.vc_gemm(1, 0, XW, D, rows, 1.0, P(dXD), XW, 0, P(U), D, 0, 0.0, P(dWx), D, 0, 1, None, None, 0, 0, 0, None,
                P(ws), ws.numel(), s)
    torch.cuda.synchronize()
    errs = _grad_errs([dXZ, dCW, dCB, dWx, dWdt, dbdt, dA, dDs, dG], c["leaves"])
    assert max(errs.values()) < 1e-4, errs
    # deferred: the partials left in ws, then every parameter reduction in one launch (vc_mamba_bwd_params)
    assert lib.vc_mamba_scan_bwd_fused(B, L, D, R, ndir, P(U), P(XD), P(c["o32"]), P(c["xz"]), P(c["cw"]), P(c["cb"]),
                                       P(c["wx"]), P(c["wdt"]), P(c["bdt"]), P(c["alog"]), P(c["dsk"]), P(c["gate"]),
                                       P(Y), P(dYP), P(CKP), P(dU), P(dDTL), P(dXD), P(CP), None, None, None, P(ws),
                                       ws.numel(), s) == 0
    qA, qDs, qG = torch.full_like(dA, float("nan")), torch.full_like(dDs, float("nan")), torch.full_like(dG, float("nan"))
    qCW, qCB = torch.full_like(dCW, float("nan")), torch.full_like(dCB, float("nan"))
    assert lib.vc_mamba_bwd_params(B, D, ndir, P(c["gate"]), P(ws), P(CP), P(qA), P(qDs), P(qG), P(qCW), P(qCB), s) == 0
    torch.cuda.synchronize()
    for got, ref in ((qA, dA), (qDs, dDs), (qG, dG), (qCW, dCW), (qCB, dCB)):   # the same sums, another fixed order
        assert float((got - ref).abs().max() / ref.abs().max()) < 1e-5


@pytest.mark.parametrize("L,D,E,use_ckpt", [(81, 72, 144, True), (49, 128, 256, True), (81, 72, 144, False),
                                            (121, 72, 144, True), (25, 40, 80, True)])
def test_mamba_kernels_vs_float64(L, D, E, use_ckpt):
    """(121, 72): the MUUFL-shape hsi1 (11x11 patches); (25, 40): an odd channel count and a
    sequence shorter than 5 checkpoint segments; use_ckpt=False recomputes the states in the
    backward."""
    lib = _lib()
    torch.manual_seed(0)
    B, ndir, N = 2, 10, 16
    R = math.ceil(E / 16)
    XW = R + 2 * N
    from vitcnn_amd.scan_orders import scan_orders, inverse
    n = int(round(L ** 0.5))
    orders = scan_orders(n)
    order = torch.tensor(orders, dtype=torch.int64)
    f64 = torch.float64
    xz = torch.randn(B * L, 2 * D, dtype=f64)
    cw, cb = torch.randn(D, 4, dtype=f64) * 0.5, torch.randn(D, dtype=f64) * 0.1
    wx = torch.randn(XW, D, dtype=f64) / math.sqrt(D)
    wdt, bdt = torch.randn(D, R, dtype=f64) / math.sqrt(R), torch.randn(D, dtype=f64) * 0.5 - 3.0
    alog = torch.log(torch.arange(1, N + 1, dtype=f64)).repeat(D, 1) + 0.1 * torch.randn(D, N, dtype=f64)
    dsk, gate = 1 + 0.2 * torch.randn(D, dtype=f64), torch.randn(ndir, dtype=f64)
    dys = torch.randn(B * L, D, dtype=f64)
    ys_ref, leaves = _ref(xz, order, cw, cb, wx, wdt, bdt, alog, dsk, gate, B, L, D, R, ndir)
    (ys_ref.reshape(B * L, D) * dys).sum().backward()

    d = lambda t: t.to(torch.float32).contiguous().to(DEV)  # noqa: E731
    s = torch.cuda.current_stream().cuda_stream
    P = lambda t: t.data_ptr()  # noqa: E731
    o32 = torch.tensor(orders, dtype=torch.int32, device=DEV)
    inv32 = torch.tensor([inverse(o) for o in orders], dtype=torch.int32, device=DEV)
    xz_d, cw_d, cb_d, wx_d = d(xz), d(cw), d(cb), d(wx)
    wdt_d, bdt_d, alog_d, dsk_d, gate_d = d(wdt), d(bdt), d(alog), d(dsk), d(gate)
    rows = ndir * B * L
    U = torch.empty(rows, D, device=DEV)
    XD = torch.empty(rows, XW, device=DEV)
    Y = torch.empty(rows, D, device=DEV)
    YS = torch.empty(B * L, D, device=DEV)
    ws = torch.empty(1 << 24, device=DEV)
    lib.vc_mamba_dirconv_fwd(B, L, D, ndir, P(o32), P(xz_d), P(cw_d), P(cb_d), P(U), s)
    lib.vc_gemm(0, 1, rows, XW, D, 1.0, P(U), D, 0, P(wx_d), D, 0, 0.0, P(XD), XW, 0, 1, None, None, 0, 0, 0, None,
                P(ws), ws.numel(), s)
    CKP = torch.empty(lib.vc_mamba_scan_ckpt_floats(B, L, D, ndir), device=DEV)
    lib.vc_mamba_scan_fwd(B, L, D, R, ndir, P(U), P(XD), P(o32), P(wdt_d), P(bdt_d), P(alog_d), P(dsk_d), P(Y),
                          P(CKP), s)
    YP = torch.empty(B * L, D, device=DEV)
    lib.vc_mamba_combine_fwd(B, L, D, ndir, P(inv32), P(gate_d), P(Y), P(xz_d), P(YP), P(YS), s)
    torch.cuda.synchronize()
    ref = ys_ref.detach().reshape(B * L, D)
    err = float((YS.cpu().double() - ref).abs().max() / ref.abs().max())
    assert err < 1e-5, ("forward", err)

    dys_d = d(dys)
    dU, dDTL = (torch.empty(rows, D, device=DEV) for _ in range(2))
    dXD = torch.empty(rows, XW, device=DEV)
    dXZ = torch.full((B * L, 2 * D), float("nan"), device=DEV)
    dYP = torch.empty(B * L, D, device=DEV)
    dA, dDs, dG = torch.empty(D, N, device=DEV), torch.empty(D, device=DEV), torch.empty(ndir, device=DEV)
    lib.vc_mamba_gate_bwd(B, L, D, P(xz_d), P(YP), P(dys_d), P(dYP), P(dXZ), s)
    lib.vc_mamba_scan_bwd(B, L, D, R, ndir, P(U), P(XD), P(o32), P(wdt_d), P(bdt_d), P(alog_d), P(dsk_d),
                          P(gate_d), P(Y), P(dYP), P(CKP) if use_ckpt else None, P(dU), P(dDTL), P(dXD), P(dA),
                          P(dDs), P(dG), P(ws), ws.numel(), s)
    if use_ckpt:
        # split form: partials left in a buffer of their own, reduced by vc_mamba_scan_bwd_params (the
        # model's deferred path) == the fused call, bit for bit; du / d(dt_lin) / dxdbl rewritten identically
        nseq = ndir * B
        spn = nseq * D * N + nseq * D + nseq
        sp = torch.full((spn,), float("nan"), device=DEV)
        lib.vc_mamba_scan_bwd(B, L, D, R, ndir, P(U), P(XD), P(o32), P(wdt_d), P(bdt_d), P(alog_d), P(dsk_d),
                              P(gate_d), P(Y), P(dYP), P(CKP), P(dU), P(dDTL), P(dXD), None, None, None, P(sp), spn, s)
        dA2, dD2, dG2 = torch.empty(D, N, device=DEV), torch.empty(D, device=DEV), torch.empty(ndir, device=DEV)
        lib.vc_mamba_scan_bwd_params(B, D, ndir, P(gate_d), P(sp), P(dA2), P(dD2), P(dG2), P(ws), ws.numel(), s)
        torch.cuda.synchronize()
        assert torch.equal(dA2.cpu(), dA.cpu()) and torch.equal(dD2.cpu(), dDs.cpu()) and torch.equal(dG2.cpu(), dG.cpu())
        # the dB / dC reduce-scatter's two forms (bank-masked DPP adds, default; selects + DPP, knob
        # SCAN_SELECT_RS=1 of the probe library) pair the same lanes in the same order: bit-identical outputs
        outs = [t.clone() for t in (dU, dDTL, dXD)]
        from vitcnn_amd._lib import probe_lib
        os.environ["VITCNN_SCAN_SELECT_RS"] = "1"
        try:
            probe_lib().vc_mamba_scan_bwd(B, L, D, R, ndir, P(U), P(XD), P(o32), P(wdt_d), P(bdt_d), P(alog_d), P(dsk_d),
                                  P(gate_d), P(Y), P(dYP), P(CKP), P(dU), P(dDTL), P(dXD), None, None, None, P(sp),
                                  spn, s)
            torch.cuda.synchronize()
        finally:
            del os.environ["VITCNN_SCAN_SELECT_RS"]
        for a_, b_ in zip(outs, (dU, dDTL, dXD)):
            assert torch.equal(a_, b_)
    dWdt, dbdt = torch.empty(D, R, device=DEV), torch.empty(D, device=DEV)
    lib.vc_gemm(0, 0, rows, R, D, 1.0, P(dDTL), D, 0, P(wdt_d), R, 0, 0.0, P(dXD), XW, 0, 1, None, None, 0, 0, 0,
                None, P(ws), ws.numel(), s)
    lib.vc_gemm(1, 0, D, R, rows, 1.0, P(dDTL), D, 0, P(XD), XW, 0, 0.0, P(dWdt), R, 0, 1, None, None, 0, 0, 0,
                P(dbdt), P(ws), ws.numel(), s)
    dWx = torch.empty(XW, D, device=DEV)
    lib.vc_gemm(1, 0, XW, D, rows, 1.0, P(dXD), XW, 0, P(U), D, 0, 0.0, P(dWx), D, 0, 1, None, None, 0, 0, 0, None,
                P(ws), ws.numel(), s)
    lib.vc_gemm(0, 0, rows, D, XW, 1.0, P(dXD), XW, 0, P(wx_d), D, 0, 1.0, P(dU), D, 0, 1, None, None, 0, 0, 0, None,
                P(ws), ws.numel(), s)
    dCW, dCB = torch.empty(D, 4, device=DEV), torch.empty(D, device=DEV)
    lib.vc_mamba_dirconv_bwd(B, L, D, ndir, P(o32), P(inv32), P(xz_d), P(cw_d), P(cb_d), P(dU), P(dXZ),
                             P(dCW), P(dCB), P(ws), ws.numel(), s)
    torch.cuda.synchronize()
    names = ["xz", "conv_w", "conv_b", "x_proj", "dt_w", "dt_b", "A_log", "D", "gate"]
    got = [dXZ, dCW, dCB, dWx, dWdt, dbdt, dA, dDs, dG]
    errs = {}
    for nm, g_, leaf in zip(names, got, leaves):
        r = leaf.grad.reshape(g_.shape)
        errs[nm] = float((g_.cpu().double() - r).abs().max() / r.abs().max())
    assert max(errs.values()) < 1e-4, errs
