"""Per-kernel parity on the MI355X: every HIP entry point vs a plain PyTorch fp32 CPU reference.

fp32 kernels, tolerance 1e-4 relative to the output's max |value| unless stated.
"""
import ctypes

import numpy as np
import pytest
import torch

from helpers import rel_err

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vitcnn_amd._lib import lib
    return lib()


@pytest.fixture(scope="module")
def probe():
    """libvitcnn_probe.so: the same kernels with the measurement knobs read from VITCNN_* (tests that
    compare two bit-identical forms in one process); the product library reads no environment"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vitcnn_amd._lib import probe_lib
    return probe_lib()


GROUP_BYTES = 16384   # VC_GEMM_GROUP_BYTES


@pytest.fixture(scope="module")
def ws():
    return torch.empty(1 << 24, device=DEV)


def S():
    return torch.cuda.current_stream().cuda_stream


S_ = S   # for tests whose own shape argument is named S


def P(t):
    return t.data_ptr() if t is not None else None


def rnd(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(*shape, generator=g) * 2 - 1) * scale


# vc_gemm flags: bit 0 ReLU, bit 1 bf16 operands (fp32 accumulate), bit 2 / bit 3 / bit 4 force the k-major /
# the K-contiguous / the LDS-DMA pipelined kernel, bit 5 keeps the older kernels (default: chosen by shape);
# bf16: the pipelined kernel's bf16 MFMAs (F_BF16 | F_PIPE) and the K-contiguous kernel's (F_BF16 | F_NOPIPE)
F_BF16, F_LEGACY, F_V2, F_PIPE, F_NOPIPE = 2, 4, 8, 16, 32
KERNELS = [0, F_LEGACY, F_V2, F_PIPE, F_BF16, F_BF16 | F_PIPE, F_BF16 | F_NOPIPE]


def bf16_round(t):
    return t.to(torch.bfloat16).to(torch.float32)


@pytest.mark.parametrize("kern", KERNELS)
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(5184, 144, 144), (37, 41, 9), (1, 16, 128), (130, 70, 1296), (68, 132, 100),
                                   (260, 36, 44), (3136, 256, 1296)])
def test_gemm_layouts(L, ws, kern, ta, tb, M, N, K):
    """fp32 kernels vs the fp32 product; the bf16 kernel vs the fp32 product of the bf16-rounded
    operands (RNE, as torch) - the same products, so only the summation order differs."""
    A = rnd(K, M, seed=1) if ta else rnd(M, K, seed=1)
    B = rnd(N, K, seed=2) if tb else rnd(K, N, seed=2)
    bias = rnd(N, seed=3)
    Ar, Br = (bf16_round(A), bf16_round(B)) if kern & F_BF16 else (A, B)
    ref = (Ar.t() if ta else Ar).double() @ (Br.t() if tb else Br).double() + bias.double()
    Ad, Bd, bd = A.to(DEV), B.to(DEV), bias.to(DEV)
    C = torch.full((M, N), float("nan"), device=DEV)
    lda = M if ta else K
    ldb = K if tb else N
    L.vc_gemm(ta, tb, M, N, K, 1.0, P(Ad), lda, 0, P(Bd), ldb, 0, 0.0, P(C), N, 0, 1, P(bd), None, 0, 0, kern,
              None, P(ws), ws.numel(), S())
    torch.cuda.synchronize()
    assert rel_err(C.cpu().numpy(), ref.float().numpy()) < 1e-5


@pytest.mark.parametrize("kern", KERNELS)
@pytest.mark.parametrize("M,N,K", [(144, 144, 5184), (41, 72, 51840), (256, 1296, 3136)])
def test_gemm_splitk_weight_grad(L, ws, kern, M, N, K):
    # dW[M,N] = dY[K,M]^T X[K,N] accumulated into existing (beta=1)
    dY, X = rnd(K, M, seed=4), rnd(K, N, seed=5)
    C0 = rnd(M, N, seed=6)
    dYr, Xr = (bf16_round(dY), bf16_round(X)) if kern & F_BF16 else (dY, X)
    ref = (dYr.t().double() @ Xr.double() * 0.5 + C0.double()).float()
    C = C0.to(DEV)
    dYd, Xd = dY.to(DEV), X.to(DEV)  # keep device copies alive until the kernel has run
    bg0 = rnd(M, seed=7)
    bg = bg0.to(DEV)
    L.vc_gemm(1, 0, M, N, K, 0.5, P(dYd), M, 0, P(Xd), N, 0, 1.0, P(C), N, 0, 1, None, None, 0, 0, kern,
              P(bg), P(ws), ws.numel(), S())
    torch.cuda.synchronize()
    assert rel_err(C.cpu().numpy(), ref.numpy()) < 1e-5
    # fused bias gradient: column sums of op(A) through the implicit ones column of op(B)
    assert rel_err(bg.cpu().numpy(), (dYr.double().sum(0) * 0.5 + bg0.double()).float().numpy()) < 1e-5


@pytest.mark.parametrize("M,N,K", [(72, 9, 51840), (16, 9, 64), (256, 1296, 200)])
def test_gemm_bias_grad_overwrite(L, ws, M, N, K):
    dY, X = rnd(K, M, seed=14), rnd(K, N, seed=15)
    dYd, Xd = dY.to(DEV), X.to(DEV)
    C = torch.full((M, N), float("nan"), device=DEV)
    bg = torch.full((M,), float("nan"), device=DEV)
    L.vc_gemm(1, 0, M, N, K, 1.0, P(dYd), M, 0, P(Xd), N, 0, 0.0, P(C), N, 0, 1, None, None, 0, 0, 0,
              P(bg), P(ws), ws.numel(), S())
    torch.cuda.synchronize()
    assert rel_err(C.cpu().numpy(), (dY.t() @ X).numpy()) < 1e-5
    assert rel_err(bg.cpu().numpy(), dY.sum(0).numpy()) < 1e-5


@pytest.mark.parametrize("kern", KERNELS)
def test_gemm_batched_relu_addend(L, ws, kern):
    Bt, M, N, K = 64, 49, 256, 81
    A, X = rnd(Bt, M, K, seed=7), rnd(Bt, K, N, seed=8)
    add = rnd(M, N, seed=9)
    rd = bf16_round if kern & F_BF16 else (lambda t: t)
    ref = torch.relu(torch.bmm(rd(A).double(), rd(X).double()) / 81.0).float()
    C = torch.empty(Bt, M, N, device=DEV)
    Ad, Xd = A.to(DEV), X.to(DEV)
    L.vc_gemm(0, 0, M, N, K, 1.0 / 81, P(Ad), K, M * K, P(Xd), N, K * N, 0.0, P(C), N, M * N, Bt,
              None, None, 0, 0, 1 | kern, None, P(ws), ws.numel(), S())
    torch.cuda.synchronize()
    assert rel_err(C.cpu().numpy(), ref.numpy()) < 1e-5
    # addend with row modulo (positional embedding broadcast over the batch)
    A2, W = rnd(4 * M, K, seed=10), rnd(N, K, seed=11)
    ref2 = (rd(A2).double() @ rd(W).double().t() + add.repeat(4, 1).double()).float()
    C2 = torch.empty(4 * M, N, device=DEV)
    A2d, Wd, addd = A2.to(DEV), W.to(DEV), add.to(DEV)
    L.vc_gemm(0, 1, 4 * M, N, K, 1.0, P(A2d), K, 0, P(Wd), K, 0, 0.0, P(C2), N, 0, 1, None,
              P(addd), N, M, kern, None, P(ws), ws.numel(), S())
    torch.cuda.synchronize()
    assert rel_err(C2.cpu().numpy(), ref2.numpy()) < 1e-5


def test_colsum(L, ws):
    X = rnd(51840, 72, seed=12)
    out = torch.ones(72, device=DEV)
    Xd = X.to(DEV)
    L.vc_colsum(51840, 72, P(Xd), 72, P(out), 1.0, P(ws), ws.numel(), S())
    torch.cuda.synchronize()
    assert rel_err(out.cpu().numpy(), (X.sum(0) + 1).numpy()) < 1e-5


@pytest.mark.parametrize("R,C", [(51840, 72), (64, 81 * 144), (256, 72 * 16), (3000, 130), (5, 7)])
def test_colsum_ticketed_is_bit_identical(L, ws, R, C):
    """vc_colsum_ex (last-arriving block of each column group reduces) == vc_colsum (separate
    reduction launch), bit for bit, twice in a row (counters left zero), and against fp64"""
    X = rnd(R, C, seed=R + C)
    Xd = X.to(DEV)
    cnt = torch.zeros(1 << 16, dtype=torch.int32, device=DEV)
    outs = []
    for ex in (False, True, True):
        out = torch.full((C,), 0.25, device=DEV)
        if ex:
            L.vc_colsum_ex(R, C, P(Xd), C, P(out), 2.0, P(ws), ws.numel(), P(cnt), cnt.numel(), S())
        else:
            L.vc_colsum(R, C, P(Xd), C, P(out), 2.0, P(ws), ws.numel(), S())
        torch.cuda.synchronize()
        outs.append(out.cpu())
        assert int(cnt.abs().sum()) == 0
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    assert rel_err(outs[0].numpy(), (X.double().sum(0) + 0.5).numpy()) < 1e-5


@pytest.mark.parametrize("R,C", [(5184, 144), (3136, 256), (7, 144)])
def test_layernorm_bwd_residual_is_bit_identical(L, ws, R, C):
    """vc_layernorm_bwd_res (dx = res + LN grad, res untouched) == vc_layernorm_bwd with dx preset to res
    and beta_dx 1, bit for bit (dw / db accumulated with beta_w 1)"""
    x, dy = (rnd(R, C, seed=3) + 0.5).to(DEV), rnd(R, C, seed=4).to(DEV)
    w, b = (rnd(C, seed=5) + 1).to(DEV), rnd(C, seed=6).to(DEV)
    res = rnd(R, C, seed=7).to(DEV)
    res0 = res.clone()
    y, mean, rstd = torch.empty(R, C, device=DEV), torch.empty(R, device=DEV), torch.empty(R, device=DEV)
    L.vc_layernorm_fwd(R, C, P(x), C, P(w), P(b), 1e-6, P(y), C, P(mean), P(rstd), S())
    outs = []
    for variant in (0, 1):
        dx = res.clone() if variant == 0 else torch.full((R, C), float("nan"), device=DEV)
        dw, db = torch.full((C,), 0.5, device=DEV), torch.full((C,), -0.5, device=DEV)
        if variant == 0:
            L.vc_layernorm_bwd(R, C, P(dy), C, P(x), C, P(w), P(mean), P(rstd), P(dx), C, 1.0, P(dw), P(db), 1.0,
                               P(ws), ws.numel(), S())
        else:
            L.vc_layernorm_bwd_res(R, C, P(dy), C, P(x), C, P(w), P(mean), P(rstd), P(res), C, P(dx), C, P(dw),
                                   P(db), 1.0, P(ws), ws.numel(), S())
        torch.cuda.synchronize()
        outs.append([t.cpu() for t in (dx, dw, db)])
    assert torch.equal(res.cpu(), res0.cpu())
    for a_, b_ in zip(*outs):
        assert torch.equal(a_, b_)
    # the split form (dx now, the parameter reduction later from a buffer of its own) is the same
    part_n = 1024 * 2 * C
    part = torch.full((part_n,), float("nan"), device=DEV)
    dx = torch.full((R, C), float("nan"), device=DEV)
    dw, db = torch.full((C,), 0.5, device=DEV), torch.full((C,), -0.5, device=DEV)
    L.vc_layernorm_bwd_dx(R, C, P(dy), C, P(x), C, P(w), P(mean), P(rstd), P(res), C, P(dx), C, 0.0, P(part), part_n,
                          S())
    L.vc_layernorm_bwd_params(R, C, P(part), part_n, P(dw), P(db), 1.0, S())
    torch.cuda.synchronize()
    for a_, b_ in zip(outs[0], (dx.cpu(), dw.cpu(), db.cpu())):
        assert torch.equal(a_, b_)


@pytest.mark.parametrize("R,C", [(5184, 144), (3136, 256), (100, 256), (7, 144)])
def test_layernorm_fwd_bwd(L, ws, R, C):
    x = rnd(R, C, seed=13, scale=3.0) + 0.5
    w, b = rnd(C, seed=14) + 1, rnd(C, seed=15)
    dy = rnd(R, C, seed=16)
    xr = x.clone().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    y = torch.nn.functional.layer_norm(xr, (C,), wr, br, 1e-6)
    y.backward(dy)
    xd, wd, bd, dyd = x.to(DEV), w.to(DEV), b.to(DEV), dy.to(DEV)
    yd = torch.empty(R, C, device=DEV)
    mean, rstd = torch.empty(R, device=DEV), torch.empty(R, device=DEV)
    L.vc_layernorm_fwd(R, C, P(xd), C, P(wd), P(bd), 1e-6, P(yd), C, P(mean), P(rstd), S())
    dx = torch.ones(R, C, device=DEV)
    dw, db = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
    L.vc_layernorm_bwd(R, C, P(dyd), C, P(xd), C, P(wd), P(mean), P(rstd), P(dx), C, 1.0, P(dw), P(db), 0.0,
                       P(ws), ws.numel(), S())
    torch.cuda.synchronize()
    assert rel_err(yd.cpu().numpy(), y.detach().numpy()) < 1e-5
    assert rel_err(dx.cpu().numpy() - 1, xr.grad.numpy()) < 1e-4
    assert rel_err(dw.cpu().numpy(), wr.grad.numpy()) < 1e-4
    assert rel_err(db.cpu().numpy(), br.grad.numpy()) < 1e-4


@pytest.mark.parametrize("M,C,relu", [(5184, 144, 0), (3136, 512, 1), (5184, 1, 0), (1600, 16, 1)])
def test_batchnorm_train_fwd_bwd(L, ws, M, C, relu):
    x = rnd(M, C, seed=17, scale=2.0) + 0.3
    w, b = rnd(C, seed=18) + 1.0, rnd(C, seed=19)
    dy = rnd(M, C, seed=20)
    rm, rv = rnd(C, seed=21) * 0.1, torch.rand(C) + 0.5
    xr = x.clone().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    rm_ref, rv_ref = rm.clone(), rv.clone()
    # channels-last rows -> NCHW with N=M, H=W=1 has identical BN semantics
    y = torch.nn.functional.batch_norm(xr, rm_ref, rv_ref, wr, br, True, 0.1, 1e-5)
    if relu:
        y = torch.relu(y)
    y.backward(dy)
    xd, wd, bd = x.to(DEV), w.to(DEV), b.to(DEV)
    rmd, rvd = rm.to(DEV), rv.to(DEV)
    mean, inv = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
    L.vc_bn_stats(1, M, C, P(xd), C, 1e-5, 0.1, P(mean), P(inv), P(rmd), P(rvd), P(ws), ws.numel(), S())
    yd = torch.empty(M, C, device=DEV)
    L.vc_bn_apply(M, C, P(xd), C, P(mean), P(inv), P(wd), P(bd), relu, P(yd), C, S())
    dx = torch.empty(M, C, device=DEV)
    dw, db = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
    dyd = dy.to(DEV)
    L.vc_bn_bwd(1, M, C, P(dyd), C, P(xd), C, P(yd) if relu else None, C, P(mean), P(inv), P(wd), P(dx), C,
                0.0, P(dw), P(db), 0.0, P(ws), ws.numel(), S())
    torch.cuda.synchronize()
    assert rel_err(yd.cpu().numpy(), y.detach().numpy()) < 1e-5
    assert rel_err(rmd.cpu().numpy(), rm_ref.numpy()) < 1e-5
    assert rel_err(rvd.cpu().numpy(), rv_ref.numpy()) < 1e-5
    assert rel_err(dx.cpu().numpy(), xr.grad.numpy()) < 1e-4
    assert rel_err(dw.cpu().numpy(), wr.grad.numpy()) < 1e-4
    assert rel_err(db.cpu().numpy(), br.grad.numpy()) < 1e-4


@pytest.mark.parametrize("train", [1, 0])
@pytest.mark.parametrize("M,C,relu", [(5184, 144, 0), (3136, 256, 1), (1600, 16, 1), (37, 200, 1)])
def test_bn_forward_fused_is_bit_identical(L, ws, train, M, C, relu):
    """vc_bn_forward (partials + a channel-tiled apply that reduces them itself) and vc_bn_forward_ex
    with counters (one launch, group barrier; twice: the counters are left zero) == vc_bn_stats +
    vc_bn_apply: y, save_mean / save_invstd and the running statistics, bit for bit"""
    x = (rnd(M, C, seed=61, scale=2.0) + 3.0).to(DEV)
    w, b = (rnd(C, seed=62) + 1.0).to(DEV), rnd(C, seed=63).to(DEV)
    cnt = torch.zeros(1 << 16, dtype=torch.int32, device=DEV)
    outs = []
    for mode in ("split", "two", "one", "one"):
        rm, rv = (rnd(C, seed=64) * 0.1).to(DEV), (rnd(C, seed=65).abs() + 0.5).to(DEV)
        mean, inv = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        y = torch.full((M, C), float("nan"), device=DEV)
        if mode == "one":
            L.vc_bn_forward_ex(train, M, C, P(x), C, 1e-5, 0.1, P(mean), P(inv), P(rm), P(rv), P(w), P(b), relu, P(y),
                               C, P(ws), ws.numel(), P(cnt), cnt.numel(), S())
        elif mode == "two":
            L.vc_bn_forward(train, M, C, P(x), C, 1e-5, 0.1, P(mean), P(inv), P(rm), P(rv), P(w), P(b), relu, P(y), C,
                            P(ws), ws.numel(), S())
        else:
            L.vc_bn_stats(train, M, C, P(x), C, 1e-5, 0.1, P(mean), P(inv), P(rm), P(rv), P(ws), ws.numel(), S())
            L.vc_bn_apply(M, C, P(x), C, P(mean), P(inv), P(w), P(b), relu, P(y), C, S())
        torch.cuda.synchronize()
        outs.append([t.cpu() for t in (y, mean, inv, rm, rv)])
        assert int(cnt.abs().sum()) == 0
    for o in outs[1:]:
        for a_, b_ in zip(outs[0], o):
            assert torch.equal(a_, b_)


@pytest.mark.parametrize("M,C,relu", [(5184, 144, 0), (3136, 512, 1), (5184, 1, 0), (1600, 16, 1), (37, 200, 1)])
def test_batchnorm_ticketed_reduction_is_bit_identical(L, ws, M, C, relu):
    """vc_bn_stats_ex (the last-arriving partial block of each channel group reduces) / vc_bn_bwd_ex
    (one launch: group barrier) == vc_bn_stats / vc_bn_bwd (separate launches), bit for bit, twice in a
    row (the arrival counters are left zero)"""
    x = (rnd(M, C, seed=41, scale=3.0) + 5.0).to(DEV)
    w, dy = (rnd(C, seed=42) + 1.0).to(DEV), rnd(M, C, seed=43).to(DEV)
    relu_out = torch.relu(rnd(M, C, seed=44)).to(DEV) if relu else None
    cnt = torch.zeros(1 << 16, dtype=torch.int32, device=DEV)
    outs = []
    for ex in (False, True):
        for _ in range(2):
            rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
            mean, inv = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
            dx = torch.full((M, C), 0.5, device=DEV)
            dw, db = torch.full((C,), 2.0, device=DEV), torch.full((C,), 3.0, device=DEV)
            sargs = (1, M, C, P(x), C, 1e-5, 0.1, P(mean), P(inv), P(rm), P(rv), P(ws), ws.numel())
            bargs = (1, M, C, P(dy), C, P(x), C, P(relu_out), C, P(mean), P(inv), P(w), P(dx), C, 1.0, P(dw), P(db),
                     0.5, P(ws), ws.numel())
            if ex:
                L.vc_bn_stats_ex(*sargs, P(cnt), cnt.numel(), S())
                L.vc_bn_bwd_ex(*bargs, P(cnt), cnt.numel(), S())
            else:
                L.vc_bn_stats(*sargs, S())
                L.vc_bn_bwd(*bargs, S())
            torch.cuda.synchronize()
            outs.append([t.cpu() for t in (mean, inv, rm, rv, dx, dw, db)])
            assert int(cnt.abs().sum()) == 0
    # the shifted fp64 sums keep a large channel offset (x ~ 5 +- 3) exact to fp32
    xm = x.double().cpu()
    assert torch.allclose(outs[0][0].double(), xm.mean(0), rtol=1e-6, atol=1e-6)
    assert torch.allclose(outs[0][1].double(), 1 / torch.sqrt(xm.var(0, unbiased=False) + 1e-5), rtol=1e-6)
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)


GROUP_PROBLEMS = [
    # ta, tb, M, N, K, batch, bias_grad, beta  (weight / data gradients, batched TokenLearner, split-K)
    (1, 0, 144, 256, 5184, 1, True, 0.0),
    (0, 0, 5184, 144, 256, 1, False, 1.0),
    (0, 1, 3136, 72, 256, 1, False, 0.0),
    (1, 0, 81, 256, 49, 64, False, 0.0),
    (0, 1, 49, 81, 256, 64, False, 0.0),
    (1, 0, 72, 9, 51840, 1, True, 0.0),
    (0, 0, 37, 29, 1000, 1, False, 0.5),
    (1, 1, 50, 70, 300, 1, False, 0.0),
    (0, 0, 64, 64, 64, 1, False, 0.0),
]


# problems the automatic choice sends to the pipelined LDS-DMA kernel (a weight gradient with its bias
# column and K split, a data gradient, a 1x1-conv forward) beside k-major ones
GROUP_PROBLEMS_PIPE = [
    (1, 0, 256, 1296, 3136, 1, True, 0.0),
    (0, 0, 3136, 512, 256, 1, False, 1.0),
    (0, 1, 3136, 256, 512, 1, False, 0.0),
    (1, 0, 72, 9, 5000, 1, True, 0.0),
    (1, 0, 144, 288, 1600, 1, True, 1.0),
]


@pytest.mark.parametrize("n,auto", [(2, False), (3, False), (9, False), (5, True), (14, True)])
def test_gemm_group_is_bit_identical(L, ws, n, auto):
    """vc_gemm_group_begin / _add / _end (one grouped k-major grid, one grouped pipelined grid, one grouped
    split-K reduce, 8 problems of each kind per launch) == the same GEMMs launched one by one, bit for
    bit, including the in-launch combine's counters; `auto`: the automatic kernel choice (pipelined
    problems mixed in), else the k-major kernel forced"""
    probs = (GROUP_PROBLEMS_PIPE + GROUP_PROBLEMS)[:n] if auto else GROUP_PROBLEMS[:n]
    cnt = torch.zeros(1 << 16, dtype=torch.int32, device=DEV)
    ins, outs = [], []
    for i, (ta, tb, M, N, K, batch, bg, beta) in enumerate(probs):
        A = (rnd(batch, K, M, seed=50 + i) if ta else rnd(batch, M, K, seed=50 + i)).to(DEV)
        B = (rnd(batch, N, K, seed=70 + i) if tb else rnd(batch, K, N, seed=70 + i)).to(DEV)
        ins.append((A, B))
    grp = ctypes.create_string_buffer(GROUP_BYTES)
    for grouped in (False, True, True):
        res = []
        if grouped:
            L.vc_gemm_group_begin(ctypes.addressof(grp), S())
        for i, (ta, tb, M, N, K, batch, bg, beta) in enumerate(probs):
            A, B = ins[i]
            C = rnd(batch, M, N, seed=90 + i).to(DEV)
            bgr = torch.full((M,), 0.25, device=DEV) if bg else None
            args = (ta, tb, M, N, K, 1.0, P(A), M if ta else K, A[0].numel(), P(B), K if tb else N, B[0].numel(),
                    beta, P(C), N, C[0].numel(), batch, None, None, 0, 0, 0 if auto else F_LEGACY, P(bgr), P(ws),
                    ws.numel(), P(cnt), cnt.numel())
            if grouped:
                L.vc_gemm_group_add(ctypes.addressof(grp), *args)
            else:
                L.vc_gemm_ex(*args, S())
            res.append((C, bgr))
        if grouped:
            L.vc_gemm_group_end(ctypes.addressof(grp))
        torch.cuda.synchronize()
        outs.append([(c.cpu(), b.cpu() if b is not None else None) for c, b in res])
        assert int(cnt.abs().sum()) == 0
    for o in outs[1:]:
        for (c0, b0), (c1, b1) in zip(outs[0], o):
            assert torch.equal(c0, c1)
            assert b0 is None or torch.equal(b0, b1)
    # and the first problem against a float64 product
    ta, tb, M, N, K, batch, bg, beta = probs[0]
    A, B = ins[0]
    ref = (A[0].double().cpu().T if ta else A[0].double().cpu()) @ (B[0].double().cpu().T if tb else B[0].double().cpu())
    ref = ref + beta * rnd(batch, M, N, seed=90)[0].double()
    assert rel_err(outs[1][0][0][0].numpy(), ref.numpy()) < 1e-5


def test_gemm_group_misuse_raises(L):
    """the group state is the caller's: ending / adding to a group that is not open is an error, and two
    groups are independent (no library state)"""
    g1, g2 = ctypes.create_string_buffer(GROUP_BYTES), ctypes.create_string_buffer(GROUP_BYTES)
    a1, a2 = ctypes.addressof(g1), ctypes.addressof(g2)
    with pytest.raises(RuntimeError):
        L.vc_gemm_group_end(a1)
    L.vc_gemm_group_begin(a1, S())
    L.vc_gemm_group_begin(a2, S())
    L.vc_gemm_group_end(a2)
    L.vc_gemm_group_end(a1)
    with pytest.raises(RuntimeError):
        L.vc_gemm_group_end(a1)
    with pytest.raises(RuntimeError):
        L.vc_gemm_group_add(a1, 0, 0, 4, 4, 4, 1.0, None, 4, 0, None, 4, 0, 0.0, None, 4, 0, 1, None, None, 0, 0, 0,
                            None, None, 0, None, 0)


@pytest.mark.parametrize("kern", KERNELS)
@pytest.mark.parametrize("ta,tb,M,N,K,bgrad", [(1, 0, 72, 9, 51840, True), (1, 0, 256, 1296, 3136, True),
                                               (0, 1, 3136, 256, 1296, False), (1, 0, 41, 72, 51840, False),
                                               (0, 0, 3136, 256, 512, False)])
def test_gemm_ex_in_launch_splitk_is_bit_identical(L, ws, kern, ta, tb, M, N, K, bgrad):
    """vc_gemm_ex (last-arriving slice combines) == vc_gemm (separate reduce kernel), bit for bit,
    and the tile counters are left zero for the next call."""
    A = (rnd(K, M, seed=31) if ta else rnd(M, K, seed=31)).to(DEV)
    B = (rnd(N, K, seed=32) if tb else rnd(K, N, seed=32)).to(DEV)
    lda, ldb = (M if ta else K), (K if tb else N)
    outs = []
    cnt = torch.zeros(1 << 16, dtype=torch.int32, device=DEV)
    for ex in (False, True):
        C = torch.full((M, N), float("nan"), device=DEV)
        bg = torch.full((M,), float("nan"), device=DEV) if bgrad else None
        args = (ta, tb, M, N, K, 1.0, P(A), lda, 0, P(B), ldb, 0, 0.0, P(C), N, 0, 1, None, None, 0, 0, kern,
                P(bg), P(ws), ws.numel())
        for _ in range(2):  # twice: the counters must be back at zero after the first call
            if ex:
                L.vc_gemm_ex(*args, P(cnt), cnt.numel(), S())
            else:
                L.vc_gemm(*args, S())
        torch.cuda.synchronize()
        outs.append((C.cpu(), bg.cpu() if bg is not None else None))
    assert torch.equal(outs[0][0], outs[1][0])
    if bgrad:
        assert torch.equal(outs[0][1], outs[1][1])
    assert int(cnt.abs().sum()) == 0
    rd = bf16_round if kern & F_BF16 else (lambda t: t)
    ref = ((rd(A.t() if ta else A).cpu().double() @ rd(B.t() if tb else B).cpu().double())).float()
    assert rel_err(outs[1][0].numpy(), ref.numpy()) < 1e-5


@pytest.mark.parametrize("B,ncls", [(64, 16), (4, 12), (100, 40), (3, 1)])
def test_weighted_cross_entropy(L, B, ncls):
    """vc_ce_fwd / vc_ce_bwd (16-lane row per sample, several passes when B > 64 or ncls > 16)
    vs torch's weighted CrossEntropyLoss (model_utils.py:311) including an ignore_index target."""
    logits = rnd(B, ncls, seed=41, scale=4.0)
    g = torch.Generator().manual_seed(42)
    target = torch.randint(0, ncls, (B,), generator=g)
    target[0] = -100
    w = torch.rand(ncls, generator=g) + 0.5
    lr = logits.clone().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(lr, target, weight=w, ignore_index=-100)
    ref.backward(torch.tensor(0.75))
    ld, td, wd = logits.to(DEV), target.to(DEV), w.to(DEV)
    loss = torch.empty(1, device=DEV)
    gout = torch.full((1,), 0.75, device=DEV)
    dl = torch.empty(B, ncls, device=DEV)
    L.vc_ce_fwd(B, ncls, P(ld), P(td), P(wd), -100, P(loss), S())
    L.vc_ce_bwd(B, ncls, P(ld), P(td), P(wd), -100, P(gout), P(dl), S())
    torch.cuda.synchronize()
    assert abs(float(loss) - float(ref)) <= 1e-5 * max(1.0, abs(float(ref)))
    assert rel_err(dl.cpu().numpy(), lr.grad.numpy()) < 1e-5
    # the training step's one-launch form (d(loss) = 1) == the two launches, bit for bit
    loss1, dl1 = torch.empty(1, device=DEV), torch.empty(B, ncls, device=DEV)
    one = torch.ones(1, device=DEV)
    L.vc_ce_bwd(B, ncls, P(ld), P(td), P(wd), -100, P(one), P(dl), S())
    L.vc_ce_fwd_bwd(B, ncls, P(ld), P(td), P(wd), -100, P(loss1), P(dl1), S())
    torch.cuda.synchronize()
    assert torch.equal(loss1, loss) and torch.equal(dl1, dl)


@pytest.mark.parametrize("B,S,Pk,Ci", [(3, 49, 9, 128), (2, 25, 4, 72), (2, 81, 16, 64), (2, 49, 9, 70), (1, 7, 1, 4),
                                       (300, 49, 9, 128), (260, 25, 4, 72)])
def test_nonlocal_attention_fwd_bwd(L, B, S, Pk, Ci):
    """vc_nonlocal_attn_fwd / _bwd (NONLocalBlock2D core, Mutimodality_Mamba7.py:140-159: unscaled
    theta . phi^T, softmax over the pooled keys, att . g) vs torch float64 autograd.  Ci % 4 == 0 takes the
    MFMA backward (S^T = phi theta^T tiles, 16 keys x 16 queries) and, from B = 256, the MFMA forward;
    Ci = 70 the wave-per-row kernels."""
    theta = rnd(B * S, Ci, seed=51)
    pooled = rnd(B * Pk, 2 * Ci, seed=52)
    dout = rnd(B * S, Ci, seed=53)
    th = theta.double().view(B, S, Ci).requires_grad_(True)
    pp = pooled.double().view(B, Pk, 2 * Ci).requires_grad_(True)
    att_ref = torch.softmax(th @ pp[..., :Ci].transpose(1, 2), dim=-1)
    o_ref = att_ref @ pp[..., Ci:]
    o_ref.backward(dout.double().view(B, S, Ci))
    td, pd, dd = theta.to(DEV), pooled.to(DEV), dout.to(DEV)
    att = torch.full((B * S * Pk,), float("nan"), device=DEV)
    o = torch.full((B * S, Ci), float("nan"), device=DEV)
    dth = torch.full((B * S, Ci), float("nan"), device=DEV)
    dpp = torch.full((B * Pk, 2 * Ci), float("nan"), device=DEV)
    assert L.vc_nonlocal_attn_fwd(B, S, Pk, Ci, P(td), P(pd), P(att), P(o), S_()) == 0
    assert L.vc_nonlocal_attn_bwd(B, S, Pk, Ci, P(td), P(pd), P(att), P(dd), P(dth), P(dpp), S_()) == 0
    torch.cuda.synchronize()
    assert rel_err(att.cpu().view(B, S, Pk).numpy(), att_ref.detach().numpy()) < 1e-5
    assert rel_err(o.cpu().view(B, S, Ci).numpy(), o_ref.detach().numpy()) < 1e-5
    assert rel_err(dth.cpu().view(B, S, Ci).numpy(), th.grad.numpy()) < 1e-5
    assert rel_err(dpp.cpu().view(B, Pk, 2 * Ci).numpy(), pp.grad.numpy()) < 1e-5


@pytest.mark.parametrize("B,Hs,Ci", [(64, 9, 72), (64, 7, 128), (3, 5, 72), (2, 6, 64), (2, 9, 70)])
def test_nonlocal_pool_bwd_matches_two_launches(L, B, Hs, Ci):
    """vc_nonlocal_attn_pool_bwd (max-pool backward folded into the attention backward) writes exactly what
    vc_nonlocal_attn_bwd + vc_maxpool2_bwd write: every dPG element (prefilled NaN), argmax taps from
    vc_maxpool2_fwd, odd grids' uncovered last row/column 0.  Ci = 70 takes the two-launch fallback."""
    S, Pk = Hs * Hs, (Hs // 2) ** 2
    pg = rnd(B * S, 2 * Ci, seed=61).to(DEV)
    th = rnd(B * S, Ci, seed=62).to(DEV)
    dout = rnd(B * S, Ci, seed=63).to(DEV)
    pp = torch.empty(B * Pk, 2 * Ci, device=DEV)
    pa = torch.empty(B * Pk * 2 * Ci, dtype=torch.uint8, device=DEV)
    att, o = torch.empty(B * S * Pk, device=DEV), torch.empty(B * S, Ci, device=DEV)
    assert L.vc_maxpool2_fwd(B, Hs, Hs, 2 * Ci, P(pg), 2 * Ci, P(pp), P(pa), S_()) == 0
    assert L.vc_nonlocal_attn_fwd(B, S, Pk, Ci, P(th), P(pp), P(att), P(o), S_()) == 0
    dth1, dth2 = (torch.full((B * S, Ci), float("nan"), device=DEV) for _ in range(2))
    dpp = torch.full((B * Pk, 2 * Ci), float("nan"), device=DEV)
    dpg1, dpg2 = (torch.full((B * S, 2 * Ci), float("nan"), device=DEV) for _ in range(2))
    assert L.vc_nonlocal_attn_bwd(B, S, Pk, Ci, P(th), P(pp), P(att), P(dout), P(dth1), P(dpp), S_()) == 0
    assert L.vc_maxpool2_bwd(B, Hs, Hs, 2 * Ci, P(dpp), P(pa), P(dpg1), 2 * Ci, S_()) == 0
    dpp2 = torch.full((B * Pk, 2 * Ci), float("nan"), device=DEV)
    assert L.vc_nonlocal_attn_pool_bwd(B, S, Pk, Ci, Hs, P(th), P(pp), P(att), P(dout), P(pa), P(dth2), P(dpp2),
                                       P(dpg2), S_()) == 0
    torch.cuda.synchronize()
    assert not torch.isnan(dpg2).any()
    assert torch.equal(dth1, dth2) and torch.equal(dpg1, dpg2)


@pytest.mark.parametrize("B,Hs,Ci", [(64, 9, 72), (64, 7, 128), (3, 5, 72), (2, 6, 64), (300, 7, 128)])
def test_nonlocal_pool_fwd_matches_two_launches(L, B, Hs, Ci):
    """vc_nonlocal_attn_pool_fwd (max pool while staging the keys) = vc_maxpool2_fwd + vc_nonlocal_attn_fwd
    bit for bit: att, o, pooled and taps (ties and a NaN planted); B = 300 takes the two-launch MFMA path."""
    S, Pk = Hs * Hs, (Hs // 2) ** 2
    pg = rnd(B * S, 2 * Ci, seed=65)
    pg[1:40:3] = pg[0]               # equal rows -> tied windows
    pg[7, 5] = float("nan")
    pg, th = pg.to(DEV), rnd(B * S, Ci, seed=66).to(DEV)
    outs = []
    for fused in (False, True):
        pp = torch.full((B * Pk, 2 * Ci), float("nan"), device=DEV)
        pa = torch.full((B * Pk * 2 * Ci,), 7, dtype=torch.uint8, device=DEV)
        att = torch.full((B * S * Pk,), float("nan"), device=DEV)
        o = torch.full((B * S, Ci), float("nan"), device=DEV)
        if fused:
            assert L.vc_nonlocal_attn_pool_fwd(B, S, Pk, Ci, Hs, P(th), P(pg), 2 * Ci, P(pp), P(pa), P(att), P(o),
                                               S_()) == 0
        else:
            assert L.vc_maxpool2_fwd(B, Hs, Hs, 2 * Ci, P(pg), 2 * Ci, P(pp), P(pa), S_()) == 0
            assert L.vc_nonlocal_attn_fwd(B, S, Pk, Ci, P(th), P(pp), P(att), P(o), S_()) == 0
        outs.append((pp, pa, att, o))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a.nan_to_num(1e30), b.nan_to_num(1e30))
    assert (outs[1][1] < 4).all()


def test_add2_dup(L):
    """vc_add2_2d_dup: out = out2 = a + b over strided rows (the GLfusion concat gradient)"""
    M, C = 301, 144
    cat = rnd(M, 2 * C, seed=64).to(DEV)
    o1, o2 = torch.full((M, C), float("nan"), device=DEV), torch.full((M, 2 * C), float("nan"), device=DEV)
    assert L.vc_add2_2d_dup(M, C, P(cat), 2 * C, P(cat) + 4 * C, 2 * C, P(o1), C, P(o2), 2 * C, S_()) == 0
    torch.cuda.synchronize()
    ref = cat[:, :C] + cat[:, C:]
    assert torch.equal(o1, ref) and torch.equal(o2[:, :C], ref) and torch.isnan(o2[:, C:]).all()


@pytest.mark.parametrize("B,H,C", [(64, 9, 144), (64, 7, 256), (3, 11, 64), (2, 5, 70), (1, 33, 16)])
def test_im2col_col2im_lds_forms(probe, B, H, C, monkeypatch):
    """vc_im2col3x3 (BN affine folded) / vc_col2im3x3: the LDS-staged forms (chunks of <= 32 channels per
    block) equal the per-thread forms (VITCNN_C2I_LDS=0) bit for bit and torch's unfold / fold; H = 33
    exceeds the LDS budget and keeps the per-thread kernels."""
    import torch.nn.functional as F
    OH = H - 2
    x = rnd(B * H * H, C, seed=71).to(DEV)
    mean, inv = rnd(C, seed=72).to(DEV), (rnd(C, seed=73).abs() + 0.5).to(DEV)
    w, b = rnd(C, seed=74).to(DEV), rnd(C, seed=75).to(DEV)
    dcol = rnd(B * OH * OH, 9 * C, seed=76).to(DEV)
    outs = []
    for lds in ("1", "0"):
        monkeypatch.setenv("VITCNN_C2I_LDS", lds)
        col = torch.full((B * OH * OH, 9 * C), float("nan"), device=DEV)
        dx = torch.full((B * H * H, C), float("nan"), device=DEV)
        assert probe.vc_im2col3x3(B, H, H, C, P(x), P(mean), P(inv), P(w), P(b), P(col), S()) == 0
        assert probe.vc_col2im3x3(B, H, H, C, P(dcol), P(dx), S()) == 0
        torch.cuda.synchronize()
        outs.append((col, dx))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    sc = inv * w
    xn = (x.double() * sc.double() + (b - mean * sc).double()).view(B, H, H, C).permute(0, 3, 1, 2)
    ref_col = F.unfold(xn, 3).permute(0, 2, 1).reshape(B * OH * OH, 9 * C)
    assert rel_err(outs[0][0].cpu().numpy(), ref_col.cpu().numpy()) < 1e-6
    ref_dx = F.fold(dcol.double().view(B, OH * OH, 9 * C).permute(0, 2, 1), (H, H), 3)
    ref_dx = ref_dx.permute(0, 2, 3, 1).reshape(B * H * H, C)
    assert rel_err(outs[0][1].cpu().numpy(), ref_dx.cpu().numpy()) < 1e-6


@pytest.mark.parametrize("B,H,C", [(64, 9, 144), (64, 7, 256), (3, 11, 64), (2, 5, 70), (1, 33, 16)])
def test_bn_im2col_matches_stats_then_im2col(L, B, H, C):
    """vc_bn_im2col3x3 (the BatchNorm statistics' final reduction inside the im2col launch) = train-mode
    vc_bn_stats_ex + vc_im2col3x3 bit for bit: save_mean / save_invstd, the running statistics and the
    col matrix; H = 33 exceeds the LDS budget and takes the three launches."""
    OH = H - 2
    x = (rnd(B * H * H, C, seed=81, scale=2.0) + 3.0).to(DEV)
    w, b = rnd(C, seed=82).to(DEV), rnd(C, seed=83).to(DEV)
    outs = []
    for fused in (True, False):
        sm, si = torch.full((C,), float("nan"), device=DEV), torch.full((C,), float("nan"), device=DEV)
        rm, rv = torch.full((C,), 0.25, device=DEV), torch.full((C,), 1.5, device=DEV)
        col = torch.full((B * OH * OH, 9 * C), float("nan"), device=DEV)
        ws = torch.empty(1 << 22, device=DEV)
        if fused:
            assert L.vc_bn_im2col3x3(B, H, H, C, P(x), 1e-5, 0.1, P(sm), P(si), P(rm), P(rv), P(w), P(b), P(col),
                                     P(ws), ws.numel(), S()) == 0
        else:
            assert L.vc_bn_stats_ex(1, B * H * H, C, P(x), C, 1e-5, 0.1, P(sm), P(si), P(rm), P(rv), P(ws),
                                    ws.numel(), None, 0, S()) == 0
            assert L.vc_im2col3x3(B, H, H, C, P(x), P(sm), P(si), P(w), P(b), P(col), S()) == 0
        torch.cuda.synchronize()
        outs.append((sm, si, rm, rv, col))
    for a_, b_ in zip(*outs):
        assert torch.equal(a_, b_)
    xd = x.double()
    assert rel_err(outs[0][0].cpu().numpy(), xd.mean(0).cpu().numpy()) < 1e-6


@pytest.mark.parametrize("M,C", [(5184, 128), (3136, 128), (100, 72)])
def test_bn_glf_combine_matches_stats_then_combine(L, M, C):
    """vc_bn_glf_combine (BN(W y) statistics finished inside the GLfusion combine) = train-mode
    vc_bn_stats_ex + vc_glf_combine_fwd bit for bit (save_*, running statistics, the [M, 2C] output)."""
    wp = (rnd(M, C, seed=91, scale=0.5) + 1.0).to(DEV)
    fc, fl = rnd(M, C, seed=92).to(DEV), rnd(M, C, seed=93).to(DEV)
    g, bt = rnd(C, seed=94).to(DEV), rnd(C, seed=95).to(DEV)
    outs = []
    for fused in (True, False):
        sm, si = torch.full((C,), float("nan"), device=DEV), torch.full((C,), float("nan"), device=DEV)
        rm, rv = torch.full((C,), 0.25, device=DEV), torch.full((C,), 1.5, device=DEV)
        out = torch.full((M, 2 * C), float("nan"), device=DEV)
        ws = torch.empty(1 << 22, device=DEV)
        if fused:
            assert L.vc_bn_glf_combine(M, C, P(wp), 1e-5, 0.1, P(sm), P(si), P(rm), P(rv), P(g), P(bt), P(fc), P(fl),
                                       P(out), P(ws), ws.numel(), S()) == 0
        else:
            assert L.vc_bn_stats_ex(1, M, C, P(wp), C, 1e-5, 0.1, P(sm), P(si), P(rm), P(rv), P(ws), ws.numel(),
                                    None, 0, S()) == 0
            assert L.vc_glf_combine_fwd(M, C, P(wp), P(sm), P(si), P(g), P(bt), P(fc), P(fl), P(out), S()) == 0
        torch.cuda.synchronize()
        outs.append((sm, si, rm, rv, out))
    for a_, b_ in zip(*outs):
        assert torch.equal(a_, b_)


@pytest.mark.parametrize("M,N,K,bf", [(3136, 256, 512, 0), (1600, 144, 288, 0), (3136, 128, 272, 0),
                                     (1600, 128, 176, 0), (130, 72, 40, 0), (3136, 256, 512, 1)])
def test_gemm_colstats_and_bn_apply_partials(L, M, N, K, bf):
    """vc_gemm_colstats (conv1x1 with the BatchNorm statistics partials in the GEMM epilogue) + vc_bn_apply_partials
    == the GEMM, then train-mode BatchNorm2d + ReLU, in float64 (running statistics included)"""
    A = (rnd(M, K, seed=71) + 0.3).to(DEV)
    W = (rnd(N, K, seed=72) * 0.2).to(DEV)
    bias = (rnd(N, seed=73) + 2.0).to(DEV)
    g, bb = (rnd(N, seed=74) + 1.0).to(DEV), rnd(N, seed=75).to(DEV)
    P_ = -(-M // 64)
    pre = torch.full((M, N), float("nan"), device=DEV)
    cs = torch.full((2 * P_ * N,), float("nan"), dtype=torch.float64, device=DEV)
    assert L.vc_gemm_colstats(M, N, K, P(A), K, P(W), K, P(bias), P(pre), N, 2 if bf else 0, P(cs), S()) == 0
    rm, rv = torch.zeros(N, device=DEV), torch.ones(N, device=DEV)
    mean, inv = torch.empty(N, device=DEV), torch.empty(N, device=DEV)
    y = torch.full((M, N), float("nan"), device=DEV)
    assert L.vc_bn_apply_partials(M, N, P(pre), N, P_, P(cs), P(bias), 1e-5, 0.1, P(mean), P(inv), P(rm), P(rv), P(g),
                                  P(bb), 1, P(y), N, S()) == 0
    torch.cuda.synchronize()
    A64, W64 = A.cpu().double(), W.cpu().double()
    if bf:   # the bf16 operands the MFMAs see
        A64, W64 = A.cpu().bfloat16().double(), W.cpu().bfloat16().double()
    ref_pre = A64 @ W64.t() + bias.cpu().double()
    assert rel_err(pre.cpu(), ref_pre) < 1e-5
    # the BatchNorm of the GEMM's own (fp32) output, float64
    x = pre.cpu().double()
    rm64, rv64 = torch.zeros(N, dtype=torch.float64), torch.ones(N, dtype=torch.float64)
    ref_y = torch.relu(torch.nn.functional.batch_norm(x, rm64, rv64, g.cpu().double(), bb.cpu().double(), True, 0.1,
                                                      1e-5))
    assert rel_err(y.cpu(), ref_y) < 1e-5
    assert rel_err(mean.cpu(), x.mean(0)) < 1e-6
    assert rel_err(rm.cpu(), rm64) < 1e-6 and rel_err(rv.cpu(), rv64) < 1e-6


@pytest.mark.parametrize("M,C,relu", [(3136, 256, 1), (5184, 144, 0), (37, 200, 1)])
def test_bn_ex_counters_do_not_change_results(L, ws, M, C, relu):
    """vc_bn_forward_ex / vc_bn_bwd_ex with arrival counters == without, bit for bit, and the counters are
    left zero (round 5: the one-launch spin-barrier forms are gone; the counters select
    only the backward-without-dx last-arriver reduction)"""
    x = (rnd(M, C, seed=81, scale=2.0) + 3.0).to(DEV)
    w, b = (rnd(C, seed=82) + 1.0).to(DEV), rnd(C, seed=83).to(DEV)
    dy = rnd(M, C, seed=84).to(DEV)
    cnt = torch.zeros(1 << 16, dtype=torch.int32, device=DEV)
    outs = []
    for c_ in (None, cnt, cnt):
        cp, cn = (P(c_), c_.numel()) if c_ is not None else (None, 0)
        rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        mean, inv = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        y = torch.full((M, C), float("nan"), device=DEV)
        dx = torch.full((M, C), 0.5, device=DEV)
        dw, db = torch.full((C,), 2.0, device=DEV), torch.full((C,), 3.0, device=DEV)
        L.vc_bn_forward_ex(1, M, C, P(x), C, 1e-5, 0.1, P(mean), P(inv), P(rm), P(rv), P(w), P(b), relu, P(y), C,
                           P(ws), ws.numel(), cp, cn, S())
        L.vc_bn_bwd_ex(1, M, C, P(dy), C, P(x), C, P(y) if relu else None, C, P(mean), P(inv), P(w), P(dx), C,
                       1.0, P(dw), P(db), 0.5, P(ws), ws.numel(), cp, cn, S())
        torch.cuda.synchronize()
        outs.append([t.cpu() for t in (y, mean, inv, rm, rv, dx, dw, db)])
        assert int(cnt.abs().sum()) == 0
    for o in outs[1:]:
        for a_, b_ in zip(outs[0], o):
            assert torch.equal(a_, b_)


@pytest.mark.parametrize("train", [1, 0])
@pytest.mark.parametrize("M,C", [(3136, 256), (5184, 144), (37, 200), (7744, 64)])
def test_bn_bwd_relu_affine_is_bit_identical(L, ws, train, M, C):
    """vc_bn_bwd_relu_ex (the ReLU decisions recomputed from x and the affine) == vc_bn_bwd_ex with
    relu_out = the forward's output, bit for bit: dx, dw, db (with and without counters)"""
    x = (rnd(M, C, seed=91, scale=2.0) + 0.3).to(DEV)
    w, b = (rnd(C, seed=92) + 0.5).to(DEV), rnd(C, seed=93).to(DEV)
    dy = rnd(M, C, seed=94).to(DEV)
    rm, rv = (rnd(C, seed=95) * 0.1).to(DEV), (rnd(C, seed=96).abs() + 0.5).to(DEV)
    mean, inv = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
    z = torch.empty(M, C, device=DEV)
    L.vc_bn_forward(train, M, C, P(x), C, 1e-5, 0.1, P(mean), P(inv), P(rm), P(rv), P(w), P(b), 1, P(z), C, P(ws),
                    ws.numel(), S())
    cnt = torch.zeros(1 << 16, dtype=torch.int32, device=DEV)
    outs = []
    for affine in (False, True):
        for c_ in (None, cnt):
            dx = torch.full((M, C), 0.25, device=DEV)
            dw, db = torch.full((C,), 2.0, device=DEV), torch.full((C,), 3.0, device=DEV)
            cp, cn = (P(c_), c_.numel()) if c_ is not None else (None, 0)
            if affine:
                L.vc_bn_bwd_relu_ex(train, M, C, P(dy), C, P(x), C, P(mean), P(inv), P(w), P(b), P(dx), C, 1.0, P(dw),
                                    P(db), 0.5, P(ws), ws.numel(), cp, cn, S())
            else:
                L.vc_bn_bwd_ex(train, M, C, P(dy), C, P(x), C, P(z), C, P(mean), P(inv), P(w), P(dx), C, 1.0, P(dw),
                               P(db), 0.5, P(ws), ws.numel(), cp, cn, S())
            torch.cuda.synchronize()
            outs.append([t.cpu() for t in (dx, dw, db)])
    assert (z > 0).any() and (z == 0).any()
    for o in outs[1:]:
        for a_, b_ in zip(outs[0], o):
            assert torch.equal(a_, b_)


@pytest.mark.parametrize("flags", [0, F_BF16])
@pytest.mark.parametrize("grouped", [False, True])
def test_gemm_pipe_two_ktiles_per_stage_is_bit_identical(probe, ws, flags, grouped, monkeypatch):
    """The pipelined GEMM with two 32-wide k-tiles per ring stage (VITCNN_PIPE_KM=2, probe library: one DMA wait and
    barrier per 64 of K) == one k-tile per stage, bit for bit: alone and grouped, fp32 and bf16 MFMAs, with the
    bias-gradient ones column, split-K slices of an odd number of k-tiles and a ragged K (the shapes force the
    pipelined kernel with F_PIPE)"""
    probs = GROUP_PROBLEMS_PIPE + [(0, 1, 3136, 256, 1296, 1, False, 0.0), (1, 0, 256, 144, 3136, 1, True, 0.0),
                                   (0, 0, 200, 96, 100, 1, False, 0.5)]
    ins = []
    for i, (ta, tb, M, N, K, batch, bg, beta) in enumerate(probs):
        A = (rnd(K, M, seed=150 + i) if ta else rnd(M, K, seed=150 + i)).to(DEV)
        B = (rnd(N, K, seed=170 + i) if tb else rnd(K, N, seed=170 + i)).to(DEV)
        ins.append((A, B))
    grp = ctypes.create_string_buffer(GROUP_BYTES)
    outs = []
    for km in ("1", "2"):
        monkeypatch.setenv("VITCNN_PIPE_KM", km)
        res = []
        if grouped:
            probe.vc_gemm_group_begin(ctypes.addressof(grp), S())
        for i, (ta, tb, M, N, K, batch, bg, beta) in enumerate(probs):
            A, B = ins[i]
            C = rnd(M, N, seed=190 + i).to(DEV)
            bgr = torch.full((M,), 0.25, device=DEV) if bg else None
            args = (ta, tb, M, N, K, 1.0, P(A), M if ta else K, 0, P(B), K if tb else N, 0, beta, P(C), N, 0, 1, None,
                    None, 0, 0, flags | F_PIPE, P(bgr), P(ws), ws.numel(), None, 0)
            if grouped:
                probe.vc_gemm_group_add(ctypes.addressof(grp), *args)
            else:
                probe.vc_gemm_ex(*args, S())
            res.append((C, bgr))
        if grouped:
            probe.vc_gemm_group_end(ctypes.addressof(grp))
        torch.cuda.synchronize()
        outs.append([(c.cpu(), b.cpu() if b is not None else None) for c, b in res])
    for (c0, b0), (c1, b1) in zip(outs[0], outs[1]):
        assert torch.equal(c0, c1)
        assert b0 is None or torch.equal(b0, b1)
