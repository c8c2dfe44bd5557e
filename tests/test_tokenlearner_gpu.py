"""TokenLearner kernels (csrc/tokenlearner.hip) against a float64 evaluation of the reference's
SpatialAttention / TokenLearner math (Mutimodality_Mamba7.py:26-64): pooled (max, mean) -> 2->1 conv ->
train-mode BatchNorm2d(1) -> ReLU -> sigmoid -> a -> the pooled tokens Z = mean_q a x, and the backward of
sum(Z * dZ) for a given dZ (vc_tl_fwd / vc_tl_bwd: the attention maps and the pooling contractions fused).

The yardstick takes the HIP path's pooled VALUES (max, argmax, mean -- rounded in fp32 as the reference
rounds them) and its ReLU decisions (vc_tl_relu_mask), exactly as tests/helpers.masked_oracle_step does
for the whole model; everything after the pooling is float64.  Inputs include the ill-conditioned regime
the model meets (a BN(1) input whose batch spread is ~1e-4 of its mean), where the
HIP path's fp64 statistics / gradient sums must hold the float64 result element-wise.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
EPS32 = float(np.float32(1e-5))   # the eps the kernels receive (a float argument), as a double


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vitcnn_amd._lib import lib
    return lib()


def _s():
    return torch.cuda.current_stream().cuda_stream


def _params(S, seed):
    g = torch.Generator().manual_seed(seed)
    p = torch.empty(S, 5)
    p[:, 0:2] = torch.rand(S, 2, generator=g) * 2 - 1          # conv.0.weight
    p[:, 2] = (torch.rand(S, generator=g) * 2 - 1) * 0.5        # conv.0.bias
    p[:, 3] = 0.5 + torch.rand(S, generator=g)                  # BN gamma
    p[:, 4] = (torch.rand(S, generator=g) * 2 - 1) * 0.5        # BN beta
    return p


def _input(B, HW, C, seed, regime):
    g = torch.Generator().manual_seed(seed)
    if regime == "uniform":
        return torch.rand(B * HW, C, generator=g)
    # ill-conditioned: every pixel row ~ one shared profile + a 1e-4 perturbation (the pooled max / mean then
    # vary by ~1e-4 of their value over the batch)
    prof = torch.rand(C, generator=g) + 1.0
    return prof[None, :] * (1.0 + 1e-4 * torch.rand(B * HW, C, generator=g))


def _run_hip(L, train, x, B, HW, C, S, par, buf, dZ):
    M = B * HW
    P = lambda t: t.data_ptr()  # noqa: E731
    xd, pard, bufd, dzd = x.to(DEV), par.reshape(-1).to(DEV), buf.reshape(-1).clone().to(DEV), dZ.to(DEV)
    mx, avg = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    amx = torch.empty(M, dtype=torch.int32, device=DEV)
    ws = torch.full(((L.vc_tl_ws_floats(B, HW, S) + 1) // 2,), float("nan"), dtype=torch.float64, device=DEV)
    st = torch.full((2 * S + 8,), float("nan"), dtype=torch.float64, device=DEV)
    a = torch.full((B * S * HW,), float("nan"), device=DEV)
    Z = torch.full((B * S * C,), float("nan"), device=DEV)
    L.vc_tl_pixel_stats(M, C, P(xd), C, P(mx), P(amx), P(avg), P(ws), _s())
    L.vc_tl_fwd(train, B, HW, C, S, P(xd), C, P(mx), P(avg), P(pard), P(bufd), 1e-5, 0.1, P(ws), P(st), P(a), P(Z),
                _s())
    mask = torch.empty(B * S * HW, dtype=torch.uint8, device=DEV)
    L.vc_tl_relu_mask(B, HW, S, P(mx), P(avg), P(pard), P(st), P(mask), _s())
    dx = torch.full((M, C), float("nan"), device=DEV)
    gp = torch.full((S * 5,), float("nan"), device=DEV)
    L.vc_tl_bwd(train, B, HW, C, S, P(xd), C, P(mx), P(avg), P(amx), P(pard), P(st), P(a), P(dzd), P(ws), P(dx), C,
                P(gp), _s())
    torch.cuda.synchronize()
    return dict(mx=mx.cpu(), amx=amx.cpu().long(), avg=avg.cpu(), st=st.cpu(), a=a.cpu(), Z=Z.cpu(),
                mask=mask.cpu().bool(), dx=dx.cpu(), gp=gp.cpu().view(S, 5), buf=bufd.cpu().view(S, 2))


def _reference(train, x, B, HW, C, S, par, buf, dZ, hip):
    """float64 SpatialAttention x S + the pooled tokens, with the HIP path's pooled values and ReLU decisions;
    backward of sum(Z * dZ)"""
    x64 = x.double().requires_grad_(True)
    p64 = par.double().requires_grad_(True)
    g = torch.gather(x64, 1, hip["amx"][:, None])[:, 0]
    m = x64.mean(dim=1)
    mx = hip["mx"].double() + (g - g.detach())
    av = hip["avg"].double() + (m - m.detach())
    f = p64[:, 0:1] * mx[None] + p64[:, 1:2] * av[None] + p64[:, 2:3]          # [S, n]
    if train:
        mean = f.mean(dim=1, keepdim=True)
        var = f.var(dim=1, unbiased=False, keepdim=True)
    else:
        mean = buf[:, 0:1].double()
        var = buf[:, 1:2].double()
    bn = (f - mean) / torch.sqrt(var + EPS32) * p64[:, 3:4] + p64[:, 4:5]
    mask = hip["mask"].view(B, S, HW).permute(1, 0, 2).reshape(S, B * HW)
    a = torch.sigmoid(bn * mask.double())                                        # [S, n]
    a_b = a.view(S, B, HW).permute(1, 0, 2)                                       # [B, S, HW]
    Z = torch.bmm(a_b, x64.view(B, HW, C)) / HW                                   # [B, S, C]
    (Z * dZ.view(B, S, C).double()).sum().backward()
    new_buf = None
    if train:
        fv = f.detach()
        new_buf = torch.stack([0.9 * buf[:, 0].double() + 0.1 * fv.mean(1),
                               0.9 * buf[:, 1].double() + 0.1 * fv.var(1, unbiased=True)], 1)
    return dict(a=a_b.detach().reshape(-1), Z=Z.detach().reshape(-1), dx=x64.grad, gp=p64.grad, buf=new_buf,
                mean=mean.detach().view(-1), var=var.detach().view(-1))


def _close(got, ref, rtol):
    got, ref = got.double(), ref.double()
    return float((got - ref).abs().max()) <= rtol * max(float(ref.abs().max()), 1e-30)


# the model's shapes (9x9 hsi1 / hsi2, MUUFL 11x11), a tiny one, and patches beyond the model's envelope (ADVICE
# r5): 13x13 (HW > 128, one chunk each), 15x15 (the forward's tokens and the backward's pixels chunked to fit the
# LDS) and 20x20 (the largest grid vc_tl_check accepts)
@pytest.mark.parametrize("B,HW,C,S", [(64, 81, 256, 49), (64, 49, 144, 25), (4, 81, 256, 49), (5, 121, 64, 81),
                                      (3, 9, 20, 4), (4, 169, 256, 121), (3, 225, 64, 169), (2, 400, 256, 324)])
@pytest.mark.parametrize("regime", ["uniform", "illcond"])
@pytest.mark.parametrize("train", [1, 0])
def test_tokenlearner_vs_float64(L, B, HW, C, S, regime, train):
    x = _input(B, HW, C, seed=B * 131 + C, regime=regime)
    par = _params(S, seed=S)
    buf = torch.stack([torch.rand(S) + 0.5, torch.rand(S) * 0.1 + 1e-3], 1)
    if regime == "illcond" and not train:
        # running statistics that match the ill-conditioned batch (eval normalises with them)
        xm = x.max(1).values.double()
        xa = x.double().mean(1)
        f = par[:, 0:1].double() * xm[None] + par[:, 1:2].double() * xa[None] + par[:, 2:3].double()
        buf = torch.stack([f.mean(1), f.var(1) * 4.0], 1).float()
    g = torch.Generator().manual_seed(7)
    dZ = torch.rand(B * S * C, generator=g) * 2 - 1
    hip = _run_hip(L, train, x, B, HW, C, S, par, buf, dZ)
    # pooled values: the same fp32 arithmetic as the reference's max / mean up to summation order
    assert torch.equal(hip["mx"], x.max(1).values)
    assert torch.equal(hip["amx"], x.argmax(1)) or bool((x.gather(1, hip["amx"][:, None])[:, 0] == hip["mx"]).all())
    assert float((hip["avg"].double() - x.double().mean(1)).abs().max()) <= 1e-6 * float(x.abs().max())
    ref = _reference(train, x, B, HW, C, S, par, buf, dZ, hip)
    n = B * HW
    # statistics
    assert torch.allclose(hip["st"][0:2 * S:2], ref["mean"], rtol=1e-12, atol=1e-14 * float(ref["mean"].abs().max()))
    assert torch.allclose(hip["st"][1:2 * S:2], 1.0 / torch.sqrt(ref["var"] + EPS32), rtol=1e-9)
    assert abs(float(hip["st"][2 * S]) - n) == 0
    assert _close(hip["a"], ref["a"], 1e-6)
    assert _close(hip["Z"], ref["Z"], 1e-5)
    if train:
        assert _close(hip["buf"], ref["buf"], 1e-6)
    else:
        assert torch.equal(hip["buf"], buf)
    # gradients: each parameter column, and the input gradient
    gref = ref["gp"]
    floor = 1e-7 * float(gref.abs().max())
    for j in range(5):
        err = float((hip["gp"][:, j].double() - gref[:, j]).abs().max())
        assert err <= 1e-5 * float(gref[:, j].abs().max()) + floor, (j, err, float(gref[:, j].abs().max()))
    assert _close(hip["dx"], ref["dx"], 1e-5)


def test_tokenlearner_is_deterministic(L):
    B, HW, C, S = 64, 81, 256, 49
    x = _input(B, HW, C, seed=3, regime="illcond")
    par = _params(S, seed=4)
    buf = torch.stack([torch.zeros(S), torch.ones(S)], 1)
    dZ = torch.rand(B * S * C) * 2 - 1
    r1 = _run_hip(L, 1, x, B, HW, C, S, par, buf, dZ)
    r2 = _run_hip(L, 1, x, B, HW, C, S, par, buf, dZ)
    for k in ("st", "a", "Z", "dx", "gp", "buf"):
        assert torch.equal(r1[k], r2[k]), k
