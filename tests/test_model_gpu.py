"""Full-model parity on the MI355X: the HIP ViT-CNN vs the CPU oracle (pinned to the reference).

Same hash-initialised parameters and the same synthetic batch go through
  * the product path  (vitcnn_amd: hand-written gfx950 kernels via the C ABI), and
  * the oracle        (oracle/vitcnn_oracle.py, fp32 CPU restatement in the reference's op order).
Tolerances (north_star): logits within 1e-3 relative (fp32), argmax bit-exact where the top-2
margin is meaningful; gradients within 1e-3 relative of their norm plus an absolute floor that
scales with the largest gradient (parameters whose true gradient is exactly zero carry only fp32
cancellation noise, see tests/test_oracle_golden.py).
"""
import numpy as np
import pytest
import torch

from helpers import (check_audit, golden_batch, hash_state_dict, load_npz, masked_oracle_step, rel_err,
                     relu_masks_from_workspace, tl_pooled_from_workspace)
from oracle import vitcnn_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _product(sd):
    from vitcnn_amd import Multimodality_Mamba
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16, "multi_clock_gate")
    m.load_state_dict(sd)
    return m.to(DEV)


def _nhwc_to_nchw(t, B, H, C):
    return t[: B * H * H * C].reshape(B, H, H, C).permute(0, 3, 1, 2).cpu()


@pytest.fixture(scope="module")
def b4():
    _need_gpu()
    sd = hash_state_dict()
    hsi, lidar, target = golden_batch("golden.b4", 4)
    # oracle, with per-block activations
    state = O.make_state(sd)
    acts = {}
    orig = (O.global_local_block, O.hsi_mamba)

    def wrap(fn):
        def inner(P, pfx, *a):
            out = fn(P, pfx, *a)
            if P.training:
                acts[pfx] = out.detach().clone()
            return out
        return inner

    O.global_local_block, O.hsi_mamba = wrap(orig[0]), wrap(orig[1])
    try:
        w = O.ce_class_weights(16)
        ref_logits, ref_loss = O.train_step(state, hsi, lidar, target, w)
    finally:
        O.global_local_block, O.hsi_mamba = orig
    ref_grads = {k: state[k].grad for k in O.param_names(state)}
    # product
    from vitcnn_amd import CrossEntropyLoss
    m = _product(sd)
    m.train()
    crit = CrossEntropyLoss(weight=w.to(DEV))
    logits = m(hsi.to(DEV), lidar.to(DEV))
    loss = crit(logits, target.to(DEV))
    loss.backward()
    torch.cuda.synchronize()
    # float64 evaluation of the same step (with the HIP path's ReLU decisions, see
    # helpers.masked_oracle_step): the yardstick for "as accurate as the fp32 reference"
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
    st64 = O.make_state(sd64)
    masks = relu_masks_from_workspace(m, 4)
    audit = []
    masked_oracle_step(O, st64, hsi.double(), lidar.double(), target, w.double(), masks,
                       pooled=tl_pooled_from_workspace(m, 4), audit=audit)
    ref64 = {k: st64[k].grad for k in O.param_names(st64)}
    # fp32 reference's own error is measured against its own ReLU decisions
    st64r = O.make_state(sd64)
    O.train_step(st64r, hsi.double(), lidar.double(), target, w.double())
    ref64_own = {k: st64r[k].grad for k in O.param_names(st64r)}
    return dict(m=m, ref_logits=ref_logits, ref_loss=ref_loss, ref_grads=ref_grads, ref64=ref64, ref64_own=ref64_own,
                ref_state=state,
                acts=acts, audit=audit,
                logits=logits.detach().cpu(), loss=float(loss.item()), hsi=hsi, lidar=lidar, target=target)


def test_forward_activations_b4(b4):
    m, acts = b4["m"], b4["acts"]
    ws = next(w for k, w in m._ws.items() if k[2] == ("train", "grad"))
    B = 4
    checks = [("hsi1.global_view", "hsi1.G", 9, 144), ("hsi2.global_view", "hsi2.G", 7, 256),
              ("hsi1", "hsi1.fusion.FusionLayer.out", 7, 256), ("hsi2", "hsi2.fusion.FusionLayer.out", 5, 144)]
    for ref_key, ws_key, H, C in checks:
        got = _nhwc_to_nchw(ws.tensor(ws_key), B, H, C)
        err = rel_err(got.numpy(), acts[ref_key].numpy())
        assert err < 1e-3, (ref_key, err)


def test_logits_loss_b4(b4):
    assert rel_err(b4["logits"].numpy(), b4["ref_logits"].numpy()) < 1e-3
    assert abs(b4["loss"] - b4["ref_loss"]) < 1e-3 * abs(b4["ref_loss"])
    g = load_npz("vitcnn_b4.npz")
    assert rel_err(b4["logits"].numpy(), g["logits"]) < 1e-3


def test_gradients_b4(b4):
    """Every gradient element vs a float64 evaluation: the HIP path must be within 1e-3 of each
    tensor's scale, or (for cancellation-dominated tensors such as the TokenLearner / NonLocal
    paths that feed train-mode BatchNorms) no worse than 3x the fp32 reference's own error."""
    m, ref, ref64, ref64_own = b4["m"], b4["ref_grads"], b4["ref64"], b4["ref64_own"]
    flat = m.flat_params.grad.detach().cpu()
    named = dict(m.named_parameters())
    gmax = max(float(g.abs().max()) for g in ref64.values() if g is not None)
    # absolute floor 1e-5 of the largest gradient in the model: a TokenLearner BN(1) pre-activation
    # within rounding distance of 0 (its ReLU decision is an fp32 tie) moves that token's tiny
    # gradients by ~1e-6 of gmax; every larger tensor is held to the per-tensor criteria below.
    floor = 1e-5 * gmax
    bad = []
    for n, off in m._poff.items():
        p = named[n]
        got = flat[off:off + p.numel()].view(p.shape).double()
        r64 = ref64.get(n)
        if r64 is None:
            assert float(got.abs().max()) == 0.0, n
            continue
        err = float((got - r64).abs().max())
        err32 = float((ref[n].double() - ref64_own[n]).abs().max())
        scale = float(r64.abs().max())
        if not (err <= 1e-3 * scale + floor or err <= 3.0 * err32 + floor):
            bad.append((n, err, err32, scale))
    assert not bad, bad[:5]


def test_adopted_decisions_are_ties_b4(b4):
    """the float64 yardstick of test_gradients_b4 takes the HIP path's ReLU masks, NonLocal
    max-pool taps and TokenLearner pooled values; each is compared with the decision float64 takes at the same
    site, and every disagreement must be a genuine fp32 near-tie (helpers._audit_*)."""
    s = check_audit(b4["audit"], "b4")
    assert s["relu"][1] > 100000 and s["maxpool"][1] > 10000 and s["tl_pool"][1] > 500 and s["tl_relu"][1] > 10000


def test_running_stats_and_counters_b4(b4):
    m, st = b4["m"], b4["ref_state"]
    sd = m.state_dict()
    for k, v in sd.items():
        if k.endswith("running_mean") or k.endswith("running_var"):
            assert rel_err(v.cpu().numpy(), st[k].numpy()) < 1e-3, k
        if k.endswith("num_batches_tracked"):
            assert int(v.item()) == int(st[k].item()), k


def test_adamw_step_b4(b4):
    """The fused AdamW kernel vs torch.optim.AdamW fed the SAME gradients (two steps).

    (Adam normalises each element by its own |g|, so comparing after independently computed
    gradients would only measure gradient noise on elements with |g| ~ eps.)"""
    from vitcnn_amd import AdamW
    m = b4["m"]
    before = {n: p.detach().cpu().clone() for n, p in m.named_parameters()}
    flat_g = m.flat_params.grad.detach().cpu().clone()
    opt = AdamW(m.parameters(), lr=8e-4)
    opt.step()
    opt.step()
    torch.cuda.synchronize()
    ref_params = {n: before[n].clone().requires_grad_(True) for n in before}
    unused = O.unused_param_prefixes()
    live = [n for n in ref_params if not n.startswith(unused)]
    ref_opt = torch.optim.AdamW([ref_params[n] for n in live], lr=8e-4)
    named = dict(m.named_parameters())
    for _ in range(2):
        for n in live:
            off = m._poff[n]
            ref_params[n].grad = flat_g[off:off + named[n].numel()].view(named[n].shape).clone()
        ref_opt.step()
    for n, p in named.items():
        got = p.detach().cpu()
        if n.startswith(unused):
            assert torch.equal(got, before[n]), n   # grad None in the reference: untouched, no decay
        else:
            assert float((got - ref_params[n].detach()).abs().max()) <= 2e-6, n


def test_eval_mode_logits(b4):
    m = b4["m"]
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    st = O.make_state(sd, requires_grad=False)
    m.eval()
    with torch.no_grad():
        got = m(b4["hsi"].to(DEV), b4["lidar"].to(DEV)).cpu()
        ref = O.forward(O.Params(st, training=False), b4["hsi"], b4["lidar"])
    m.train()
    assert rel_err(got.numpy(), ref.numpy()) < 1e-3


def test_b64_against_reference_golden():
    _need_gpu()
    from vitcnn_amd import CrossEntropyLoss
    g = load_npz("vitcnn_b64.npz")
    m = _product(hash_state_dict())
    m.train()
    hsi, lidar, target = golden_batch("golden.b64", 64)
    crit = CrossEntropyLoss(weight=O.ce_class_weights(16).to(DEV))
    logits = m(hsi.to(DEV), lidar.to(DEV))
    loss = crit(logits, target.to(DEV))
    loss.backward()
    got = logits.detach().cpu().numpy()
    ref = g["logits"]
    assert rel_err(got, ref) < 1e-3
    assert abs(float(loss.item()) - float(g["loss"])) < 1e-3 * abs(float(g["loss"]))
    # argmax must agree wherever the reference's top-2 margin is above fp32 noise
    top2 = np.sort(ref, axis=1)[:, -2:]
    margin = (top2[:, 1] - top2[:, 0]) / np.abs(ref).max()
    sel = margin > 1e-3
    assert np.array_equal(got.argmax(1)[sel], ref.argmax(1)[sel])
    flat = m.flat_params.grad.detach().cpu()
    # At B=64 the TokenLearner BN(1) gradients are sums of 5184 strongly cancelling terms: the
    # reference's own fp32 values deviate from a float64 evaluation by up to 1.3x
    # (1e-3*|g| + 1e-5*max|g|) (measured; e.g. channel_token.tokenizers.19.conv.1.bias
    # ref32 1.1741e-3, fp64 1.1316e-3, this path 1.1329e-3).  The floor is widened accordingly.
    atol = 5e-5 * float(g["grad_norm"].max())
    named = dict(m.named_parameters())
    for n, ref_n in zip(list(g["grad_norm_names"]), g["grad_norm"]):
        off, numel = m._poff[n], named[n].numel()
        gn = float(flat[off:off + numel].double().norm())
        if ref_n < 0:
            assert gn == 0.0, n
        else:
            assert abs(gn - ref_n) <= 2e-3 * ref_n + atol, (n, gn, float(ref_n))


@pytest.mark.timeout(900)   # up to three B = 64 CPU oracle steps (two of them float64) on the box's 16 cores
def test_b64_gradients_per_tensor_vs_oracle():
    """the headline shape (Houston2013, B = 64) held per tensor, not by norm only.  The fp32
    oracle (pinned to the reference's own B = 64 logits / loss / gradient norms, tests/test_oracle_golden.py)
    runs the same step on the box; every parameter gradient must be within 1e-3 of its norm (+5e-5 of the
    largest norm) of the oracle's, ||g - ref||.  A tensor outside that is then held to a float64 evaluation
    that takes the HIP path's ReLU / max-pool / TokenLearner decisions -- each of which must be a genuine fp32
    near-tie (the decision audit, always run here) -- and must be within the same bound of it, or no further
    from it than 3x the fp32 oracle's own distance to the plain float64 evaluation."""
    _need_gpu()
    from vitcnn_amd import CrossEntropyLoss
    sd = hash_state_dict()
    hsi, lidar, target = golden_batch("golden.b64", 64)
    w = O.ce_class_weights(16)
    state = O.make_state(sd)
    ref_logits, ref_loss = O.train_step(state, hsi, lidar, target, w)
    print("b64: fp32 oracle step done", flush=True)
    m = _product(sd).train()
    logits = m(hsi.to(DEV), lidar.to(DEV))
    loss = CrossEntropyLoss(weight=w.to(DEV))(logits, target.to(DEV))
    loss.backward()
    torch.cuda.synchronize()
    assert rel_err(logits.detach().cpu().numpy(), ref_logits.numpy()) < 1e-3
    assert abs(float(loss) - float(ref_loss)) < 1e-3 * abs(float(ref_loss))
    flat = m.flat_params.grad.detach().cpu()
    named = dict(m.named_parameters())
    names = O.param_names(state)
    norms = {n: float(state[n].grad.norm()) for n in names if state[n].grad is not None}
    gmax = max(norms.values())
    atol = 5e-5 * gmax
    got = {}
    for n, off in m._poff.items():
        g = flat[off:off + named[n].numel()].view(named[n].shape).double()
        if n not in norms:
            assert float(g.abs().max()) == 0.0, n
            continue
        got[n] = g
    direct = [n for n, g in got.items() if float((g - state[n].grad.double()).norm()) <= 1e-3 * norms[n] + atol]
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
    st64 = O.make_state(sd64)
    audit = []
    masked_oracle_step(O, st64, hsi.double(), lidar.double(), target, w.double(), relu_masks_from_workspace(m, 64),
                       pooled=tl_pooled_from_workspace(m, 64), audit=audit)
    print("b64: decision-matched float64 step done", flush=True)
    check_audit(audit, "b64")
    cand = [n for n in got if n not in set(direct)]
    far = [(n, float((got[n] - st64[n].grad).norm())) for n in cand]
    far = [(n, e) for n, e in far if not e <= 1e-3 * float(st64[n].grad.norm()) + atol]
    bad = []
    if far:
        st64r = O.make_state(sd64)
        O.train_step(st64r, hsi.double(), lidar.double(), target, w.double())
        for n, e in far:
            own = float((state[n].grad.double() - st64r[n].grad).norm())
            if not e <= 3.0 * own + atol:
                bad.append((n, e, own, norms[n]))
    print(f"b64 per-tensor: {len(direct)} of {len(got)} within 1e-3 of the fp32 oracle, {len(cand) - len(far)} "
          f"within 1e-3 of the decision-matched float64 step, {len(far) - len(bad)} by the 3x-own-error argument")
    assert len(direct) >= 0.9 * len(got), (len(direct), len(got))
    assert not bad, bad[:5]


def test_fused_step_and_graph_capture_match_autograd():
    """fused_train_step (caller-thread, multi-stream) == crit(model(x)).backward() (autograd), bit for
    bit, and a hipGraph capture of either replays to the same gradients."""
    _need_gpu()
    from vitcnn_amd import CrossEntropyLoss, fused_train_step
    sd = hash_state_dict()
    hsi, lidar, target = (t.to(DEV) for t in golden_batch("golden.b64", 64))
    crit = CrossEntropyLoss(weight=O.ce_class_weights(16).to(DEV))
    m = _product(sd).train()
    loss_a = crit(m(hsi, lidar), target)
    loss_a.backward()
    g_auto = m.flat_params.grad.clone()
    m2 = _product(sd).train()
    loss_f = fused_train_step(m2, crit, hsi, lidar, target)
    torch.cuda.synchronize()
    assert float(loss_a) == float(loss_f)
    assert torch.equal(m2.flat_params.grad, g_auto)
    for use_fused in (True, False):
        m3 = _product(sd).train()
        holder = {}

        def step():
            if use_fused:
                holder["l"] = fused_train_step(m3, crit, hsi, lidar, target)
            else:
                holder["l"] = crit(m3(hsi, lidar), target)
                holder["l"].backward()

        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step()
        torch.cuda.current_stream().wait_stream(s)
        m3.zero_grad(set_to_none=True)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        m3.load_state_dict(sd)  # the warm-up step above updated the BN running statistics
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(m3.flat_params.grad, g_auto), use_fused


def test_gradients_vs_reference_golden_b4(b4):
    """Element-wise gradient parity with NO HIP-derived inputs: every small-parameter gradient the
    reference module itself produced (vitcnn_b4.npz grad/*, the reference's fp32 autograd) against the
    HIP gradient.  A tensor passes directly when max|hip - ref| <= 1e-3 max|ref| + floor.  Otherwise it
    must pass the fp64 argument: max|hip - exact| <= 3 max|ref - exact| + floor, exact = the pure float64
    oracle (no HIP ReLU decisions or pooled values fed in) -- i.e. the HIP value is no further from the
    exact gradient than the reference's own fp32 value is (measured: 594 of 671 tensors pass directly;
    the rest are the train-mode-BatchNorm-conditioned families -- TokenLearner BN(1) tokenizers, BN /
    LN affine parameters downstream of them -- and sums over all 10 x B x L tokens such as the conv1d,
    D and bias gradients, where the reference's fp32 value is up to 0.7 % off the exact one and the HIP
    value within 1e-5 of it).  The per-tensor outcome (and whether the name is in a BN-conditioned
    family) is written to gpurun_out/grad_parity_b4.json when that directory exists."""
    import json
    import os
    m, exact = b4["m"], b4["ref64_own"]
    g = load_npz("vitcnn_b4.npz")
    flat = m.flat_params.grad.detach().cpu()
    named = dict(m.named_parameters())
    keys = [k[5:] for k in g.files if k.startswith("grad/")]
    gmax = max(float(abs(g["grad/" + k]).max()) for k in keys)
    floor = 1e-5 * gmax
    direct, fp64, bad = [], [], []
    conditioned = ("tokenizers", "cross_attention", ".ln", "norm", ".bn", "FusionLayer", "local_feature", "weights")
    for k in keys:
        ref = torch.from_numpy(g["grad/" + k]).double()
        off = m._poff[k]
        got = flat[off:off + named[k].numel()].view(named[k].shape).double()
        scale = float(ref.abs().max())
        err = float((got - ref).abs().max())
        if err <= 1e-3 * scale + floor:
            direct.append(k)
            continue
        ex = exact[k].double()
        err_ex, ref_ex = float((got - ex).abs().max()), float((ref - ex).abs().max())
        if err_ex <= 3.0 * ref_ex + floor:
            fp64.append((k, err, scale, err_ex, ref_ex, any(c in k for c in conditioned)))
        else:
            bad.append((k, err, scale, err_ex, ref_ex))
    if os.path.isdir("gpurun_out"):
        with open("gpurun_out/grad_parity_b4.json", "w") as f:
            json.dump({"tensors": len(keys), "direct": len(direct), "fp64_argument": fp64, "failed": bad}, f, indent=1)
    assert not bad, bad[:5]
    assert len(direct) >= 0.85 * len(keys), (len(direct), len(keys))


def test_trained_eval_mode_class_indices():
    """Eval-mode class indices that vary across samples (the untrained fixture's eval argmax
    is one class everywhere): 8 AdamW(8e-4) steps on the golden B=64 batch, 40 val-style train-mode
    forwards (running statistics settle, the reference's val() runs without net.eval()), then eval-mode
    logits of the trained batch (15 distinct classes in the reference's run) and of a fresh batch,
    against vitcnn_eval64.npz made by the reference module itself (tests/golden/gen_golden.py
    --eval-only).  Eight Adam steps amplify fp32 rounding-order differences (measured between the CPU
    oracle and the reference itself: losses 1e-3, eval logits 2e-2 relative, argmax identical,
    tests/test_oracle_golden.py); the same bounds hold here: losses 3e-3, logits 6e-2, argmax identical
    wherever the reference's top-2 margin exceeds 2e-2 of the logit scale."""
    _need_gpu()
    from vitcnn_amd import AdamW, CrossEntropyLoss, fused_train_step
    z = load_npz("vitcnn_eval64.npz")
    sd = hash_state_dict()
    hsi, lidar, target = golden_batch("golden.b64", 64)
    ehsi, elidar, _ = golden_batch("golden.eval64", 64)
    m = _product(sd).train()
    crit = CrossEntropyLoss(weight=O.ce_class_weights(16).to(DEV))
    opt = AdamW(m.parameters(), lr=8e-4)
    x1, x2, t = hsi.to(DEV), lidar.to(DEV), target.to(DEV)
    losses = []
    for _ in range(int(z["steps"])):
        opt.zero_grad()
        losses.append(float(fused_train_step(m, crit, x1, x2, t, optimizer=opt)))
    assert np.allclose(losses, z["losses"], rtol=3e-3, atol=1e-5), (losses, z["losses"])
    with torch.no_grad():
        for _ in range(int(z["val_passes"])):
            m(x1, x2)
        m.eval()
        for key, (a, b) in (("eval", (x1, x2)), ("eval2", (ehsi.to(DEV), elidar.to(DEV)))):
            got = m(a, b).cpu().numpy()
            ref = z[key + "_logits"]
            assert rel_err(got, ref) < 6e-2, (key, rel_err(got, ref))
            top2 = np.sort(ref, axis=1)[:, -2:]
            sel = (top2[:, 1] - top2[:, 0]) > 2e-2 * np.abs(ref).max()
            assert sel.sum() >= 56, (key, int(sel.sum()))
            assert np.array_equal(got.argmax(1)[sel], ref.argmax(1)[sel]), key
    assert len(set(z["eval_argmax"].tolist())) >= 10


def _schedule_grad(sd, batch, crit, captured, lanes_bwd=True, lane_map=(), ch_lane=1, ch_ordered=True):
    """(loss, flat gradient) of one fused training step under a given lane schedule, eager or replayed
    from a hipGraph capture"""
    import vitcnn_amd.model as VM
    from vitcnn_amd import fused_train_step
    saved = (VM._LANES_BWD, VM._LANE_MAP, VM._CH_LANE, VM._CH_ORDERED)
    VM._LANES_BWD, VM._LANE_MAP, VM._CH_LANE, VM._CH_ORDERED = lanes_bwd, list(lane_map), ch_lane, ch_ordered
    try:
        hsi, lidar, target = batch
        m = _product(sd).train()
        if not captured:
            loss = fused_train_step(m, crit, hsi, lidar, target)
            torch.cuda.synchronize()
            return float(loss), m.flat_params.grad.detach().clone()
        holder = {}
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fused_train_step(m, crit, hsi, lidar, target)     # warm-up: workspaces, events, streams
        torch.cuda.current_stream().wait_stream(s)
        m.zero_grad(set_to_none=True)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            holder["l"] = fused_train_step(m, crit, hsi, lidar, target)
        m.load_state_dict(sd)       # the warm-up step updated the BN running statistics
        g.replay()
        torch.cuda.synchronize()
        return float(holder["l"]), m.flat_params.grad.detach().clone()
    finally:
        VM._LANES_BWD, VM._LANE_MAP, VM._CH_LANE, VM._CH_ORDERED = saved


@pytest.mark.parametrize("lane_map,lanes_bwd,ch_lane", [((), True, 1), ((), False, 1), ((0, 0, 0, 0), True, 1),
                                                        ((0, 1, 1, 1), True, 1), ((0, 1, 2, 1), True, 1),
                                                        ((), True, 3)])
def test_lane_schedules_are_bit_identical(lane_map, lanes_bwd, ch_lane):
    """the step's result does not depend on its schedule.  The default four-lane step
    (eager) is the reference; every other lane map (logical lanes folded onto fewer streams), the
    single-stream backward, and the channel chain on a lane of its own (its dX accumulation ordered after
    the local chain's) -- each eager AND replayed from a hipGraph capture -- give the same loss and the
    same flat gradient bit for bit.  (A cross-lane accumulation without a fixed order -- the round-3
    channel-lane experiment -- makes the sum depend on the schedule: DESIGN.md section 11.)"""
    _need_gpu()
    from vitcnn_amd import CrossEntropyLoss
    sd = hash_state_dict()
    batch = tuple(t.to(DEV) for t in golden_batch("golden.b64", 64))
    crit = CrossEntropyLoss(weight=O.ce_class_weights(16).to(DEV))
    ref_loss, ref = _schedule_grad(sd, batch, crit, False)
    for captured in (False, True):
        loss, g = _schedule_grad(sd, batch, crit, captured, lanes_bwd, lane_map, ch_lane)
        assert loss == ref_loss, (captured, loss, ref_loss)
        assert torch.equal(g, ref), (captured, float((g - ref).abs().max()))
