"""Device patch windows (vc_patch_gather / vc_center_accumulate) and the plugin surface on the GPU:
test() whole-image inference vs the reference's sliding-window loop evaluated by the oracle,
train()/val() over device-assembled batches."""
import numpy as np
import pytest
import torch

from helpers import hash_state_dict

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _ref_windows(W, H, P, step):
    offw, offh = (W - P) % step, (H - P) % step
    out = []
    for x in range(0, W - P + offw + 1, step):
        if x + P > W:
            x = W - P
        for y in range(0, H - P + offh + 1, step):
            if y + P > H:
                y = H - P
            out.append((x, y))
    return out


def _np_xform(p, code):
    """datasets.py flip / rotate on a [P, P, C] patch"""
    if code & 3:
        if code & 1:
            p = np.fliplr(p)
        if code & 2:
            p = np.flipud(p)
    elif code >> 2:
        p = np.rot90(p, k=code >> 2)
    return p


@pytest.mark.parametrize("C,P,step", [(144, 9, 1), (1, 9, 2), (66, 11, 3), (37, 5, 1)])
def test_patch_gather_sliding_and_corners(C, P, step):
    _need_gpu()
    from vitcnn_amd._lib import lib
    L = lib()
    rng = np.random.default_rng(C + P)
    W, H = 23, 19
    img = rng.random((W, H, C), dtype=np.float32)
    cube = torch.from_numpy(img).to(DEV)
    wins = _ref_windows(W, H, P, step)
    s = torch.cuda.current_stream().cuda_stream
    # sliding-window mode, in two launches (k0 offset)
    n = len(wins)
    out = torch.full((n, C, P, P), float("nan"), device=DEV)
    h = n // 2
    L.vc_patch_gather(W, H, C, P, cube.data_ptr(), None, 0, step, h, None, out.data_ptr(), s)
    L.vc_patch_gather(W, H, C, P, cube.data_ptr(), None, h, step, n - h, None, out[h:].data_ptr(), s)
    ref = np.stack([img[x:x + P, y:y + P].transpose(2, 0, 1) for x, y in wins])
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), ref)
    # explicit corners + every augmentation code
    codes = np.array([0, 1, 2, 3, 4, 8, 12] * 3, dtype=np.uint8)
    cor = np.array([wins[i % n] for i in range(0, 7 * len(codes), 7)], dtype=np.int32)
    ref2 = np.stack([_np_xform(img[x:x + P, y:y + P], c).transpose(2, 0, 1) for (x, y), c in zip(cor, codes)])
    cd, xd = torch.from_numpy(cor).to(DEV), torch.from_numpy(codes).to(DEV)
    out2 = torch.empty(len(codes), C, P, P, device=DEV)
    L.vc_patch_gather(W, H, C, P, cube.data_ptr(), cd.data_ptr(), 0, 0, len(codes), xd.data_ptr(), out2.data_ptr(), s)
    torch.cuda.synchronize()
    assert np.array_equal(out2.cpu().numpy(), np.ascontiguousarray(ref2))


def test_center_accumulate():
    _need_gpu()
    from vitcnn_amd._lib import lib
    L = lib()
    W, H, P, step, ncls = 21, 17, 9, 2, 16
    wins = _ref_windows(W, H, P, step)
    logits = torch.randn(len(wins), ncls)
    probs = torch.zeros(W, H, ncls, dtype=torch.float64)
    for (x, y), lg in zip(wins, logits):
        probs[x + P // 2, y + P // 2] += lg.double()
    got = torch.full((W, H, ncls), 0.5, dtype=torch.float64, device=DEV)
    ld = logits.to(DEV)
    L.vc_center_accumulate(W, H, P, ncls, None, 0, step, len(wins), ld.data_ptr(), got.data_ptr(),
                           torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(got.cpu() - 0.5, probs)


def test_test_whole_image_matches_reference_loop():
    """model_utils.test on a small scene == the reference loop (windows -> eval forward -> centre
    accumulation) evaluated by the CPU oracle, within the 1e-3 fp32 tolerance."""
    _need_gpu()
    from oracle import vitcnn_oracle as O
    from vitcnn_amd import model_utils as mu
    rng = np.random.default_rng(7)
    W, H, P = 14, 12, 9
    img1 = rng.random((W, H, 144), dtype=np.float32)
    img2 = rng.random((W, H, 1), dtype=np.float32)
    sd = hash_state_dict()
    model, _, _, hp = mu.get_model("Multimodality_Mamba", n_classes=16, n_bands=(144, 1), ignored_labels=[0],
                                   dataset="synthetic", device=torch.device(DEV))
    model.load_state_dict(sd)
    hp["test_stride"] = 1
    probs = mu.test(0, model, img1, img2, hp)
    assert probs.dtype == np.float64 and probs.shape == (W, H, 16)
    wins = _ref_windows(W, H, P, 1)
    x1 = torch.from_numpy(np.stack([img1[x:x + P, y:y + P].transpose(2, 0, 1) for x, y in wins]))
    x2 = torch.from_numpy(np.stack([img2[x:x + P, y:y + P].transpose(2, 0, 1) for x, y in wins]))
    st = O.make_state(sd, requires_grad=False)
    with torch.no_grad():
        ref_logits = O.forward(O.Params(st, training=False), x1, x2)
    ref = np.zeros((W, H, 16))
    for (x, y), lg in zip(wins, ref_logits.numpy()):
        ref[x + P // 2, y + P // 2] += lg
    err = np.abs(probs - ref).max() / np.abs(ref).max()
    assert err < 1e-3, err
    assert np.array_equal(probs.argmax(-1)[ref.any(-1)], ref.argmax(-1)[ref.any(-1)])
    untouched = ~ref.any(-1)
    assert np.all(probs[untouched] == 0)


def test_train_and_val_over_device_batches(tmp_path, monkeypatch):
    """model_utils.train over PatchBatcher batches (flip augmentation on) on a learnable synthetic scene
    (4 classes in spatial blocks, class-dependent spectra + noise; label 0 ignored): the optimizer moves
    the parameters, the training loss falls, val() equals an independent count over the same batches,
    and the trained model separates the classes well above chance (0.25)."""
    _need_gpu()
    from vitcnn_amd import model_utils as mu
    from vitcnn_amd.window import PatchBatcher
    monkeypatch.chdir(tmp_path)
    rng = np.random.default_rng(1)
    W, H = 40, 36
    gt = np.zeros((W, H), dtype=np.int64)
    gt[:20, :18], gt[20:, :18], gt[:20, 18:], gt[20:, 18:] = 1, 2, 3, 4
    gt[::7, ::5] = 0                                               # scattered ignored pixels
    mean1 = rng.random((5, 144), dtype=np.float32)
    img1 = (mean1[gt] + 0.3 * rng.standard_normal((W, H, 144))).astype(np.float32)
    img2 = (gt[..., None] / 4.0 + 0.3 * rng.standard_normal((W, H, 1))).astype(np.float32)
    model, opt, crit, hp = mu.get_model("Multimodality_Mamba", n_classes=5, n_bands=(144, 1), ignored_labels=[0],
                                        dataset="synthetic", device=torch.device(DEV))
    p0 = {k: v.detach().clone() for k, v in model.state_dict().items()}
    loader = PatchBatcher(img1, img2, gt, 9, ignored_labels=[0], batch_size=64, flip_augmentation=True, device=DEV)
    val_loader = PatchBatcher(img1, img2, gt, 9, ignored_labels=[0], batch_size=64, device=DEV)

    def mean_loss():
        tot, n = 0.0, 0
        with torch.no_grad():
            for d1, d2, t in val_loader:
                tot += float(crit(model(d1, d2), t)) * t.numel()
                n += t.numel()
        return tot / n

    loss0 = mean_loss()
    best = mu.train("t", 0, None, model, opt, crit, loader, 3, scheduler=hp["scheduler"], display_iter=0,
                    device=torch.device(DEV))
    assert best is not None and set(best.keys()) == set(model.state_dict().keys())
    sd = model.state_dict()
    assert all(torch.isfinite(v.float()).all() for v in sd.values())
    moved = [k for k, v in sd.items() if v.is_floating_point() and not torch.equal(v, p0[k])]
    # ~1020 trained tensors; the rest of the 1470 floating-point entries belong to modules of the reference's
    # parameter tree that its forward never calls (kept for the state_dict) or are unused running stats
    assert len(moved) >= 1000, len(moved)
    assert any(k.startswith("hsi1.global_view.layers.0.") for k in moved)
    loss1 = mean_loss()
    assert loss1 < 0.7 * loss0, (loss0, loss1)
    acc = mu.val(model, val_loader, device=DEV)
    correct = counted = 0
    with torch.no_grad():
        for d1, d2, t in val_loader:
            pred = model(d1, d2).argmax(dim=1).cpu().numpy()
            t = t.cpu().numpy()
            keep = pred != 0
            correct += int(((pred == t) & keep).sum())
            counted += int(keep.sum())
    assert acc == correct / counted
    assert acc > 0.6, acc


def test_test_whole_image_production_batch_matches_reference_loop():
    """test() at its production batch -- a 26 x 26 scene = 324 windows goes through
    the model as ONE batch of 324 (>= 256: the MFMA NonLocal forward `nl_fwd_mfma` and every B >= 256
    kernel configuration run) -- against the reference loop evaluated by the CPU oracle: 1e-3
    relative on the probability map, argmax bit-exact on every window centre."""
    _need_gpu()
    from oracle import vitcnn_oracle as O
    from vitcnn_amd import model_utils as mu
    rng = np.random.default_rng(17)
    W = H = 26
    P = 9
    # a scene of 9 regions with their own band profiles (i.i.d. pixels would give every window the same
    # class: the network's eval output barely depends on white noise), so the class indices vary
    xx, yy = np.meshgrid(np.arange(W), np.arange(H), indexing="ij")
    region = (xx * 3 // W) * 3 + (yy * 3 // H)
    prof = rng.random((9, 144), dtype=np.float32)
    img1 = (0.7 * prof[region] + 0.3 * rng.random((W, H, 144), dtype=np.float32)).astype(np.float32)
    img2 = (region[:, :, None] / 9.0 + 0.1 * rng.random((W, H, 1))).astype(np.float32)
    sd = hash_state_dict()
    # running statistics away from their init values, so eval-mode BatchNorm normalises for real
    g = torch.Generator().manual_seed(3)
    for k, v in sd.items():
        if k.endswith("running_mean"):
            sd[k] = torch.rand(v.shape, generator=g) * 0.2 - 0.1
        elif k.endswith("running_var"):
            sd[k] = torch.rand(v.shape, generator=g) + 0.5
    sd["classifier.bias"] = torch.zeros(16)
    model, _, _, hp = mu.get_model("Multimodality_Mamba", n_classes=16, n_bands=(144, 1), ignored_labels=[0],
                                   dataset="synthetic", device=torch.device(DEV))
    model.load_state_dict(sd)
    hp["test_stride"] = 1
    wins = _ref_windows(W, H, P, 1)
    assert len(wins) == 324
    probs = mu.test(0, model, img1, img2, hp)
    x1 = torch.from_numpy(np.stack([img1[x:x + P, y:y + P].transpose(2, 0, 1) for x, y in wins]))
    x2 = torch.from_numpy(np.stack([img2[x:x + P, y:y + P].transpose(2, 0, 1) for x, y in wins]))
    st = O.make_state(sd, requires_grad=False)
    with torch.no_grad():
        ref_logits = O.forward(O.Params(st, training=False), x1, x2).numpy()
    ref = np.zeros((W, H, 16))
    for (x, y), lg in zip(wins, ref_logits):
        ref[x + P // 2, y + P // 2] += lg
    err = np.abs(probs - ref).max() / np.abs(ref).max()
    assert err < 1e-3, err
    hit = ref.any(-1)
    assert len(set(ref.argmax(-1)[hit].tolist())) > 1      # the class indices vary over the scene
    assert np.array_equal(probs.argmax(-1)[hit], ref.argmax(-1)[hit])


def _noise_batcher(rad, mix, seed=5):
    from vitcnn_amd.window import PatchBatcher
    rng = np.random.default_rng(seed)
    W, H = 40, 36
    img1 = rng.random((W, H, 144), dtype=np.float32)
    img2 = rng.random((W, H, 1), dtype=np.float32)
    gt = rng.integers(0, 6, size=(W, H))
    pb = PatchBatcher(img1, img2, gt, 9, ignored_labels=[0], batch_size=64, flip_augmentation=True, device=DEV,
                      seed=seed, radiation_augmentation=rad, mixture_augmentation=mix)
    return pb, img1, gt


def test_patch_noise_exact_given_the_draws():
    """vc_patch_noise == the CPU restatement (oracle/patch_noise_oracle.py) of datasets.py:529-545 fed the
    same host decisions, transformed label windows and hash fields; and the mixture's candidate table
    pairs the unshuffled labels with the shuffled indices as the reference does (:505-506, :540-543)."""
    _need_gpu()
    from oracle import patch_noise_oracle as NO
    pb, img1, gt = _noise_batcher(True, True)
    # the candidate table: class v -> idx_shuffled[j] over j with labels_unshuffled[j] == v
    mask = gt != 0
    xs, ys = np.nonzero(mask)
    keep = (xs > 4) & (xs < gt.shape[0] - 4) & (ys > 4) & (ys < gt.shape[1] - 4)
    idx = np.stack([xs[keep], ys[keep]], axis=1)
    labels = gt[idx[:, 0], idx[:, 1]]
    sh = idx.copy()
    np.random.RandomState(5).shuffle(sh)
    off, pix = pb.mix_off.cpu().numpy(), pb.mix_pix.cpu().numpy()
    for v in range(1, 6):
        want = sorted((sh[labels == v][:, 0] * gt.shape[1] + sh[labels == v][:, 1]).tolist())
        assert sorted(pix[off[v]:off[v + 1]].tolist()) == want
    assert off[1] == off[0]                                   # the ignored class has no candidates
    # one batch with forced decisions: every sample noised one way or the other
    from vitcnn_amd._lib import lib
    n = 12
    s = torch.cuda.current_stream().cuda_stream
    cor = pb.corners[:n]
    codes = np.array([0, 1, 2, 3, 4, 8, 12, 0, 1, 4, 2, 0], dtype=np.uint8)
    xd = torch.from_numpy(codes).to(DEV)
    x1 = torch.empty(n, 144, 9, 9, device=DEV)
    lib().vc_patch_gather(pb.W, pb.H, 144, 9, pb.c1.data_ptr(), cor.data_ptr(), 0, 0, n, xd.data_ptr(), x1.data_ptr(), s)
    clean = x1.clone()
    rad = np.array([1.05, 0, 0.93, 0, 1.0, 0, 0, 0.9, 0, 1.1, 0, 0], dtype=np.float32)
    mix = np.zeros((n, 2), dtype=np.float32)
    mix[[1, 2, 5, 6, 8, 11]] = [[0.5, 0.3], [0.02, 0.9], [1.0, 1.0], [0.2, 0.7], [0.9, 0.01], [0.4, 0.4]]
    pb.gid = 1000
    pb.apply_noise(x1, cor, xd.data_ptr(), rad, mix, s)
    lab = pb._last_noise[2].cpu().numpy().reshape(n, 9, 9)
    torch.cuda.synchronize()
    cube = img1.reshape(-1, 144)
    ref = NO.apply_noise(clean.cpu().numpy(), lab, rad, mix, off, pix, cube, pb.seed, 1000)
    got = x1.cpu().numpy()
    assert np.abs(got - ref).max() < 2e-5
    assert np.array_equal(got[[3, 10]], clean.cpu().numpy()[[3, 10]])   # samples without a draw stay untouched
    # the label windows are the transformed gt windows
    for i in range(n):
        x, y = pb.centers[i] - 4
        assert np.array_equal(lab[i], _np_xform(gt[x:x + 9, y:y + 9, None], codes[i])[:, :, 0].astype(np.float32))


def test_patch_noise_distribution():
    """radiation p 0.1 and mixture p 0.2 per sample (datasets.py:565-568); the noise fields are
    N(0, 1) / 25; alpha ~ U(0.9, 1.1), a1, a2 ~ U(0.01, 1)."""
    _need_gpu()
    pb, _, _ = _noise_batcher(True, True, seed=9)
    codes, rad, mix = pb.decisions(20000)
    assert abs((rad != 0).mean() - 0.1) < 0.01 and abs((mix[:, 0] > 0).mean() - 0.2) < 0.012
    r = rad[rad != 0]
    assert r.min() >= 0.9 and r.max() <= 1.1 and abs(r.mean() - 1.0) < 0.005
    m = mix[mix[:, 0] > 0]
    assert m.min() >= 0.01 and m.max() <= 1.0
    # the radiation field: x' - alpha x = N / 25 over many elements
    from vitcnn_amd._lib import lib
    pb2, _, _ = _noise_batcher(True, False, seed=9)
    n = 64
    x = torch.zeros(n, 144, 9, 9, device=DEV)
    rad = np.full(n, 1.0, dtype=np.float32)
    pb2.apply_noise(x, pb2.corners[:n], None, rad, np.zeros((n, 2), dtype=np.float32),
                    torch.cuda.current_stream().cuda_stream)
    z = x.cpu().numpy().reshape(-1) * 25
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1.0) < 0.01
    assert abs(np.mean(z ** 4) - 3.0) < 0.05                  # normal kurtosis
    # batches iterate with the noise on, finite
    tot = 0
    for x1, x2, t in pb:
        assert torch.isfinite(x1).all()
        tot += x1.shape[0]
    assert tot == len(pb.centers)
