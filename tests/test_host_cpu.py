"""Host-side checks that need no GPU: the C ABI library, the plugin surface, the state_dict contract,
scan orders, window enumeration, DP sharding and the checkpoint scheme."""
import ctypes
import glob
import json
import os
import re

import numpy as np
import pytest
import torch

from helpers import GOLDEN, reference_keys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    names = set()
    for h in glob.glob(os.path.join(REPO, "include", "*.h")):
        txt = re.sub(r"/\*.*?\*/", " ", open(h).read(), flags=re.S)
        names |= set(re.findall(r"VC_API\s+int\s+(vc_\w+)\s*\(", txt))
    return names


def test_c_abi_library_exports_every_declared_symbol():
    from vitcnn_amd import _lib
    assert os.path.exists(_lib.LIB_PATH), "run __graft_entry__.build() first"
    handle = ctypes.CDLL(_lib.LIB_PATH)
    declared = _declared_symbols()
    assert len(declared) >= 38
    missing = [n for n in sorted(declared) if not hasattr(handle, n)]
    assert not missing, missing
    # the ctypes binding covers exactly the header
    assert set(_lib.parse_header().keys()) == declared


def test_product_loader_ignores_the_environment():
    """no environment variable can point the product path at another build (the probe
    library's VITCNN_* knobs change results); only a tool's explicit use_library_for_tools call can."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); from vitcnn_amd import _lib; "
            "L = _lib.lib(); print(L.path)") % os.path.join(REPO, "vit-cnn_amd")
    probe = os.path.join(REPO, "vit-cnn_amd", "vitcnn_amd", "libvitcnn_probe.so")
    env = dict(os.environ, VITCNN_LIB=probe, VITCNN_BN_FUSED="1")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True).stdout
    assert os.path.basename(out.strip()) == "libvitcnn_hip.so"
    from vitcnn_amd import _lib
    assert "os.environ" not in open(_lib.__file__).read()


def test_c_abi_rejects_bad_shapes_without_a_gpu():
    from vitcnn_amd._lib import lib
    L = lib()
    with pytest.raises(RuntimeError, match="invalid"):
        L.vc_window_count(4, 4, 9, 1, ctypes.addressof(ctypes.c_long(0)))  # window larger than image


def test_model_rejects_unsupported_patches_at_construction():
    """a shape some kernel would refuse mid-step is refused by the constructor instead: patches beyond
    the NonLocal's 16 pooled keys (P > 11), too many bands, and TokenLearner grids beyond its LDS plans."""
    from vitcnn_amd import Multimodality_Mamba
    from vitcnn_amd._lib import lib
    for P in (7, 9, 11):
        Multimodality_Mamba(P, 1, 1, 64, 2, 32, 12)
    for P in (12, 13, 15):
        with pytest.raises(ValueError, match="not supported"):
            Multimodality_Mamba(P, 1, 1, 64, 2, 32, 12)
    with pytest.raises(ValueError, match="bands"):
        Multimodality_Mamba(9, 1, 1, 600, 1, 32, 16)
    raw = lib().raw["vc_tl_check"]
    assert all(raw(P * P, 256, (P - 2) ** 2) == 0 for P in range(3, 21))
    assert raw(21 * 21, 256, 19 * 19) == 1 and raw(81, 513, 49) == 1


def _ref_sliding_window_corners(W, H, P, step):
    """utils.py:357-399 restated (the order and clamping of the reference generator)."""
    offw, offh = (W - P) % step, (H - P) % step
    for x in range(0, W - P + offw + 1, step):
        if x + P > W:
            x = W - P
        for y in range(0, H - P + offh + 1, step):
            if y + P > H:
                y = H - P
            yield x, y


@pytest.mark.parametrize("W,H,P,step", [(349, 1905, 9, 1), (20, 17, 9, 1), (20, 17, 9, 2), (8, 8, 3, 2),
                                        (30, 31, 11, 4), (9, 9, 9, 1)])
def test_window_count_matches_reference_generator(W, H, P, step):
    from vitcnn_amd.window import window_count
    if W * H > 10000:
        assert window_count(W, H, P, step) == (W - P + 1) * (H - P + 1)
    else:
        assert window_count(W, H, P, step) == sum(1 for _ in _ref_sliding_window_corners(W, H, P, step))


def test_get_model_defaults_and_unknown_name():
    from vitcnn_amd import model_utils as mu
    from vitcnn_amd import AdamW, CrossEntropyLoss, Multimodality_Mamba
    with pytest.raises(KeyError):
        mu.get_model("Mutimodality_Mamba", n_classes=16, n_bands=(144, 1), ignored_labels=[0], dataset="Houston2013")
    model, opt, crit, kw = mu.get_model("Multimodality_Mamba", n_classes=16, n_bands=(144, 1), ignored_labels=[0],
                                        dataset="Houston2013", device=torch.device("cpu"))
    assert isinstance(model, Multimodality_Mamba) and isinstance(opt, AdamW) and isinstance(crit, CrossEntropyLoss)
    assert kw["patch_size"] == 9 and kw["lr"] == 8e-4 and kw["epoch"] == 200 and kw["batch_size"] == 64
    assert kw["center_pixel"] is True and kw["supervision"] == "full" and kw["applyPCA"] is False
    sch = kw["scheduler"]
    assert isinstance(sch, torch.optim.lr_scheduler.StepLR) and sch.step_size == 30 and sch.gamma == 0.9
    assert opt.param_groups[0]["lr"] == 8e-4 and opt.param_groups[0]["weight_decay"] == 1e-2
    w = kw["weights"]
    assert w[0] == 0 and float(w[1:].sum()) == 15
    assert sum(p.numel() for p in model.parameters()) == 1661260
    # 1,660,090 of them receive gradients; in the flat buffer every parameter starts 16-B aligned, so the
    # active section [0, n_active) also holds zero-filled alignment gaps (fewer than 4 floats each)
    from vitcnn_amd.model import UNUSED_PREFIXES
    named = dict(model.named_parameters())
    active = [n for n in named if not n.startswith(UNUSED_PREFIXES)]
    assert sum(named[n].numel() for n in active) == 1661260 - 1170
    assert all(model._poff[n] % 4 == 0 for n in named if named[n].numel() >= 64)
    assert model.n_active_params % 4 == 0 and 0 <= model.n_active_params - 1660090 < 4 * len(active)
    assert len(model._gaps) == model.n_active_params - 1660090


def test_state_dict_contract():
    from vitcnn_amd import Multimodality_Mamba
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16, "multi_clock_gate")
    ref = reference_keys()
    sd = m.state_dict()
    assert list(sd.keys()) == [e["name"] for e in ref]
    for e in ref:
        assert tuple(sd[e["name"]].shape) == tuple(e["shape"]), e["name"]
    # round trip through load_state_dict keeps the flat storage
    sd2 = {k: (torch.randn_like(v) if v.is_floating_point() else v) for k, v in sd.items()}
    m.load_state_dict(sd2)
    for k, v in m.state_dict().items():
        assert torch.equal(v, sd2[k]), k
    flat = m.flat_params
    p = dict(m.named_parameters())["classifier.weight"]
    assert p.data_ptr() == flat.data_ptr() + 4 * m._poff["classifier.weight"]


def test_scan_orders_match_reference_tables():
    from vitcnn_amd.scan_orders import inverse, scan_orders
    with open(os.path.join(GOLDEN, "scan_orders.json")) as f:
        ref = json.load(f)
    for n, key in ((9, "n9"), (7, "n7")):
        o = scan_orders(n)
        for k, name in ((2, "vf"), (4, "37df"), (6, "19df"), (8, "ltcw"), (9, "ltacw")):
            assert o[k] == ref[key][name], (key, name)
        assert o[0] == list(range(n * n)) and o[1] == o[0][::-1]
        for k in (3, 5, 7):  # reversed directions
            assert o[k] == o[k - 1][::-1]
        for t in o:
            inv = inverse(t)
            assert [t[i] for i in inv] == list(range(n * n))


def test_shard_indices_disjoint_cover():
    from vitcnn_amd.parallel import shard_indices
    for n, world in [(1000, 8), (1001, 8), (7, 2), (64 * 8, 8)]:
        shards = [shard_indices(n, r, world, seed=3) for r in range(world)]
        assert len({len(s) for s in shards}) == 1
        allidx = np.concatenate(shards)
        assert set(allidx.tolist()) == set(range(n))
        if n % world == 0:
            assert len(allidx) == n and len(set(allidx.tolist())) == n


def test_camel_to_snake_and_checkpoint_scheme(tmp_path, monkeypatch):
    from vitcnn_amd import Multimodality_Mamba
    from vitcnn_amd import model_utils as mu
    assert mu.camel_to_snake("Multimodality_Mamba") == "multimodality__mamba"
    monkeypatch.chdir(tmp_path)
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16)
    path = mu.save_model("x", m, mu.camel_to_snake(m.__class__.__name__), "Houston2013", train_state="train",
                         type="best_epoch", run=0, epoch=10, metric=0.5)
    assert path.startswith("./checkpoints/multimodality__mamba/Houston2013/train/best_epoch/")
    assert path.endswith("x_run0_epoch10_0.50.pth")
    sd = torch.load(path, weights_only=True)
    assert list(sd.keys()) == [e["name"] for e in reference_keys()]


def test_product_path_has_no_cpu_fallback():
    from vitcnn_amd import CrossEntropyLoss, Multimodality_Mamba
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m(torch.zeros(2, 144, 9, 9), torch.zeros(2, 1, 9, 9))
    with pytest.raises(RuntimeError):
        CrossEntropyLoss()(torch.zeros(2, 16), torch.zeros(2, dtype=torch.int64))


def test_window_xform_codes_follow_reference_distribution():
    """PatchBatcher's flip/rot decisions use the reference's branch structure (datasets.py:511-526)."""
    from vitcnn_amd.window import PatchBatcher
    pb = PatchBatcher.__new__(PatchBatcher)
    pb.flip, pb.P, pb.rng = True, 9, np.random.RandomState(0)
    pb.radiation = pb.mixture = False
    codes = pb.xform_codes(20000)
    flips = (codes & 3) != 0
    rots = (codes >> 2) != 0
    assert not np.any(flips & rots)
    # P(flip branch) = 0.5 * P(at least one of h/v) = 0.375; P(rotate) = 0.25
    assert abs(flips.mean() - 0.375) < 0.02 and abs(rots.mean() - 0.25) < 0.02
    assert set(np.unique(codes >> 2).tolist()) <= {0, 1, 2, 3}


def test_to_same_device_keeps_workspaces_and_binding():
    """.to() onto the device the model is already on must not free the workspaces: train() calls
    net.to(device) on entry, and hipGraphs captured by an earlier train() call write into them (a
    rebind there freed memory a replayed graph then wrote to).  A real move, a scratch growth or a
    re-flatten bumps the binding generation the TrainStepper checks before replaying."""
    from vitcnn_amd import Multimodality_Mamba
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16)
    ws = m._workspace("cpu", 4, ("train", "grad"))
    gen = m._bind_gen
    m.to("cpu")
    m.to(torch.device("cpu"))
    assert m._bind_gen == gen and m._ws.get(("cpu", 4, ("train", "grad"))) is ws
    m._scratch("cpu", 4)
    m._scratch("cpu", 4096)                       # grows: the old scratch is gone
    assert m._bind_gen == gen + 1
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m.load_state_dict(sd, assign=True)
    m._ensure_flat()
    assert m._bind_gen == gen + 2 and not m._ws
