"""Two real HIP ranks through `model_utils.train`.

Two processes share the one leased MI355X and form a gloo group (RCCL refuses two ranks on one
device; gloo moves the CUDA buckets through the host).  Each rank builds the product model with
`get_model("Multimodality_Mamba")`, the same hash-initialised parameters, and its own `PatchBatcher`
shard of one synthetic scene (rank / world / seed: the sharding train() must not repeat).  What is
checked -- the loop being sharded is the reference's `model_utils.py:906-936` over the `main.py:434-440`
loader:

* the first step's exchanged flat gradient (`fused_train_step(exchange=GradExchange)`: the three
  head-first buckets all-reduced on the exchange's side stream while the backward runs) is the same
  on both ranks and equals the sum of the two ranks' local HIP gradients, and its mean equals the mean
  of the two shards' oracle gradients within the per-tensor tolerance of
  test_model_gpu.py::test_gradients_b4 (float64 yardstick with each shard's ReLU decisions and
  TokenLearner pooled values, or 3x the fp32 reference's own error);
* `train()` for two epochs over the PatchBatcher shards -- the fused step eagerly (gloo collectives are
  not capturable: `launch` says so), the bucket exchange, the fused AdamW with the 1/world average --
  ends with identical flat parameters, BatchNorm running statistics and counters on both ranks, and
  both ranks ran the same number of batches.
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

B, WORLD, EPOCHS = 4, 2, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scene():
    """a 26 x 24 scene of 9 regions with their own band profiles (as test_window_gpu's production test:
    i.i.d. pixels would make every TokenLearner BN(1) input nearly constant over the batch -- the
    ill-conditioned case DESIGN.md section 6 describes), ~40 % of the pixels labelled"""
    rng = np.random.default_rng(21)
    W, H = 26, 24
    xx, yy = np.meshgrid(np.arange(W), np.arange(H), indexing="ij")
    region = (xx * 3 // W) * 3 + (yy * 3 // H)
    prof = rng.random((9, 144), dtype=np.float32)
    img1 = (0.7 * prof[region] + 0.3 * rng.random((W, H, 144), dtype=np.float32)).astype(np.float32)
    img2 = (region[:, :, None] / 9.0 + 0.1 * rng.random((W, H, 1))).astype(np.float32)
    gt = (1 + region + rng.integers(0, 2, size=(W, H)) * 6) % 16
    gt[rng.random((W, H)) < 0.6] = 0          # ~40 % labelled: ~6 batches of 4 per rank
    return img1, img2, gt


def _worker(rank, world, port, tmp, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    os.chdir(tmp)
    import torch.distributed as dist
    from helpers import hash_state_dict, relu_masks_from_workspace, tl_pooled_from_workspace
    from vitcnn_amd import fused_train_step
    from vitcnn_amd import model_utils as mu
    from vitcnn_amd import parallel
    from vitcnn_amd.window import PatchBatcher
    parallel.init_from_env(backend="gloo")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    sd = hash_state_dict()
    model, opt, crit, hp = mu.get_model("Multimodality_Mamba", n_classes=16, n_bands=(144, 1), ignored_labels=[0],
                                        dataset="synthetic", device=dev)
    model.load_state_dict(sd)
    img1, img2, gt = _scene()
    loader = PatchBatcher(img1, img2, gt, 9, ignored_labels=[0], batch_size=B, device=dev, seed=5, rank=rank,
                          world=world)
    x1, x2, t = next(iter(loader))
    loader.gid = 0
    # 1. the first step's exchanged gradient (no optimizer step: the exchange leaves the mean)
    ex = parallel.GradExchange(model)
    model.zero_grad(set_to_none=True)
    fused_train_step(model, crit, x1, x2, t, optimizer=None, exchange=ex)
    torch.cuda.synchronize()
    g_sum = model.flat_params.grad.detach().cpu().clone()
    # 2. this rank's local gradient of the same batch (no exchange), and the HIP path's decisions
    model.load_state_dict(sd)                  # the running statistics the first forward updated
    model.zero_grad(set_to_none=True)
    fused_train_step(model, crit, x1, x2, t)
    torch.cuda.synchronize()
    g_loc = model.flat_params.grad.detach().cpu().clone()
    masks = relu_masks_from_workspace(model, B)
    pooled = tl_pooled_from_workspace(model, B)
    # 3. train() over the PatchBatcher shards from the same initial state
    model.load_state_dict(sd)
    model.zero_grad(set_to_none=True)
    mu.train("t", 0, None, model, opt, crit, loader, EPOCHS, scheduler=hp["scheduler"], display_iter=0, device=dev)
    torch.cuda.synchronize()
    st = mu.train.last_stats
    bflat, iflat = model.flat_buffers()
    out[rank] = dict(batch=(x1.cpu(), x2.cpu(), t.cpu()), g_sum=g_sum, g_loc=g_loc, masks=masks, pooled=pooled,
                     flat=model.flat_params.detach().cpu().clone(), bflat=bflat.cpu().clone(),
                     iflat=iflat.cpu().clone(), launch=st["launch"], nb=[e["batches"] for e in st["epochs"]],
                     losses=list(st["losses"]), n_active=model.n_active_params,
                     poff=dict(model._poff), shapes={n: tuple(p.shape) for n, p in model.named_parameters()})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(900)
def test_train_world2_hip_ranks(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    from helpers import check_audit, hash_state_dict, masked_oracle_step
    from oracle import vitcnn_oracle as O
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(WORLD, port, str(tmp_path), out), nprocs=WORLD, join=True)
    r0, r1 = out[0], out[1]
    n_act = r0["n_active"]
    # the step ran the fused HIP program eagerly (gloo cannot be captured), never a torch fallback
    assert r0["launch"].startswith("eager") and "gloo" in r0["launch"], r0["launch"]
    # the two shards are different batches
    assert not torch.equal(r0["batch"][0], r1["batch"][0])
    # --- exchanged gradient: identical on both ranks, = the mean of the local gradients (without an
    # optimizer to fold the 1/world into, GradExchange.finish scales the summed buffer: exact, a power of 2)
    assert torch.equal(r0["g_sum"], r1["g_sum"])
    assert torch.equal(r0["g_sum"][:n_act], ((r0["g_loc"] + r1["g_loc"]) * 0.5)[:n_act])
    assert float(r0["g_sum"][n_act:].abs().sum()) == 0.0        # the never-used parameters' tail
    got_mean = r0["g_sum"].double()
    # --- the mean of the two shards' oracle gradients (test_gradients_b4's per-tensor criterion)
    sd = hash_state_dict()
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
    w = O.ce_class_weights(16)
    ref32, ref64, ref64_own = {}, {}, {}
    audit = []   # every adopted HIP decision of both ranks must be an fp32 near-tie
    for r in (r0, r1):
        hsi, lidar, target = r["batch"]
        st = O.make_state(sd)
        O.train_step(st, hsi, lidar, target, w)
        st64 = O.make_state(sd64)
        masked_oracle_step(O, st64, hsi.double(), lidar.double(), target, w.double(), r["masks"], pooled=r["pooled"],
                           audit=audit)
        st64o = O.make_state(sd64)
        O.train_step(st64o, hsi.double(), lidar.double(), target, w.double())
        for dst, s_ in ((ref32, st), (ref64, st64), (ref64_own, st64o)):
            for k in O.param_names(s_):
                g = s_[k].grad
                if g is None:
                    continue
                dst[k] = dst.get(k, 0) + g.double() / WORLD
    check_audit(audit, "dp_world2")
    # Every tensor element-wise (test_gradients_b4's criterion), the TokenLearner tokenizers included (VERDICT r4
    # item 1: round 4 held them to a norm only; the cause of their divergence is in DESIGN.md section 6)
    gmax = max(float(g.abs().max()) for g in ref64.values())
    floor = 1e-5 * gmax
    bad = []
    for n, off in r0["poff"].items():
        shape = r0["shapes"][n]
        numel = int(np.prod(shape)) if shape else 1
        got = got_mean[off:off + numel].view(shape)
        if n not in ref64:
            assert float(got.abs().max()) == 0.0, n
            continue
        err = float((got - ref64[n]).abs().max())
        err32 = float((ref32[n] - ref64_own[n]).abs().max())
        scale = float(ref64[n].abs().max())
        if not (err <= 1e-3 * scale + floor or err <= 3.0 * err32 + floor):
            bad.append((n, err, err32, scale))
    assert not bad, bad[:5]
    # --- after two epochs of train(): one model on both ranks
    assert r0["nb"] == r1["nb"] and len(r0["nb"]) == EPOCHS and r0["nb"][0] > 1
    assert r0["losses"] != r1["losses"]                  # the ranks trained on different shards
    assert torch.equal(r0["flat"], r1["flat"])
    assert torch.equal(r0["bflat"], r1["bflat"])          # broadcast from rank 0 at the last epoch
    assert torch.equal(r0["iflat"], r1["iflat"])
    assert not torch.equal(r0["flat"][:n_act], torch.cat([sd[n].reshape(-1) for n in r0["poff"]])[:n_act])
