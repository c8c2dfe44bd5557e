"""Data-parallel path on CPU processes (gloo, world size 2): the exchange step of SURVEY.md 8(e).

Each rank computes the oracle gradient of its own shard (the per-rank B-patch step, BatchNorm
local as in the MI355X path), writes it into the model's flat gradient layout and calls
`parallel.allreduce_gradients`; the result must equal the mean of both shards' gradients computed
in one process.  Parameter / buffer broadcasts are checked the same way.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import golden_batch, hash_state_dict

B_SHARD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_grad(model, sd, r):
    """oracle gradient of shard r in the model's flat layout"""
    from oracle import vitcnn_oracle as O
    hsi, lidar, target = golden_batch("golden.b4", 4)
    sl = slice(r * B_SHARD, (r + 1) * B_SHARD)
    st = O.make_state(sd)
    O.train_step(st, hsi[sl], lidar[sl], target[sl], O.ce_class_weights(16))
    flat = torch.zeros(model.flat_params.numel())
    for n, off in model._poff.items():
        g = st[n].grad
        if g is not None:
            flat[off:off + g.numel()] = g.reshape(-1)
    return flat


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    from vitcnn_amd import Multimodality_Mamba, parallel
    r, w, _ = parallel.init_from_env(backend="gloo")
    assert (r, w) == (rank, world) and parallel.is_distributed()
    sd = hash_state_dict()
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16)
    m.load_state_dict(sd)
    # replicas diverge, then broadcast_parameters makes them identical to rank 0
    with torch.no_grad():
        m.flat_params.add_(float(rank))
        m.flat_buffers()[0].add_(float(rank))
    parallel.broadcast_parameters(m)
    parallel.broadcast_buffers(m)
    ok_bcast = bool(torch.equal(m.flat_params.detach(), _load(sd).flat_params.detach()))
    ok_buf = bool(torch.equal(m.flat_buffers()[0], _load(sd).flat_buffers()[0]))
    m.flat_params.grad = _shard_grad(m, sd, rank)

    class _Opt:
        grad_scale = 1.0

    opt = _Opt()
    parallel.allreduce_gradients(m, opt)
    g = m.flat_params.grad * opt.grad_scale
    if rank == 0:
        out.put((ok_bcast, ok_buf, g[: m.n_active_params].clone(), float(opt.grad_scale),
                 float(m.flat_params.grad[m.n_active_params:].abs().sum())))
    dist.barrier()
    dist.destroy_process_group()


def _load(sd):
    from vitcnn_amd import Multimodality_Mamba
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16)
    m.load_state_dict(sd)
    return m


def test_allreduce_equals_mean_of_shard_gradients():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        ok_bcast, ok_buf, g, scale, tail = q.get(timeout=600)
    finally:
        for p in procs:
            p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs)
    assert ok_bcast and ok_buf
    assert scale == 0.5 and tail == 0.0
    sd = hash_state_dict()
    m = _load(sd)
    nt = torch.get_num_threads()
    torch.set_num_threads(2)  # the workers' thread count: same CPU reduction order
    try:
        ref = (_shard_grad(m, sd, 0) + _shard_grad(m, sd, 1))[: m.n_active_params] / 2
    finally:
        torch.set_num_threads(nt)
    err = float((g - ref).abs().max() / ref.abs().max())
    assert err < 1e-6, err


def _s2eft_worker(rank, world, port, out):
    """config 5 data parallelism: each rank's S2EFT shard gradient (oracle, B = 2 of the golden
    batch) in the model's flat layout, all-reduced through the same helpers as ViT-CNN"""
    import numpy as np
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    from oracle import s2eft_oracle as O
    from vitcnn_amd import parallel
    from vitcnn_amd.optim import AdamW
    from vitcnn_amd.s2eft import ViT
    parallel.init_from_env(backend="gloo")
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "s2eft_b4.npz"))
    sd = {k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("p:")}
    m = ViT(image_size=7, near_band=3, num_patches=144, num_classes=16, dim=64, depth=5, heads=4, mlp_dim=8)
    m.load_state_dict(sd)
    opt = AdamW(m.parameters(), lr=5e-4, weight_decay=0.0)
    sl = slice(rank * 2, rank * 2 + 2)
    x, t, w = torch.from_numpy(z["x"])[sl], torch.from_numpy(z["target"])[sl], torch.from_numpy(z["weight"])
    _, _, g = O.train_step(sd, x, t, w)
    fl = torch.zeros(m.flat_params.numel())   # the model's flat layout (16-B aligned parameters, zero gaps)
    for n, o in m._poff.items():
        fl[o:o + g[n].numel()] = g[n].reshape(-1)
    m.flat_params.grad = fl
    parallel.allreduce_gradients(m, opt)
    G = m.flat_params.grad * opt.grad_scale
    out[rank] = (torch.cat([G[o:o + g[n].numel()] for n, o in m._poff.items()]), opt.grad_scale)
    dist.destroy_process_group()


def test_s2eft_gradient_allreduce_world2():
    import numpy as np
    from oracle import s2eft_oracle as O
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_s2eft_worker, args=(2, port, out), nprocs=2, join=True)
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "s2eft_b4.npz"))
    sd = {k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("p:")}
    x, t, w = torch.from_numpy(z["x"]), torch.from_numpy(z["target"]), torch.from_numpy(z["weight"])
    names = list(sd.keys())
    mean = None
    for r in range(2):
        _, _, g = O.train_step(sd, x[r * 2:r * 2 + 2], t[r * 2:r * 2 + 2], w)
        flat = torch.cat([g[n].reshape(-1) for n in names])
        mean = flat / 2 if mean is None else mean + flat / 2
    for r in range(2):
        got, scale = out[r]
        assert scale == 0.5
        assert torch.allclose(got, mean, rtol=1e-5, atol=1e-7)


def _perparam_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from vitcnn_amd import parallel
    parallel.init_from_env(backend="gloo")
    m = torch.nn.Sequential(torch.nn.Linear(3, 4), torch.nn.Linear(4, 2))
    for i, p in enumerate(m.parameters()):
        p.grad = torch.full_like(p, float(rank + 1) * (i + 1))
    opt = torch.optim.Adam(m.parameters())
    parallel.allreduce_gradients(m, opt)
    out[rank] = [p.grad.clone() for p in m.parameters()]
    dist.destroy_process_group()


def test_perparam_gradient_allreduce_world2():
    """models without the flat buffer (FusAtNet with torch Adam): per-parameter gradients averaged"""
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_perparam_worker, args=(2, port, out), nprocs=2, join=True)
    for r in range(2):
        for i, g in enumerate(out[r]):
            assert torch.allclose(g, torch.full_like(g, 1.5 * (i + 1)))


def _bucket_worker(rank, world, port, out):
    """GradExchange (the bench / fused-step exchange): each rank's oracle shard gradient is
    all-reduced bucket by bucket in the backward's completion order; world 4."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from vitcnn_amd import Multimodality_Mamba, parallel
    parallel.init_from_env(backend="gloo")
    sd = hash_state_dict()
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16)
    m.load_state_dict(sd)
    ex = parallel.GradExchange(m)
    grad = ex.begin(m, "cpu")
    grad.copy_(_shard_grad8(m, sd, rank, world))

    class _Opt:
        grad_scale = 1.0

    opt = _Opt()
    for name in ex.order:
        ex.bucket_ready(name, ())
    ex.finish(opt)
    out[rank] = (grad[: m.n_active_params].clone() * opt.grad_scale, opt.grad_scale, dict(ex.ranges))
    dist.destroy_process_group()


def _shard_grad8(model, sd, r, world):
    """oracle gradient of shard r of an 8-patch batch split over `world` ranks, flat layout"""
    from oracle import vitcnn_oracle as O
    hsi, lidar, target = golden_batch("golden.dp8", 8)
    b = 8 // world
    sl = slice(r * b, (r + 1) * b)
    st = O.make_state(sd)
    O.train_step(st, hsi[sl], lidar[sl], target[sl], O.ce_class_weights(16))
    flat = torch.zeros(model.flat_params.numel())
    for n, off in model._poff.items():
        g = st[n].grad
        if g is not None:
            flat[off:off + g.numel()] = g.reshape(-1)
    return flat


def test_bucketed_exchange_world4_equals_mean_of_shards():
    """SURVEY.md 8(e) / VERDICT item 4: three head-first buckets (LiDAR+fusion+classifier, hsi2,
    hsi1) tile the active gradient; their all-reduce over 4 ranks = the mean of the 4 shards'
    oracle gradients, with 1/world folded into the optimizer's grad_scale."""
    world = 4
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_bucket_worker, args=(world, port, out), nprocs=world, join=True)
    sd = hash_state_dict()
    m = _load(sd)
    nt = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        ref = sum(_shard_grad8(m, sd, r, world) for r in range(world))[: m.n_active_params] / world
    finally:
        torch.set_num_threads(nt)
    ranges = out[0][2]
    # the buckets tile [0, n_active): hsi1 first in the layout, then hsi2, then the tail (LiDAR, fusion,
    # classifier), each holding exactly its block's parameters (plus alignment gaps)
    assert ranges["hsi1"][0] == 0 and ranges["hsi1"][1] == ranges["hsi2"][0]
    assert ranges["hsi2"][1] == ranges["tail"][0] and ranges["tail"][1] == m.n_active_params
    named = dict(m.named_parameters())
    for n, o in m._poff.items():
        if o >= m.n_active_params:
            continue
        b = "hsi1" if n.startswith("hsi1.") else "hsi2" if n.startswith("hsi2.") else "tail"
        assert ranges[b][0] <= o and o + named[n].numel() <= ranges[b][1], n
    for r in range(world):
        g, scale, _ = out[r]
        assert scale == 1.0 / world
        err = float((g - ref).abs().max() / ref.abs().max())
        assert err < 1e-6, (r, err)


def test_bucket_order_is_checked():
    from vitcnn_amd import Multimodality_Mamba, parallel
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16)
    ex = parallel.GradExchange(m)
    ex.begin(m, "cpu")
    ex.bucket_ready("hsi2")
    ex.bucket_ready("tail")
    ex.bucket_ready("hsi1")
    with pytest.raises(RuntimeError):
        ex.finish()


def _bn_model_worker(rank, world, port, out):
    """models without flat buffers (FusAtNet-like: Conv + BatchNorm, torch optimizer): parameter and
    buffer broadcasts, and a gradient bucket when one rank's graph left a parameter without .grad"""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from vitcnn_amd import parallel
    parallel.init_from_env(backend="gloo")
    torch.manual_seed(rank)
    m = torch.nn.Sequential(torch.nn.Conv2d(2, 3, 3), torch.nn.BatchNorm2d(3), torch.nn.Linear(3, 2))
    m.train()
    m(torch.rand(4, 2, 5, 5))   # rank-dependent running statistics
    parallel.broadcast_parameters(m)
    parallel.broadcast_buffers(m)
    params = [p.detach().clone() for p in m.parameters()]
    bufs = [b.clone() for b in m.buffers()]
    for i, p in enumerate(m.parameters()):
        p.grad = None if (rank == 1 and i == 0) else torch.full_like(p, float(rank + 1))
    parallel.allreduce_gradients(m, torch.optim.Adam(m.parameters()))
    out[rank] = (params, bufs, [p.grad.clone() for p in m.parameters()])
    dist.destroy_process_group()


def test_broadcasts_and_sparse_grads_without_flat_buffers():
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_bn_model_worker, args=(2, port, out), nprocs=2, join=True)
    p0, b0, g0 = out[0]
    p1, b1, g1 = out[1]
    assert all(torch.equal(a, b) for a, b in zip(p0, p1))
    assert all(torch.equal(a, b) for a, b in zip(b0, b1))
    for i, (a, b) in enumerate(zip(g0, g1)):
        expect = 0.5 if i == 0 else 1.5     # rank 1 had no gradient for parameter 0: it counts as zeros
        assert torch.allclose(a, torch.full_like(a, expect)) and torch.equal(a, b)


def test_sharded_loader_partitions_batches():
    from vitcnn_amd import parallel
    batches = list(range(11))

    class _L(list):
        dataset = None

    loader = _L(batches)
    parts = [list(parallel.ShardedLoader(loader, r, 4)) for r in range(4)]
    # every batch once, padded by wrapping so that every rank gets the same number (one
    # gradient all-reduce per batch must pair up across ranks): 11 batches -> 3 + 3 + 3 + 3
    assert sorted(set(sum(parts, []))) == batches
    assert [len(p) for p in parts] == [3, 3, 3, 3] and parts[3] == [3, 7, 0]
    assert [len(parallel.ShardedLoader(loader, r, 4)) for r in range(4)] == [len(p) for p in parts]
