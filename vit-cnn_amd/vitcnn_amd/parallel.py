"""Data parallelism for the ViT-CNN training step: one process per GPU, RCCL over xGMI.

The reference is single-process (`Mutimodality_Mamba7.py:60` pins
`cuda:0`); patches are independent, so the minibatch shards across ranks and the only exchange per
step is the gradient all-reduce.

* The model's gradients are ONE flat fp32 tensor (`model.flat_params.grad`).  `GradExchange` splits
  its active part (1,660,090 floats; the 1,170 never-used parameters sit at the tail and are
  excluded) into three contiguous buckets in the order the backward completes them, head side
  first: "tail" (LiDAR convs, fusion1/2, classifier: 65k floats), "hsi2" (722k), "hsi1" (873k).
  Each bucket's RCCL all-reduce is issued on a side stream as soon as the backward program has
  written it (`_Program.backward(bucket_hook=...)`), so the first two overlap the remaining
  backward; the optimizer step waits for the side stream.  The 1/world average is folded into the
  fused AdamW kernel (`AdamW.grad_scale`) instead of a separate scaling pass.  The buffers are
  persistent, so the whole step — forward, backward, the bucket all-reduces and AdamW — can be
  captured into one hipGraph (bench.py).
* `allreduce_gradients` is the single-bucket form used by `train()` and by models without the
  bucket layout (S2EFT's flat buffer; FusAtNet / plain torch modules: one flattened bucket over
  every parameter that requires grad, zeros for parameters that got none, so every rank's bucket
  has the same size and layout).
* BatchNorm stays local (not SyncBN): each rank's B=64 forward equals the reference's B=64
  forward.  Running statistics are rank-local during training; `broadcast_buffers` copies
  rank 0's before evaluation / checkpointing (DDP `broadcast_buffers` semantics).
* `broadcast_parameters` makes every replica start from rank 0's parameters (train() calls it).

Everything here also works with the `gloo` backend on CPU tensors, which is how the N>1 path is
tested without GPUs (tests/test_parallel_cpu.py).
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.distributed as dist


def is_distributed() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def world() -> int:
    return dist.get_world_size() if is_distributed() else 1


def rank() -> int:
    return dist.get_rank() if is_distributed() else 0


def init_from_env(backend: str | None = None):
    """Initialise the default process group from torchrun's env (RANK/WORLD_SIZE/MASTER_*).
    Returns (rank, world_size, local_rank).  A no-op for a single process."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1:
        return 0, 1, 0
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        dist.init_process_group(backend=backend)
    return dist.get_rank(), dist.get_world_size(), local


def active_grad(model) -> torch.Tensor | None:
    """View of the flat gradient over the parameters that receive gradients (the exchange set)."""
    flat = model.flat_params
    if flat.grad is None:
        return None
    return flat.grad[: model.n_active_params]


def _set_scale(optimizer, grad, n):
    if optimizer is not None and hasattr(optimizer, "grad_scale"):
        optimizer.grad_scale = 1.0 / n
    else:
        grad.mul_(1.0 / n)


def allreduce_gradients(model, optimizer=None, group=None):
    """Sum the gradient over ranks (one bucket); the 1/world average goes into the optimizer's fused
    update when it supports it (vitcnn_amd.AdamW.grad_scale), else the gradient is scaled."""
    if not is_distributed():
        if optimizer is not None and hasattr(optimizer, "grad_scale"):
            optimizer.grad_scale = 1.0
        return
    n = dist.get_world_size(group)
    if not hasattr(model, "flat_params"):
        # per-parameter gradients (torch modules): one flattened bucket over EVERY parameter that
        # requires grad (zeros where backward produced none), so the bucket size and offsets are the
        # same on every rank whatever the local graph touched.  A has-gradient flag per parameter is
        # summed first: a parameter no rank produced a gradient for keeps grad None (torch optimizers
        # skip it, as single-process training does) instead of receiving zeros that weight decay /
        # momentum would then act on.
        params = [p for p in model.parameters() if p.requires_grad]
        if not params:
            raise RuntimeError("allreduce_gradients: the model has no trainable parameters")
        dev = params[0].device
        has = torch.tensor([p.grad is not None for p in params], dtype=torch.int32, device=dev)
        dist.all_reduce(has, op=dist.ReduceOp.SUM, group=group)
        has = has.tolist()
        bucket = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in params])
        dist.all_reduce(bucket, op=dist.ReduceOp.SUM, group=group)
        bucket.mul_(1.0 / n)
        o = 0
        for p, h in zip(params, has):
            v = bucket[o:o + p.numel()].view_as(p)
            if h == 0:
                p.grad = None
            elif p.grad is None:
                p.grad = v.clone()
            else:
                p.grad.copy_(v)
            o += p.numel()
        return
    g = active_grad(model)
    if g is None:
        raise RuntimeError("allreduce_gradients: backward has not produced a gradient")
    dist.all_reduce(g, op=dist.ReduceOp.SUM, group=group)
    _set_scale(optimizer, g, n)


# bucket name -> state_dict prefixes, in the order the backward program completes them
BUCKETS = (("tail", ("lidar1.", "lidar2.", "fusion1.", "fusion2.", "classifier.")),
           ("hsi2", ("hsi2.",)),
           ("hsi1", ("hsi1.",)))


def bucket_ranges(model):
    """{bucket: (lo, hi)} over the model's flat parameter layout; the buckets are contiguous,
    disjoint and together cover exactly the active parameters [0, n_active).  Parameters start 16-B
    aligned (model.PARAM_ALIGN), so a bucket may hold alignment gaps (< 4 floats each, zero in every
    gradient); each bucket runs up to the next bucket's first parameter."""
    named = dict(model.named_parameters())
    spans = {}
    for name, prefixes in BUCKETS:
        offs = sorted((o, o + named[n].numel()) for n, o in model._poff.items()
                      if n.startswith(prefixes) and o < model.n_active_params)
        if any(b[0] - a[1] >= 4 or b[0] < a[1] for a, b in zip(offs, offs[1:])):
            raise RuntimeError(f"gradient bucket {name} is not contiguous in the flat layout")
        spans[name] = (offs[0][0], offs[-1][1])
    order = sorted(spans, key=lambda k: spans[k][0])
    if spans[order[0]][0] != 0 or spans[order[-1]][1] > model.n_active_params:
        raise RuntimeError("gradient buckets do not tile the active parameters")
    out = {}
    for i, name in enumerate(order):
        hi = spans[order[i + 1]][0] if i + 1 < len(order) else model.n_active_params
        if hi - spans[name][1] >= 4 or hi < spans[name][1]:
            raise RuntimeError("gradient buckets do not tile the active parameters")
        out[name] = (spans[name][0], hi)
    return out


class GradExchange:
    """Bucketed gradient all-reduce overlapped with the backward.

    Usage (vitcnn_amd.step.fused_train_step(..., exchange=ex)):
        grad = ex.begin(model, device)            # persistent flat gradient buffer
        prog.backward(dlog, bucket_hook=ex.bucket_ready, out=grad)
        ex.finish(optimizer)                       # caller's stream waits for the last bucket
    On GPU tensors each bucket's collective runs on the exchange's side stream after the events the
    backward hands over; on CPU (gloo) it runs inline.  `force` exchanges even in a world of one
    (exercises the collective path on a single device)."""

    def __init__(self, model, group=None, force: bool = False):
        self.ranges = bucket_ranges(model)
        self.order = [n for n, _ in BUCKETS]
        self.group = group
        self.force = force
        self.grad = None
        self.stream = None
        self.done = []

    @property
    def active(self) -> bool:
        return is_distributed() or (self.force and dist.is_available() and dist.is_initialized())

    def begin(self, model, device):
        n = model.flat_params.numel()
        if self.grad is None or self.grad.numel() != n or self.grad.device != torch.device(device):
            self.grad = torch.empty(n, dtype=torch.float32, device=device)
            if self.grad.is_cuda:
                self.stream = torch.cuda.Stream(device)
        self.done = []
        return self.grad

    def bucket_ready(self, name, events=()):
        """all-reduce bucket `name` of the current gradient once `events` have fired"""
        self.done.append(name)
        if not self.active:
            return
        lo, hi = self.ranges[name]
        t = self.grad[lo:hi]
        if t.is_cuda:
            for e in events:
                self.stream.wait_event(e)
            with torch.cuda.stream(self.stream):
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)

    def finish(self, optimizer=None):
        if self.done != self.order:
            raise RuntimeError(f"gradient buckets completed as {self.done}, expected {self.order}")
        n = dist.get_world_size(self.group) if self.active else 1
        if self.grad.is_cuda and self.active:
            torch.cuda.current_stream(self.grad.device).wait_stream(self.stream)
        if optimizer is not None and hasattr(optimizer, "grad_scale"):
            optimizer.grad_scale = 1.0 / n
        elif n > 1:
            self.grad.mul_(1.0 / n)


def _scalar_device(group=None):
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")


def mean_over_ranks(x: float, group=None) -> float:
    """The mean of a host scalar over the ranks (every rank returns the same value): train() decides
    its best-epoch branch -- which contains collectives -- on this, never on a rank-local number."""
    if not is_distributed():
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=_scalar_device(group))
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return float(t.item()) / dist.get_world_size(group)


def sum_over_ranks(values, group=None):
    """Element-wise sum of a list of host numbers over the ranks (float64)."""
    if not is_distributed():
        return [float(v) for v in values]
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=_scalar_device(group))
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t.tolist()


def broadcast_parameters(model, src: int = 0, group=None):
    """Make every replica start from rank `src`'s parameters: one broadcast of the flat buffer, or of
    one flattened bucket for models without it."""
    if not is_distributed():
        return
    with torch.no_grad():
        if hasattr(model, "flat_params"):
            dist.broadcast(model.flat_params.data, src=src, group=group)
            return
        params = [p for p in model.parameters()]
        if not params:
            return
        bucket = torch.cat([p.detach().reshape(-1) for p in params])
        dist.broadcast(bucket, src=src, group=group)
        o = 0
        for p in params:
            p.data.copy_(bucket[o:o + p.numel()].view_as(p))
            o += p.numel()


def broadcast_buffers(model, src: int = 0, group=None):
    """BN running statistics and counters from rank `src` (before eval / checkpoint): the model's two
    flat buffers, or every registered buffer for models without them."""
    if not is_distributed():
        return
    if hasattr(model, "flat_buffers"):
        for b in model.flat_buffers():
            dist.broadcast(b, src=src, group=group)
        return
    for b in model.buffers():
        dist.broadcast(b, src=src, group=group)


def shard_indices(n: int, rank_: int, world_: int, seed: int = 0, epoch: int = 0, shuffle: bool = True):
    """DistributedSampler-style disjoint shard of range(n): shuffle with (seed + epoch), pad to a
    multiple of world by wrapping, then take every world-th index starting at rank."""
    idx = np.arange(n)
    if shuffle:
        idx = np.random.default_rng(seed + epoch).permutation(n)
    per = -(-n // world_)
    total = per * world_
    if total > n:
        idx = np.concatenate([idx, idx[: total - n]])
    return idx[rank_:total:world_]


def rank_batches(n: int, rank_: int, world_: int):
    """Batch positions rank `rank_` trains on out of a pass of `n` batches: b = rank_, rank_ + world_, ...
    over the pass padded by wrapping to ceil(n / world_) * world_ (as `shard_indices` / DistributedSampler
    pad their index lists), so EVERY rank gets the same number of batches -- train() issues one gradient
    all-reduce per batch, and ranks with different batch counts would pair their collectives across
    epochs (or block forever in the last one).  Padded position j repeats batch j % n."""
    if n <= 0:
        return []
    total = -(-n // world_) * world_
    return [j % n for j in range(rank_, total, world_)]


def _broadcast_order(order, group=None):
    """rank 0's sample order, on every rank (one broadcast of its length, one of the indices)"""
    dev = _scalar_device(group)
    n = torch.tensor([len(order) if rank() == 0 else 0], dtype=torch.int64, device=dev)
    dist.broadcast(n, src=0, group=group)
    t = torch.tensor(order if rank() == 0 else [0] * int(n.item()), dtype=torch.int64, device=dev)
    dist.broadcast(t, src=0, group=group)
    return t.cpu().tolist()


class ShardedLoader:
    """Wrap a reference-style loader (batches of (data, data2, target)) so each rank iterates a disjoint
    shard of the pass's batches -- batch b goes to rank b % world, every rank the same number of batches
    (`rank_batches`) -- and materialises ONLY its own batches:

    * a torch DataLoader (main.py:434-440: MultiModalX, shuffle=True, num_workers=0): sharded at the
      sampler level.  Each pass, rank 0 draws the loader's own sample order (its RandomSampler, i.e. the
      draw a single-process epoch would make) and broadcasts it; every rank cuts that shared order into
      the loader's batches and builds a DataLoader over its own batch list (same dataset, collate_fn,
      workers).  The shards are disjoint by construction, whatever each rank's torch seed is;
    * an indexable loader (a list of batches): rank r takes its batch positions directly;
    * any other iterable: the pass is iterated and the other ranks' batches are discarded (the only form
      that assembles every batch on every rank; documented fallback).

    Used by train() when a process group is up and the loader is not already sharded (a loader whose
    sampler is a DistributedSampler, or which carries `rank`/`world` attributes -- PatchBatcher -- is)."""

    def __init__(self, loader, rank_, world_, group=None):
        self.loader, self.rank, self.world, self.group = loader, rank_, world_, group
        self.dataset = getattr(loader, "dataset", None)
        DL = torch.utils.data.DataLoader
        if isinstance(loader, DL) and loader.batch_size is not None and \
                not isinstance(loader.dataset, torch.utils.data.IterableDataset):
            self.mode = "sampler"
        elif hasattr(loader, "__getitem__") and hasattr(loader, "__len__"):
            self.mode = "indexed"
        else:
            self.mode = "iterate"

    def __len__(self):
        n = len(self.loader)
        return -(-n // self.world) if n > 0 else 0

    def __iter__(self):
        if self.mode == "sampler":
            yield from self._iter_sampler()
        elif self.mode == "indexed":
            for b in rank_batches(len(self.loader), self.rank, self.world):
                yield self.loader[b]
        else:
            yield from self._iter_discard()

    def _iter_sampler(self):
        ld = self.loader
        if self.world > 1 and not is_distributed():
            raise RuntimeError("ShardedLoader(mode='sampler') with world > 1 needs a process group: each rank would "
                               "draw its own sample order and the shards would overlap")
        # the order is drawn by rank 0's sampler from a dedicated generator (seeded from rank 0's torch RNG, the
        # draw a single-process epoch makes), so the ranks' global RNG states stay in step: every rank consumes
        # one draw for the seed, only rank 0 uses it
        seed = int(torch.empty((), dtype=torch.int64).random_().item())
        if is_distributed():
            order = _broadcast_order(self._draw_order(seed) if rank() == 0 else [], self.group)
        else:
            order = self._draw_order(seed)
        bs = ld.batch_size
        batches = [order[i:i + bs] for i in range(0, len(order), bs)]
        if ld.drop_last and batches and len(batches[-1]) < bs:
            batches.pop()
        mine = [batches[b] for b in rank_batches(len(batches), self.rank, self.world)]
        kw = dict(num_workers=ld.num_workers, collate_fn=ld.collate_fn, pin_memory=ld.pin_memory,
                  worker_init_fn=ld.worker_init_fn, timeout=ld.timeout, generator=ld.generator,
                  multiprocessing_context=ld.multiprocessing_context)
        if ld.num_workers > 0:
            kw.update(persistent_workers=ld.persistent_workers, prefetch_factor=ld.prefetch_factor)
        sub = torch.utils.data.DataLoader(ld.dataset, batch_sampler=mine, **kw)
        yield from sub

    def _draw_order(self, seed):
        """the loader's sampler order; a RandomSampler without its own generator draws from a dedicated one"""
        smp = self.loader.sampler
        if isinstance(smp, torch.utils.data.RandomSampler) and smp.generator is None:
            g = torch.Generator()
            g.manual_seed(seed)
            smp.generator = g
            try:
                return list(iter(smp))
            finally:
                smp.generator = None
        return list(iter(smp))

    def _iter_discard(self):
        """stream the pass: a batch this rank owns at its first position (b % world == rank, b < n) is yielded
        as it arrives; only the wrap-around padding batches (positions j >= n repeat batch j % n, all among the
        pass's first `world` batches) are kept until the pass ends"""
        n = len(self.loader)
        pad = [j % n for j in range(n, -(-n // self.world) * self.world) if j % self.world == self.rank] if n else []
        need_pad = set(pad)
        kept = {}
        for b, item in enumerate(self.loader):
            if b in need_pad:
                kept[b] = item
            if b % self.world == self.rank:
                yield item
        for b in pad:
            yield kept[b]


def is_sharded(loader) -> bool:
    sampler = getattr(loader, "sampler", None)
    if isinstance(sampler, torch.utils.data.distributed.DistributedSampler):
        return True
    if isinstance(loader, ShardedLoader):
        return True
    ds = getattr(loader, "dataset", None)
    return getattr(ds, "world", 1) > 1 or getattr(loader, "world", 1) > 1


def check_loader_shard(loader, group=None):
    """A loader that shards itself (PatchBatcher: `rank` / `world` / `seed`) must agree with the process
    group: its rank and world are this process's, and every rank built it from the same seed (the
    shuffled order the shards are cut from is then the same permutation on every rank).  Raises
    RuntimeError otherwise -- nothing else would notice overlapping or missing shards."""
    if not is_distributed() or getattr(loader, "world", None) is None:
        return
    # a world-1 loader does not shard itself (train() wraps it in a ShardedLoader, each rank taking batches
    # b % world of ITS OWN shuffled order), so only its rank / world are exempt: the seeds must still agree
    if int(loader.world) > 1 and (int(loader.world) != world() or int(loader.rank) != rank()):
        raise RuntimeError(f"loader shard (rank {loader.rank} of {loader.world}) does not match the process group "
                           f"(rank {rank()} of {world()})")
    seed = getattr(loader, "seed", None)
    if seed is not None:
        s = int(seed) & ((1 << 62) - 1)
        t = torch.tensor([s, -s], dtype=torch.int64, device=_scalar_device(group))
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        if int(t[0].item()) != -int(t[1].item()):
            raise RuntimeError("the ranks' loaders were built from different seeds: their shards would overlap")


def capturable(group=None) -> bool:
    """Can the gradient exchange be captured into a hipGraph?  RCCL ("nccl") collectives can; gloo's
    host-side collectives cannot, so a gloo-backed data-parallel step runs eagerly."""
    return not is_distributed() or dist.get_backend(group) == "nccl"
