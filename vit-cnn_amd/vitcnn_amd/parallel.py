"""Data parallelism for the ViT-CNN training step: one process per GPU, RCCL over xGMI.

The reference is single-process; patches are independent, so the
minibatch shards across ranks and the only exchange per step is the gradient all-reduce.

* The model's gradients are ONE flat fp32 tensor (`model.flat_params.grad`), so the exchange is a
  single `all_reduce(SUM)` of 1,660,090 floats (the 1,170 never-used parameters sit at the tail
  of the buffer and are excluded).  The 1/world average is folded into the fused AdamW kernel
  (`AdamW.grad_scale`) instead of a separate scaling pass.
* BatchNorm stays local (not SyncBN): each rank's B=64 forward equals the reference's B=64
  forward.  Running statistics are rank-local during training; `broadcast_buffers` copies
  rank 0's before evaluation / checkpointing (DDP `broadcast_buffers` semantics).
* Parameters are broadcast from rank 0 once at start so every replica starts identical.

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


def allreduce_gradients(model, optimizer=None, group=None):
    """Sum the flat gradient over ranks; the 1/world average goes into the optimizer's fused
    update when it supports it (vitcnn_amd.AdamW.grad_scale), else the gradient is scaled."""
    if not is_distributed():
        if optimizer is not None and hasattr(optimizer, "grad_scale"):
            optimizer.grad_scale = 1.0
        return
    n = dist.get_world_size(group)
    if not hasattr(model, "flat_params"):
        # per-parameter gradients (FusAtNet: torch.optim.Adam over .grad): one flattened bucket
        grads = [p.grad for p in model.parameters() if p.grad is not None]
        if not grads:
            raise RuntimeError("allreduce_gradients: backward has not produced a gradient")
        bucket = torch.cat([g.reshape(-1) for g in grads])
        dist.all_reduce(bucket, op=dist.ReduceOp.SUM, group=group)
        bucket.mul_(1.0 / n)
        o = 0
        for g in grads:
            g.copy_(bucket[o:o + g.numel()].view_as(g))
            o += g.numel()
        return
    g = active_grad(model)
    if g is None:
        raise RuntimeError("allreduce_gradients: backward has not produced a gradient")
    dist.all_reduce(g, op=dist.ReduceOp.SUM, group=group)
    if optimizer is not None and hasattr(optimizer, "grad_scale"):
        optimizer.grad_scale = 1.0 / n
    else:
        g.mul_(1.0 / n)


def broadcast_parameters(model, src: int = 0, group=None):
    """Make every replica start from rank `src`'s parameters (one broadcast of the flat buffer)."""
    if not is_distributed():
        return
    with torch.no_grad():
        dist.broadcast(model.flat_params.data, src=src, group=group)


def broadcast_buffers(model, src: int = 0, group=None):
    """BN running statistics and counters from rank `src` (before eval / checkpoint)."""
    if not is_distributed():
        return
    for b in model.flat_buffers():
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
