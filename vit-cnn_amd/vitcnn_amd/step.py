"""One fused training step on the caller's thread: forward, weighted CE, backward (+ optimizer), and
`TrainStepper`, the per-batch step of `model_utils.train` (replayed as one hipGraph per batch shape).

`loss = crit(model(hsi, lidar), target); loss.backward(); opt.step()` is the reference loop
(model_utils.py:918-934) and works unchanged with this package.  Its backward, however, runs on
the autograd engine's device thread, from which the step's side streams cannot be forked inside
a hipGraph capture on this ROCm release.  `fused_train_step` issues the SAME kernels (same
program, same numerics: tests/test_model_gpu.py checks both entry points agree bit-for-bit)
from the caller's thread, so a training loop or the benchmark can capture the whole
multi-stream step — forward, CE, backward and AdamW — into one hipGraph.
"""
from __future__ import annotations

import torch

from . import parallel
from .flat import expose_grad_views
from .losses import CrossEntropyLoss, ce_forward_backward
from .model import Multimodality_Mamba, _Program
from .optim import AdamW


def fused_train_step(model: Multimodality_Mamba, criterion: CrossEntropyLoss, hsi, lidar, target,
                     optimizer=None, grad_hook=None, exchange=None):
    """Returns the loss tensor (device scalar).  Gradients land in `model.flat_params.grad`
    (accumulated like autograd if a gradient is already present); `grad_hook(model)` runs between
    backward and the optimizer step.  `exchange` (parallel.GradExchange) all-reduces the gradient
    bucket by bucket on its own stream while the backward is still running, and the optimizer step
    is ordered after the last bucket."""
    if not model.training:
        raise RuntimeError("fused_train_step needs the model in train mode")
    if hsi.device.type != "cuda":
        raise RuntimeError("ViT-CNN MI355X path: inputs must be on a ROCm (cuda) device; no CPU fallback")
    model._ensure_flat()
    hsi = hsi.detach().to(torch.float32).contiguous()
    lidar = lidar.detach().to(torch.float32).contiguous()
    target = target.to(torch.int64).contiguous()
    prog = _Program(model, hsi.device, hsi.shape[0], True, "grad")
    logits = prog.forward(hsi, lidar)
    w = criterion.weight
    if w is not None and w.device != logits.device:
        w = w.to(logits.device)
    loss, dlog = ce_forward_backward(logits, target, w, criterion.ignore_index)
    flat = model.flat_params
    if exchange is not None:
        if flat.grad is not None:
            raise RuntimeError("fused_train_step(exchange=...): zero the gradients first (set_to_none)")
        grad = exchange.begin(model, hsi.device)
        prog.backward(dlog, bucket_hook=exchange.bucket_ready, out=grad)
        exchange.finish(optimizer)
        flat.grad = grad
    else:
        grad = prog.backward(dlog)
        if flat.grad is None:
            flat.grad = grad
        else:
            flat.grad.add_(grad)
    expose_grad_views(model)
    if grad_hook is not None:
        grad_hook(model)
    if optimizer is not None:
        optimizer.step()
    return loss


class _Captured:
    """One batch shape's captured step: static inputs, the graph, and its loss / gradient outputs."""

    def __init__(self, hsi, lidar, target):
        self.hsi, self.lidar, self.target = hsi, lidar, target
        self.graph = torch.cuda.CUDAGraph()
        self.loss = None
        self.grad = None


class TrainStepper:
    """The optimizer step `model_utils.train` runs per batch (model_utils.py:918-934: zero_grad,
    forward, criterion, backward, step), as fast as the model allows:

    * ViT-CNN with the fused AdamW: the whole step — forward, CE, backward, (data parallel: the three
      head-first gradient buckets all-reduced by RCCL on a side stream while the backward runs,
      parallel.GradExchange), AdamW — is `fused_train_step`, captured once per batch shape into a
      hipGraph and replayed for every later batch of that shape.  The first batch of a shape runs the
      same step eagerly (it is a real update, and it builds the persistent workspaces the capture
      records); the second is captured and replayed; capture does not run the step, so every batch is
      exactly one update.  A short last batch is simply another shape.  The optimizer's
      hyper-parameters live in device memory and are synced before each replay (`AdamW.sync_hyper`),
      so StepLR's lr changes take effect as with torch.optim.
    * anything else (torch modules / optimizers, S2EFT's one-input forward, FusAtNet): the reference's
      eager sequence, with `parallel.allreduce_gradients` between backward and step under DP.

    `launch` says which path ran ("hipGraph", "eager", or the capture failure), never silently."""

    def __init__(self, net, optimizer, criterion, use_graph: bool = True):
        self.net, self.opt, self.crit = net, optimizer, criterion
        self.fused = (isinstance(net, Multimodality_Mamba) and isinstance(optimizer, AdamW)
                      and isinstance(criterion, CrossEntropyLoss))
        self.use_graph = use_graph and self.fused
        self.graphs = {}
        self.seen = set()
        self.binding = None
        self.launch = "hipGraph" if self.use_graph else "eager"
        self.exchange = None
        if self.fused and parallel.is_distributed():
            self.exchange = parallel.GradExchange(net)
            optimizer.grad_scale = 1.0 / parallel.world()
            if self.use_graph and not parallel.capturable():
                # gloo's host-side collectives cannot be captured: the same fused step, eagerly
                self.use_graph = False
                self.launch = "eager (the gloo exchange is not graph-capturable)"

    def _check_binding(self):
        """captured graphs hold the parameter / buffer / optimizer-state addresses of their capture:
        drop them if the model was re-flattened (load_state_dict with assign, .to(), ...)"""
        m = self.net
        key = (m._bind_gen, m._flat_store.data_ptr(), m._bflat.data_ptr(), m._iflat.data_ptr(),
               id(self.opt._dev["m"]) if self.opt._dev is not None else None)
        if key != self.binding:
            self.graphs, self.seen = {}, set()
            self.binding = key

    def _eager_fused(self, data, data2, target):
        self.opt.zero_grad(set_to_none=True)
        return fused_train_step(self.net, self.crit, data, data2, target, optimizer=self.opt, exchange=self.exchange)

    def _capture(self, key, data, data2, target):
        dev = data.device
        c = _Captured(torch.empty_like(data, memory_format=torch.contiguous_format),
                      torch.empty_like(data2, memory_format=torch.contiguous_format),
                      torch.empty(target.shape, dtype=torch.int64, device=dev))
        torch.cuda.synchronize(dev)
        self.opt.sync_hyper()          # nothing may change inside the capture (AdamW.step's copy)
        self.opt.zero_grad(set_to_none=True)
        try:
            with torch.cuda.graph(c.graph):
                c.loss = fused_train_step(self.net, self.crit, c.hsi, c.lidar, c.target, optimizer=self.opt,
                                          exchange=self.exchange)
        except RuntimeError as e:    # reported through `launch`, and this shape stays eager
            torch.cuda.synchronize(dev)
            self.opt.zero_grad(set_to_none=True)
            self.launch = f"eager (graph capture failed: {str(e)[:100]})"
            self.use_graph = False
            return None
        c.grad = self.net.flat_params.grad
        self.graphs[key] = c
        return c

    def step(self, data, data2, target):
        """one optimizer step on this batch; returns the loss as a device scalar"""
        net = self.net
        if not self.fused:
            self.opt.zero_grad()
            out = net(data, data2)
            loss = self.crit(out, target)
            loss.backward()
            parallel.allreduce_gradients(net, self.opt)
            self.opt.step()
            return loss
        dev = net.flat_params.device
        data = data.to(dev, non_blocking=True)
        data2 = data2.to(dev, non_blocking=True)
        target = target.to(dev, non_blocking=True)
        net._ensure_flat()
        self.opt._device_state(net.flat_params)   # the optimizer state exists before the binding is taken
        self._check_binding()
        key = (tuple(data.shape), tuple(data2.shape), tuple(target.shape))
        c = self.graphs.get(key)
        if c is None and self.use_graph and key in self.seen:
            c = self._capture(key, data, data2, target)
        self.seen.add(key)
        if c is None:
            return self._eager_fused(data, data2, target)
        c.hsi.copy_(data)
        c.lidar.copy_(data2)
        c.target.copy_(target)
        self.opt.sync_hyper()
        c.graph.replay()
        net.flat_params.grad = c.grad
        return c.loss
