"""One fused training step on the caller's thread: forward, weighted CE, backward (+ optimizer).

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

from .losses import CrossEntropyLoss, ce_forward_backward
from .model import Multimodality_Mamba, _Program


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
    if grad_hook is not None:
        grad_hook(model)
    if optimizer is not None:
        optimizer.step()
    return loss
