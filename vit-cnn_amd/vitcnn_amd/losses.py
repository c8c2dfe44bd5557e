"""Weighted cross-entropy on the MI355X (nn.CrossEntropyLoss(weight) of model_utils.py:311)."""
from __future__ import annotations

import torch
import torch.nn as nn

from ._lib import lib


class _CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, weight, ignore_index):
        B, ncls = logits.shape
        loss = torch.empty((), dtype=torch.float32, device=logits.device)
        s = torch.cuda.current_stream(logits.device).cuda_stream
        lib().vc_ce_fwd(B, ncls, logits.data_ptr(), target.data_ptr(), weight.data_ptr() if weight is not None else None,
                        ignore_index, loss.data_ptr(), s)
        ctx.save_for_backward(logits, target, weight if weight is not None else torch.empty(0))
        ctx.has_w = weight is not None
        ctx.ignore_index = ignore_index
        return loss

    @staticmethod
    def backward(ctx, gout):
        logits, target, weight = ctx.saved_tensors
        B, ncls = logits.shape
        gout = gout.detach().to(torch.float32).contiguous()
        dlog = torch.empty_like(logits)
        s = torch.cuda.current_stream(logits.device).cuda_stream
        lib().vc_ce_bwd(B, ncls, logits.data_ptr(), target.data_ptr(), weight.data_ptr() if ctx.has_w else None,
                        ctx.ignore_index, gout.data_ptr(), dlog.data_ptr(), s)
        return dlog, None, None, None


def ce_forward_backward(logits, target, weight, ignore_index=-100):
    """(loss, dlogits) of the weighted mean CE with d(loss) = 1, as one kernel on the current
    stream (the loss half of `fused_train_step`; vc_ce_fwd_bwd = vc_ce_fwd + vc_ce_bwd bit for bit)."""
    B, ncls = logits.shape
    s = torch.cuda.current_stream(logits.device).cuda_stream
    loss = torch.empty((), dtype=torch.float32, device=logits.device)
    dlog = torch.empty_like(logits)
    w = weight.data_ptr() if weight is not None else None
    lib().vc_ce_fwd_bwd(B, ncls, logits.data_ptr(), target.data_ptr(), w, ignore_index, loss.data_ptr(),
                        dlog.data_ptr(), s)
    return loss, dlog


class CrossEntropyLoss(nn.Module):
    """Drop-in for nn.CrossEntropyLoss(weight=...) with reduction='mean' (the reference's criterion)."""

    def __init__(self, weight=None, ignore_index: int = -100, reduction: str = "mean"):
        super().__init__()
        if reduction != "mean":
            raise ValueError("only reduction='mean' (the reference's setting) is implemented")
        self.register_buffer("weight", None if weight is None else weight.detach().to(torch.float32).clone())
        self.ignore_index = int(ignore_index)

    def forward(self, logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        if logits.device.type != "cuda":
            raise RuntimeError("ViT-CNN MI355X path: loss inputs must be on a ROCm (cuda) device")
        if logits.dim() != 2 or target.dim() != 1 or target.shape[0] != logits.shape[0]:
            raise RuntimeError(f"expected logits [B, C] and target [B], got {list(logits.shape)} / {list(target.shape)}")
        w = self.weight
        if w is not None:
            if w.numel() != logits.shape[1]:
                raise RuntimeError("weight tensor should be defined either for all classes or no classes")
            if w.device != logits.device:
                w = w.to(logits.device)
        return _CrossEntropyFn.apply(logits.to(torch.float32).contiguous(), target.to(torch.int64).contiguous(), w,
                                     self.ignore_index)
