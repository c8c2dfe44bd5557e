"""One flat fp32 parameter buffer behind an nn.Module's parameter tree (S2EFT, FusAtNet).

Every registered nn.Parameter is re-pointed at a view of one contiguous fp32 buffer (`flat_params`),
in `named_parameters()` order, so state_dict() / load_state_dict() / parameters() keep the reference's
names and shapes while the hand-written backward writes ONE flat gradient (`flat_params.grad`): the
fused optimizer (vitcnn_amd.optim.AdamW, one HBM pass) and the data-parallel exchange
(parallel.allreduce_gradients, one collective) then each touch a single tensor instead of a
per-parameter list.  Buffers (BatchNorm running statistics) stay ordinary registered buffers.
"""
from __future__ import annotations

import weakref

import torch
import torch.nn as nn

F32 = 4
PARAM_ALIGN = 4   # floats (16 B)
ALIGN_MIN = 64


def _last_active_name(model, names):
    """the last parameter (in flat order) that receives gradients: the views fast path checks it, not
    names[-1] (ViT-CNN's tail holds the never-used parameters, whose .grad stays None by design)"""
    last = getattr(model, "_vc_last_active", None)   # the flat layout is fixed at construction
    if last is None:
        last = max((n for n in names if model._poff[n] < model._n_active), key=lambda n: model._poff[n])
        object.__setattr__(model, "_vc_last_active", last)
    return last


def expose_grad_views(model):
    """Point every parameter's .grad at its slice of the flat gradient (`flat_params.grad`), so torch
    optimizers (e.g. the reference's torch.optim.Adam(model.parameters()), model_utils.py:109-118),
    gradient clipping or inspection see the gradient the hand-written backward wrote.  A no-op when
    the views are current, or while the model is being stepped by vitcnn_amd.optim.AdamW (which reads
    the flat gradient and clears `_grad_views` when it steps: ~1000 views per ViT-CNN step would cost
    milliseconds); a torch optimizer stepping the model turns them back on (optim._torch_step_pre_hook)."""
    if not getattr(model, "_grad_views", True):
        return
    g = model._flat_store.grad
    if g is None:
        return
    base = g.data_ptr()
    names = model._pnames if hasattr(model, "_pnames") else list(model._pmods)
    lastn = _last_active_name(model, names)
    first, last = model._pmods[names[0]], model._pmods[lastn]
    p0, p1 = first[0]._parameters[first[1]], last[0]._parameters[last[1]]
    if p0.grad is not None and p1.grad is not None and p0.grad.data_ptr() == base + F32 * model._poff[names[0]] \
            and p1.grad.data_ptr() == base + F32 * model._poff[lastn]:
        return
    n_active = model._n_active
    for n in names:
        m, pn = model._pmods[n]
        p = m._parameters[pn]
        o = model._poff[n]
        # parameters the forward never uses (ViT-CNN's hsiMamba.tokenlearner / ln3) get no gradient,
        # as under the reference's autograd
        p.grad = g[o:o + p.numel()].view(p.shape) if o < n_active else None


def install_grad_views(model):
    """Register expose_grad_views as the flat buffer's post-accumulate hook (autograd backward), and a
    pre-accumulate hook that honours a torch optimizer's zero_grad(): that clears the per-parameter
    views (grad = None) but cannot see the flat gradient, which autograd would otherwise keep
    accumulating into -- so a flat gradient whose views were cleared is dropped before the new one
    lands (zero_grad(set_to_none=False) zeroes the views, i.e. the flat gradient, in place)."""
    me = weakref.ref(model)

    def pre(_g):
        m = me()
        if m is not None and getattr(m, "_grad_views", True) and m._flat_store.grad is not None:
            names = m._pnames if hasattr(m, "_pnames") else list(m._pmods)
            mod, pn = m._pmods[names[0]]
            if mod._parameters[pn].grad is None:
                m._flat_store.grad = None
        return None

    def hook(_t):
        m = me()
        if m is not None:
            expose_grad_views(m)

    model._flat_store.register_hook(pre)
    model._flat_store.register_post_accumulate_grad_hook(hook)


class FlatParams:
    """Mixin for an nn.Module whose parameters live in one flat buffer; call `_build_flat()` at the end
    of __init__.  Provides flat_params, n_active_params, _ensure_flat (re-pack after a parameter was
    replaced, e.g. by load_state_dict with assign), device moves and zero_grad on the flat buffer."""

    def _build_flat(self):
        named = list(nn.Module.named_parameters(self))
        self._poff, off = {}, 0
        for n, p in named:
            # every parameter of >= ALIGN_MIN elements starts 16-B aligned, as in ViT-CNN's layout (model.py): the
            # weights then qualify for the pipelined GEMM's 16-B LDS-DMA staging (gemm.hip pipe_fits); the gaps
            # hold zeros in the parameters and in every gradient (the backward zero-fills the flat gradient)
            if p.numel() >= ALIGN_MIN:
                off = -(-off // PARAM_ALIGN) * PARAM_ALIGN
            self._poff[n] = off
            off += p.numel()
        off = -(-off // PARAM_ALIGN) * PARAM_ALIGN
        self._n_params = self._n_active = off
        self._n_elems = sum(p.numel() for _, p in named)   # the parameters proper (without the alignment gaps)
        flat = torch.zeros(off, dtype=torch.float32, device=named[0][1].device)
        for n, p in named:
            flat[self._poff[n]:self._poff[n] + p.numel()].copy_(p.detach().reshape(-1))
        self._pmods = {}
        for mn, m in nn.Module.named_modules(self):
            for pn, p in m._parameters.items():
                if p is None:
                    continue
                self._pmods[(mn + "." if mn else "") + pn] = (m, pn)
        self._rebind(flat)
        me = weakref.ref(self)
        for _, p in named:
            p._vc_owner = me

    def _rebind(self, flat):
        object.__setattr__(self, "_flat_store", flat.detach().requires_grad_(True))
        install_grad_views(self)
        base = self._flat_store.detach()
        for n, (m, pn) in self._pmods.items():
            p = m._parameters[pn]
            o = self._poff[n]
            p.data = base[o:o + p.numel()].view(p.shape)

    def _repack(self, device):
        flat = torch.zeros(self._n_params, dtype=torch.float32, device=device)
        for n, (m, pn) in self._pmods.items():
            o = self._poff[n]
            flat[o:o + m._parameters[pn].numel()].copy_(m._parameters[pn].detach().reshape(-1))
        self._rebind(flat)

    def _apply(self, fn, recurse=True):
        # parameters and buffers through nn.Module (buffers: BN running statistics), then the
        # parameters re-packed into one flat buffer on their new device
        nn.Module._apply(self, fn, recurse)
        first = next(iter(self._pmods.values()))
        p0 = first[0]._parameters[first[1]]
        if p0.dtype != torch.float32:
            raise RuntimeError(f"{type(self).__name__} MI355X path computes in fp32; dtype casts are not supported")
        self._repack(p0.device)
        return self

    def _ensure_flat(self):
        base = self._flat_store.data_ptr()
        for n, (m, pn) in self._pmods.items():
            if m._parameters[pn].data_ptr() != base + F32 * self._poff[n]:
                self._repack(self._flat_store.device)
                return

    @property
    def flat_params(self) -> torch.Tensor:
        return self._flat_store

    @property
    def n_active_params(self) -> int:
        return self._n_active

    def zero_grad(self, set_to_none: bool = True):
        nn.Module.zero_grad(self, set_to_none=set_to_none)
        if set_to_none:
            self._flat_store.grad = None
        elif self._flat_store.grad is not None:
            self._flat_store.grad.zero_()
