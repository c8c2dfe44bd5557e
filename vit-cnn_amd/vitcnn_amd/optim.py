"""Fused AdamW over the model's flat parameter buffer (torch.optim.AdamW semantics, model_utils.py:309-310).

One kernel updates every active parameter (the reference's per-tensor loop over ~1000 tensors
becomes a single HBM-bound pass).  Hyper-parameters and the step counter live in device memory,
so a step can be replayed inside a hipGraph and a scheduler (StepLR) that edits
`param_groups[0]['lr']` takes effect on the next step.
"""
from __future__ import annotations

import torch

from ._lib import lib


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, amsgrad=False):
        if amsgrad:
            raise ValueError("amsgrad is not used by the reference and is not implemented")
        params = list(params)
        owners = {id(getattr(p, "_vc_owner", None)) for p in params if isinstance(p, torch.Tensor)}
        owner = getattr(params[0], "_vc_owner", None) if params else None
        if owner is None or len(owners) != 1:
            raise ValueError("vitcnn_amd.optim.AdamW expects the parameters of one vitcnn_amd model")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        if sum(p.numel() for g in self.param_groups for p in g["params"]) != getattr(owner(), "_n_elems",
                                                                                      owner()._n_params):
            raise ValueError("vitcnn_amd.optim.AdamW must be given all parameters of the model")
        self._owner = owner
        self.grad_scale = 1.0   # data-parallel: 1/world_size folded into the update
        self._dev = None
        self._hyper_vals = None

    def sync_hyper(self):
        """Copy lr / betas / eps / weight decay / grad_scale to the device tensor the kernel reads, if
        they changed.  step() does this itself; a replayed hipGraph of the step does not run Python, so
        the caller (vitcnn_amd.step.TrainStepper) calls it before every replay (a scheduler's new lr then
        takes effect on the next step, as with torch.optim)."""
        flat = self._owner().flat_params
        st = self._device_state(flat)
        grp = self.param_groups[0]
        vals = (float(grp["lr"]), float(grp["betas"][0]), float(grp["betas"][1]), float(grp["eps"]),
                float(grp["weight_decay"]), float(self.grad_scale))
        if vals != self._hyper_vals:
            st["hyper"].copy_(torch.tensor(vals, dtype=torch.float32))
            self._hyper_vals = vals
        return st

    def _device_state(self, flat):
        st = self._dev
        if st is None or st["m"].device != flat.device:
            n = self._owner()._n_active
            st = dict(m=torch.zeros(n, device=flat.device), v=torch.zeros(n, device=flat.device),
                      step=torch.zeros(3, device=flat.device), hyper=torch.zeros(6, device=flat.device))
            self._dev = st
            self._hyper_vals = None
        return st

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        model = self._owner()
        flat = model.flat_params
        g = flat.grad
        if g is None:
            return loss
        st = self.sync_hyper()
        # this optimizer reads the flat gradient: the model need not rebuild ~1000 per-parameter .grad views
        # after every backward while it is the one stepping (a torch optimizer stepping the same model turns
        # them back on: _torch_step_pre_hook)
        model._grad_views = False
        s = torch.cuda.current_stream(flat.device).cuda_stream
        lib().vc_adamw(model._n_active, flat.data_ptr(), g.data_ptr(), st["m"].data_ptr(), st["v"].data_ptr(),
                       st["hyper"].data_ptr(), st["step"].data_ptr(), s)
        return loss

    def zero_grad(self, set_to_none: bool = True):
        super().zero_grad(set_to_none=set_to_none)
        self._owner().zero_grad(set_to_none=set_to_none)


def _torch_step_pre_hook(opt, args, kwargs):
    """Global step pre-hook of every torch optimizer: a torch optimizer (e.g. the reference pattern
    torch.optim.Adam(model.parameters())) stepping a flat-buffer vitcnn_amd model needs the per-parameter
    .grad views; if the fused AdamW stepped that model before (and switched them off), they are turned
    back on and built now, before this step reads them."""
    if isinstance(opt, AdamW):
        return
    owners = getattr(opt, "_vc_owners", None)
    if owners is None or owners[0] != len(opt.param_groups):
        found = {}
        for grp in opt.param_groups:
            for p in grp["params"]:
                o = getattr(p, "_vc_owner", None)
                if o is not None:
                    found[id(o)] = o
        owners = (len(opt.param_groups), list(found.values()))
        opt._vc_owners = owners
    for o in owners[1]:
        m = o()
        if m is not None and not getattr(m, "_grad_views", True):
            from .flat import expose_grad_views
            m._grad_views = True
            expose_grad_views(m)


from torch.optim.optimizer import register_optimizer_step_pre_hook  # noqa: E402

register_optimizer_step_pre_hook(_torch_step_pre_hook)
