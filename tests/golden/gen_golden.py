"""Generate golden vectors from the REFERENCE ViT-CNN model (run in the build container only).

This script imports `/root/reference/model/Multimodality_Mamba/Mutimodality_Mamba7.py`
(the reference's "ViT-CNN (ours)" model, registered as "Multimodality_Mamba",
model_utils.py:297-313) with small stand-ins for third-party packages that are not
installed here (mmengine, mmcv, thop, visdom, spectral, seaborn) and for the absent
`model/changer.py` (ChannelExchange, semantics inferred from open-cd Changer, p=1/2;
SURVEY.md section 8 row A10: parity for that op is pinned only to this inference).
The recipe is the one SURVEY.md section 8c verified.  The only patch to reference
behaviour is TokenLearner.forward allocating on the input's device instead of the
hard-coded "cuda:0" (Mutimodality_Mamba7.py:60).

Outputs only numbers (no reference source) into tests/golden/*.npz / *.json:
  state_dict_keys.json      names, shapes and dtypes of the 1704 state_dict entries
  vitcnn_b4.npz             B=4 train step: inputs are regenerated from hashinit; stores
                            logits, loss, per-parameter grad L2 norms, full grads of
                            small tensors, per-module activations, post-AdamW parameter
                            norms, BN running stats, eval-mode logits after the step
  vitcnn_b64.npz            B=64 (bench shape): train-mode logits, loss, grad norms
  mamba_mixer.npz           transformers MambaMixer (the reference's token mixer) alone

Run:  python tests/golden/gen_golden.py      (needs /root/reference; CPU only)
"""
from __future__ import annotations

import importlib.util
import json
import math
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))
from vitcnn_amd.hashinit import fill_module_, param_fill, synthetic_batch  # noqa: E402

N_CLASSES = 16  # Houston2013 incl. "Unclassified" (datasets.py:135-152)


def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


def load_reference():
    sys.path.insert(0, REF)
    from transformers.models.mamba.configuration_mamba import MambaConfig

    class BaseModule(nn.Module):
        def __init__(self, init_cfg=None):
            super().__init__()
            self.init_cfg = init_cfg

    class AttrCfg(dict):
        """mmengine.Config stand-in: attribute access; missing keys fall back to MambaConfig."""
        _fallback = None

        def __getattr__(self, k):
            if k in self:
                return self[k]
            if AttrCfg._fallback is None:
                AttrCfg._fallback = MambaConfig()
            return getattr(AttrCfg._fallback, k)

    class Registry:
        def __init__(self, *a, **k):
            self._m = {"LN": nn.LayerNorm}
            self.scope = "stub"

        def get(self, k):
            return self._m.get(k)

        def register_module(self, *a, **k):
            return lambda c: c

    _stub("mmengine", Config=AttrCfg)
    _stub("mmengine.model", ModuleList=nn.ModuleList, BaseModule=BaseModule)
    _stub("mmengine.model.weight_init", trunc_normal_=nn.init.trunc_normal_)
    _stub("mmengine.utils", digit_version=lambda v: tuple(int(x) for x in v.split("+")[0].split(".")[:3]))
    reg = _stub("mmengine.registry", Registry=Registry)
    for n in ["DATA_SAMPLERS", "DATASETS", "EVALUATOR", "HOOKS", "LOG_PROCESSORS", "LOOPS", "METRICS",
              "MODEL_WRAPPERS", "MODELS", "OPTIM_WRAPPER_CONSTRUCTORS", "OPTIM_WRAPPERS", "OPTIMIZERS",
              "PARAM_SCHEDULERS", "RUNNER_CONSTRUCTORS", "RUNNERS", "TASK_UTILS", "TRANSFORMS",
              "VISBACKENDS", "VISUALIZERS", "WEIGHT_INITIALIZERS"]:
        setattr(reg, n, None)

    class PatchEmbed(nn.Module):  # mmcv PatchEmbed with conv projection, no norm
        def __init__(self, in_channels, input_size, embed_dims, conv_type, kernel_size, stride, padding, bias, **kw):
            super().__init__()
            self.projection = nn.Conv2d(in_channels, embed_dims, kernel_size, stride, padding, bias=bias)
            h = (input_size + 2 * padding - (kernel_size - 1) - 1) // stride + 1
            self.init_out_size = (h, h)

        def forward(self, x):
            x = self.projection(x)
            return x.flatten(2).transpose(1, 2), (x.shape[2], x.shape[3])

    _stub("mmcv")
    _stub("mmcv.cnn")
    _stub("mmcv.cnn.bricks")
    _stub("mmcv.cnn.bricks.transformer", PatchEmbed=PatchEmbed)
    _stub("thop", profile=None, clever_format=None)

    class ChannelExchange(nn.Module):  # open-cd Changer semantics (inferred)
        def __init__(self, p=1 / 2):
            super().__init__()
            self.p = int(1 / p)

        def forward(self, x1, x2):
            n, c = x1.shape[:2]
            m = (torch.arange(c, device=x1.device) % self.p == 0).unsqueeze(0).expand((n, -1))
            o1, o2 = torch.zeros_like(x1), torch.zeros_like(x2)
            o1[~m, ...] = x1[~m, ...]
            o2[~m, ...] = x2[~m, ...]
            o1[m, ...] = x2[m, ...]
            o2[m, ...] = x1[m, ...]
            return o1, o2

    _stub("model.changer", ChannelExchange=ChannelExchange, SpatialExchange=None, ChannelInsert=None)
    for n in ["visdom", "spectral", "seaborn"]:
        _stub(n)
    spec = importlib.util.spec_from_file_location(
        "ref_vitcnn", REF + "/model/Multimodality_Mamba/Mutimodality_Mamba7.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)

    def tl_forward(self, x):  # only deviation: allocate on x.device (ref :60 pins cuda:0)
        b, c = x.shape[:2]
        z = torch.empty(b, self.S, c, device=x.device, dtype=x.dtype)
        for i in range(self.S):
            a, _ = self.tokenizers[i](x)
            z[:, i, :] = a
        return z

    mod.TokenLearner.forward = tl_forward
    return mod


def build_net(mod, c1=144, c2=1, ncls=N_CLASSES):
    net = mod.Multimodality_Mamba(img_size=9, patch_size=1, stride=1, in_channels1=c1, in_channels2=c2,
                                  dim_embedding=32, num_class=ncls, path_type="multi_clock_gate")
    fill_module_(net)
    return net


def ce_weights(ncls):
    w = torch.ones(ncls)
    w[0] = 0.0  # ignored_labels=[0] (model_utils.py:63-66)
    return w


ACT_MODULES = [
    "hsi1.global_view", "hsi1", "hsi2.global_view", "hsi2", "lidar1", "lidar2", "fusion1", "fusion2",
    "hsi1.local_feature", "hsi1.global_feature", "hsi1.channel_token", "hsi1.FusionLayer.cross_attention",
    "hsi2.FusionLayer", "hsi2.channel_token",
]


def train_step_fixture(mod, batch, tag, full_grad_max=2048, acts=True, opt_step=True):
    torch.manual_seed(0)
    net = build_net(mod)
    net.train()
    hsi, lidar, target = synthetic_batch(tag, batch, 144, 1, 9, N_CLASSES)
    hsi_t, lidar_t, tgt_t = torch.from_numpy(hsi), torch.from_numpy(lidar), torch.from_numpy(target)
    out = {}
    captured = {}
    hooks = []
    if acts:
        mods = dict(net.named_modules())
        for name in ACT_MODULES:
            def hk(m, i, o, name=name):
                o = o[0] if isinstance(o, (list, tuple)) else o
                captured[name] = o.detach().clone()
            hooks.append(mods[name].register_forward_hook(hk))
    crit = nn.CrossEntropyLoss(weight=ce_weights(N_CLASSES))
    opt = torch.optim.AdamW(net.parameters(), lr=8e-4)
    opt.zero_grad()
    logits = net(hsi_t, lidar_t)
    loss = crit(logits, tgt_t)
    loss.backward()
    for h in hooks:
        h.remove()
    out["logits"] = logits.detach().numpy()
    out["loss"] = np.array(loss.item(), dtype=np.float64)
    out["target"] = target
    names, gnorm = [], []
    for n, p in net.named_parameters():
        names.append(n)
        if p.grad is None:
            gnorm.append(-1.0)
            continue
        gnorm.append(float(p.grad.double().norm()))
        if p.numel() <= full_grad_max:
            out["grad/" + n] = p.grad.numpy().copy()
    out["grad_norm_names"] = np.array(names)
    out["grad_norm"] = np.array(gnorm, dtype=np.float64)
    for k, v in captured.items():
        out["act/" + k] = v.numpy()
    if opt_step:
        # eval-mode logits with the running stats this train forward produced, before the optimizer
        # step (parameters whose true gradient is 0 get a noise-signed Adam step that eval-mode BN
        # no longer cancels, so logits after the step are only loosely comparable)
        net.eval()
        with torch.no_grad():
            out["eval_logits_before_step"] = net(hsi_t, lidar_t).numpy()
        net.train()
        opt.step()
        pn = [float(p.detach().double().norm()) for _, p in net.named_parameters()]
        out["param_norm_after_step"] = np.array(pn, dtype=np.float64)
        for n, b in net.named_buffers():
            if ("running_mean" in n or "running_var" in n) and b.numel() <= 512:
                out["buf/" + n] = b.numpy().copy()
        for n, p in net.named_parameters():
            if p.numel() <= 256:
                out["param_after/" + n] = p.detach().numpy().copy()
        net.eval()
        with torch.no_grad():
            out["eval_logits_after_step"] = net(hsi_t, lidar_t).numpy()
    return out


TRAIN_STEPS_EVAL = 8
VAL_PASSES = 40


def trained_eval_fixture(mod, steps=TRAIN_STEPS_EVAL):
    """Eval-mode class indices that vary across samples: the reference module (hash init) takes `steps`
    AdamW(lr 8e-4) training steps on the golden B=64 batch (model_utils.py:918-934) and VAL_PASSES
    train-mode no-grad forwards of it (the reference's val()), then predicts the trained batch and a
    second synthetic batch in eval mode (running-statistic BatchNorm, model_utils.py:1067-1132 test()).
    The untrained network's eval argmax is degenerate (one class for every sample); after training it
    is not.  Saved: the loss trajectory, eval logits and argmax."""
    torch.manual_seed(0)
    net = build_net(mod)
    net.train()
    hsi, lidar, target = synthetic_batch("golden.b64", 64, 144, 1, 9, N_CLASSES)
    hsi_t, lidar_t, tgt_t = torch.from_numpy(hsi), torch.from_numpy(lidar), torch.from_numpy(target)
    crit = nn.CrossEntropyLoss(weight=ce_weights(N_CLASSES))
    opt = torch.optim.AdamW(net.parameters(), lr=8e-4)
    losses = []
    for _ in range(steps):
        opt.zero_grad()
        loss = crit(net(hsi_t, lidar_t), tgt_t)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    # val-style train-mode forwards (model_utils.py:1135-1158 runs val() without net.eval(), so every
    # val batch updates the BatchNorm running statistics): they settle at the trained batch's statistics
    with torch.no_grad():
        for _ in range(VAL_PASSES):
            net(hsi_t, lidar_t)
    ehsi, elidar, _ = synthetic_batch("golden.eval64", 64, 144, 1, 9, N_CLASSES)
    net.eval()
    with torch.no_grad():
        logits = net(hsi_t, lidar_t).numpy()                                   # the trained batch
        logits2 = net(torch.from_numpy(ehsi), torch.from_numpy(elidar)).numpy()  # a fresh batch
    return {"losses": np.array(losses, dtype=np.float64), "eval_logits": logits, "eval_argmax": logits.argmax(1),
            "eval2_logits": logits2, "eval2_argmax": logits2.argmax(1), "target": target, "steps": np.array(steps),
            "val_passes": np.array(VAL_PASSES)}


def mixer_fixture(mod):
    from transformers.models.mamba.modeling_mamba import MambaMixer
    cfgs = {"e144": (144, 72, 81), "e256": (256, 128, 49)}
    out = {}
    for tag, (e, d, L) in cfgs.items():
        cfg = sys.modules["mmengine"].Config(dict(hidden_size=e, state_size=16, intermediate_size=d, conv_kernel=4,
                                                  time_step_rank=math.ceil(e / 16), use_conv_bias=True,
                                                  hidden_act="silu", use_bias=False))
        mixer = MambaMixer(cfg, 0)
        with torch.no_grad():
            for n, p in mixer.named_parameters():
                p.copy_(torch.from_numpy(param_fill("mixer." + n, p.shape)))
        mixer.train()
        from vitcnn_amd.hashinit import hash_u01
        x = torch.from_numpy((2 * hash_u01(f"mixer.{tag}.x", 3 * L * e) - 1).astype(np.float32).reshape(3, L, e))
        x.requires_grad_(True)
        y = mixer(x)
        gy = torch.from_numpy((2 * hash_u01(f"mixer.{tag}.gy", 3 * L * e) - 1).astype(np.float32).reshape(3, L, e))
        (y * gy).sum().backward()
        out[f"{tag}/y"] = y.detach().numpy()
        out[f"{tag}/gx"] = x.grad.numpy()
        for n, p in mixer.named_parameters():
            if p.numel() <= 10000:
                out[f"{tag}/grad/{n}"] = p.grad.numpy()
            else:
                out[f"{tag}/gradnorm/{n}"] = np.array(float(p.grad.double().norm()))
    return out


def capture_scan_orders(mod, net):
    """Record the literal direction tables (Mutimodality_Mamba7.py:609-640, :788-806) as data.

    They are local int64 literals inside hsiMamba.forward, so torch.tensor is wrapped during
    one no-grad forward and every 81- or 49-entry integer list it receives is recorded in
    creation order (vf, 37df, 19df, ltcw, ltacw per block).
    """
    seen = []
    real = torch.tensor

    def spy(data, *a, **k):
        if isinstance(data, list) and len(data) in (81, 49) and all(isinstance(v, int) for v in data):
            seen.append(list(data))
        return real(data, *a, **k)

    hsi, lidar, _ = synthetic_batch("orders", 2, 144, 1, 9, N_CLASSES)
    torch.tensor = spy
    try:
        with torch.no_grad():
            net(torch.from_numpy(hsi), torch.from_numpy(lidar))
    finally:
        torch.tensor = real
    names = ["vf", "37df", "19df", "ltcw", "ltacw"]
    out = {}
    for tab in seen:
        n = len(tab)
        key = f"n{int(round(n ** 0.5))}"
        out.setdefault(key, {})
        nm = names[len(out[key])]
        out[key][nm] = tab
    return out


def main():
    torch.set_num_threads(os.cpu_count())
    mod = load_reference()
    if "--eval-only" in sys.argv:   # only the trained eval-mode fixture (the others unchanged)
        z = trained_eval_fixture(mod)
        np.savez_compressed(os.path.join(HERE, "vitcnn_eval64.npz"), **z)
        am, am2 = z["eval_argmax"], z["eval2_argmax"]
        print("eval64 fixture done: losses", np.round(z["losses"], 4), "distinct classes", len(set(am.tolist())),
              "(fresh batch:", len(set(am2.tolist())), ") argmax == target", float((am == z["target"]).mean()))
        return
    net = build_net(mod)
    with open(os.path.join(HERE, "scan_orders.json"), "w") as f:
        json.dump(capture_scan_orders(mod, net), f)
    keys = [{"name": k, "shape": list(v.shape), "dtype": str(v.dtype).replace("torch.", "")}
            for k, v in net.state_dict().items()]
    with open(os.path.join(HERE, "state_dict_keys.json"), "w") as f:
        json.dump(keys, f, indent=0)
    print("state_dict entries:", len(keys), "params:", sum(p.numel() for p in net.parameters()))
    np.savez_compressed(os.path.join(HERE, "mamba_mixer.npz"), **mixer_fixture(mod))
    print("mixer fixture done")
    np.savez_compressed(os.path.join(HERE, "vitcnn_b4.npz"), **train_step_fixture(mod, 4, "golden.b4"))
    print("b4 fixture done")
    b64 = train_step_fixture(mod, 64, "golden.b64", full_grad_max=0, acts=False, opt_step=False)
    np.savez_compressed(os.path.join(HERE, "vitcnn_b64.npz"), **b64)
    print("b64 fixture done")


if __name__ == "__main__":
    main()
