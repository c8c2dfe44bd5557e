"""GPU diagnostic: per-tensor gradient error of the HIP b4 training step vs the float64 oracle
evaluated with the HIP path's ReLU decisions (tests/test_model_gpu.py criteria), worst first."""
import os, sys
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/vit-cnn_amd"); sys.path.insert(0, "/root/repo/tests")
import torch
from helpers import golden_batch, hash_state_dict, masked_oracle_step, relu_masks_from_workspace
from oracle import vitcnn_oracle as O
import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
from vitcnn_amd import Multimodality_Mamba, CrossEntropyLoss
sd = hash_state_dict()
hsi, lidar, target = golden_batch("golden.b4", 4)
w = O.ce_class_weights(16)
m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16); m.load_state_dict(sd); m = m.cuda().train()
crit = CrossEntropyLoss(weight=w.cuda())
crit(m(hsi.cuda(), lidar.cuda()), target.cuda()).backward(); torch.cuda.synchronize()
sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
masks = relu_masks_from_workspace(m, 4)
st64 = O.make_state(sd64)
masked_oracle_step(O, st64, hsi.double(), lidar.double(), target, w.double(), masks)
st64n = O.make_state(sd64)
masked_oracle_step(O, st64n, hsi.double(), lidar.double(), target, w.double(),
                   {k: v for k, v in masks.items() if "token" not in k and "feature" not in k or "local" in k})
flat = m.flat_params.grad.cpu().double()
named = dict(m.named_parameters())
gmax = max(float(st64[k].grad.abs().max()) for k in O.param_names(st64) if st64[k].grad is not None)
rows = []
for n, off in m._poff.items():
    if st64[n].grad is None:
        continue
    got = flat[off:off + named[n].numel()].view(named[n].shape)
    r, rn = st64[n].grad, st64n[n].grad
    err = float((got - r).abs().max()); errn = float((got - rn).abs().max())
    tol = 1e-3 * float(r.abs().max()) + 1e-5 * gmax
    rows.append((err / tol, n, err, errn, float(r.abs().max())))
rows.sort(reverse=True)
for q, n, e, en, sc in rows[:25]:
    print(f"{q:8.3f} {n:60s} err {e:.2e} (without TL masks {en:.2e}) scale {sc:.2e}")
