import os, sys
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/vit-cnn_amd"); sys.path.insert(0, "/root/repo/tests")
import torch
from helpers import golden_batch, hash_state_dict
from oracle import vitcnn_oracle as O
import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
from vitcnn_amd import Multimodality_Mamba, CrossEntropyLoss
sd = hash_state_dict()
hsi, lidar, target = golden_batch("golden.b4", 4)
m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16); m.load_state_dict(sd); m = m.to("cuda").train()
w = O.ce_class_weights(16)
crit = CrossEntropyLoss(weight=w.to("cuda"))
logits = m(hsi.cuda(), lidar.cuda())
torch.cuda.synchronize()
ws = next(v for k, v in m._ws.items() if k[2][0] == "train")
snap = {k: t.clone() for k, t in ws.t.items()}
loss = crit(logits, target.cuda()); loss.backward(); torch.cuda.synchronize()
for k, t in ws.t.items():
    if k in snap and not k.startswith(("hsi1.d", "hsi2.d")) and ".d" not in k[-6:]:
        a, b = snap[k], t
        if a.dtype.is_floating_point:
            diff = (a - b).abs().max().item()
        else:
            diff = (a != b).sum().item()
        if diff != 0:
            print("CHANGED", k, a.numel(), diff, a.data_ptr())
print("done")
