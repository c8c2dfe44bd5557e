"""GPU tool: how far the bf16-operand mode (BASELINE config 2) lands from the fp32 oracle on the
reference's B=64 golden batch — logits, argmax, loss, gradients, and a short training trajectory.
usage: python tools/bf16_check.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "vit-cnn_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from helpers import golden_batch, hash_state_dict, load_npz  # noqa: E402
from oracle import vitcnn_oracle as O  # noqa: E402
import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
from vitcnn_amd import AdamW, CrossEntropyLoss, Multimodality_Mamba, fused_train_step  # noqa: E402


def run(prec, sd, hsi, lidar, target, w, steps=0):
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16, precision=prec)
    m.load_state_dict(sd)
    m = m.cuda().train()
    crit = CrossEntropyLoss(weight=w.cuda())
    logits = m(hsi.cuda(), lidar.cuda())
    loss = crit(logits, target.cuda())
    loss.backward()
    torch.cuda.synchronize()
    out = dict(logits=logits.detach().cpu().numpy(), loss=float(loss), grad=m.flat_params.grad.detach().cpu().clone())
    if steps:
        opt = AdamW(m.parameters(), lr=8e-4)
        m.zero_grad()
        losses = []
        for _ in range(steps):
            m.zero_grad()
            losses.append(float(fused_train_step(m, crit, hsi.cuda(), lidar.cuda(), target.cuda(), optimizer=opt)))
        out["traj"] = losses
        m.eval()
        with torch.no_grad():
            out["eval_logits"] = m(hsi.cuda(), lidar.cuda()).cpu().numpy()
    return out


def main():
    sd = hash_state_dict()
    hsi, lidar, target = golden_batch("golden.b64", 64)
    w = O.ce_class_weights(16)
    g = load_npz("vitcnn_b64.npz")
    ref = g["logits"]
    res = {p: run(p, sd, hsi, lidar, target, w, steps=30) for p in ("fp32", "bf16")}
    for p, r in res.items():
        lg = r["logits"]
        rel = np.abs(lg - ref).max() / np.abs(ref).max()
        agree = (lg.argmax(1) == ref.argmax(1)).mean()
        top2 = np.sort(ref, axis=1)[:, -2:]
        margin = (top2[:, 1] - top2[:, 0]) / np.abs(ref).max()
        print(f"{p}: logits rel err vs reference golden {rel:.3e}, argmax agreement {agree*100:.1f}% "
              f"(margins: min {margin.min():.2e} median {np.median(margin):.2e}), loss {r['loss']:.6f} "
              f"(golden {float(g['loss']):.6f})")
    g32, g16 = res["fp32"]["grad"].double(), res["bf16"]["grad"].double()
    cos = float((g32 @ g16) / (g32.norm() * g16.norm()))
    print(f"flat gradient: cos(bf16, fp32) {cos:.6f}, rel L2 {float((g16 - g32).norm() / g32.norm()):.3e}")
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16)
    named = dict(m.named_parameters())
    worst = []
    for n, off in m._poff.items():
        k = named[n].numel()
        a, b = g32[off:off + k], g16[off:off + k]
        if float(a.norm()) > 0:
            worst.append((float((a - b).norm() / a.norm()), n))
    worst.sort(reverse=True)
    print("largest per-tensor gradient rel L2 errors:", [(f"{e:.2e}", n) for e, n in worst[:8]])
    print("trajectory fp32:", [f"{x:.4f}" for x in res["fp32"]["traj"][::5]])
    print("trajectory bf16:", [f"{x:.4f}" for x in res["bf16"]["traj"][::5]])
    e32, e16 = res["fp32"]["eval_logits"], res["bf16"]["eval_logits"]
    print(f"after 30 steps, eval logits: rel err {np.abs(e16 - e32).max() / np.abs(e32).max():.3e}, "
          f"argmax agreement {(e16.argmax(1) == e32.argmax(1)).mean()*100:.1f}%, classes {len(set(e32.argmax(1)))}")


if __name__ == "__main__" and "--stages" not in sys.argv:
    main()


def stage_errors():
    """rel error of every named workspace activation, bf16 mode vs fp32 mode (same weights / batch)"""
    sd = hash_state_dict()
    hsi, lidar, target = golden_batch("golden.b64", 64)
    ws = {}
    for prec in ("fp32", "bf16"):
        m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16, precision=prec)
        m.load_state_dict(sd)
        m = m.cuda().train()
        with torch.no_grad():
            m(hsi.cuda(), lidar.cuda())
        torch.cuda.synchronize()
        w = next(v for k, v in m._ws.items() if k[2][0] == "train")
        ws[prec] = {k: t.detach().float().cpu().clone() for k, t in w.t.items() if t.is_floating_point()}
    rows = []
    for k, a in ws["fp32"].items():
        b = ws["bf16"].get(k)
        if b is None or a.numel() != b.numel() or a.numel() < 16:
            continue
        sc = float(a.abs().max())
        if sc == 0:
            continue
        rows.append((float((a - b).abs().max()) / sc, k))
    order = [k for k in ws["fp32"]]
    for e, k in sorted(rows, key=lambda r: order.index(r[1])):
        print(f"  {k:45s} {e:.3e}")


if __name__ == "__main__" and "--stages" in sys.argv:
    stage_errors()
