"""Which gradient slices depend on the lane schedule?

For a channel-chain placement (_CH_LANE, _CH_ORDERED), the fused B=64 step's flat gradient under the
four-lane schedule (eager, twice, and replayed from a hipGraph) and under the single-stream backward
(eager and replayed) is compared with the first four-lane eager run, parameter slice by parameter slice:
the slices that differ name the kernels whose inputs were formed in a schedule-dependent order.
usage: python tools/lane_probe.py CH_LANE ORDERED   (e.g. 3 0 = the round-3 experiment, no ordering)
"""
import os
import sys

import knobs  # noqa: F401,E402
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from helpers import golden_batch, hash_state_dict  # noqa: E402
from oracle import vitcnn_oracle as O  # noqa: E402
from test_model_gpu import _product, _schedule_grad  # noqa: E402
from vitcnn_amd import CrossEntropyLoss  # noqa: E402

ch_lane, ordered = int(sys.argv[1]), sys.argv[2] == "1"
sd = hash_state_dict()
batch = tuple(t.to("cuda") for t in golden_batch("golden.b64", 64))
crit = CrossEntropyLoss(weight=O.ce_class_weights(16).to("cuda"))
m = _product(sd)
names = sorted(m._poff, key=lambda n: m._poff[n])
ref_loss, ref = _schedule_grad(sd, batch, crit, False, True, (), ch_lane, ordered)
runs = [("four lanes, eager (again)", False, True), ("four lanes, replayed", True, True),
        ("single-stream backward, eager", False, False), ("single-stream backward, replayed", True, False)]
print(f"channel chain on lane {ch_lane}, dX accumulation ordered: {ordered}")
for label, captured, lanes_bwd in runs:
    loss, g = _schedule_grad(sd, batch, crit, captured, lanes_bwd, (), ch_lane, ordered)
    diff = []
    for n in names:
        o, k = m._poff[n], dict(m.named_parameters())[n].numel()
        d = float((g[o:o + k] - ref[o:o + k]).abs().max())
        if d > 0:
            diff.append((n, d, float(ref[o:o + k].abs().max())))
    blocks = sorted({n.split(".")[0] + "." + n.split(".")[1] for n, _, _ in diff})
    print(f"  {label}: loss equal {loss == ref_loss}, {len(diff)} of {len(names)} slices differ; blocks: {blocks}")
    for n, d, sc in diff[:12]:
        print(f"      {n}: max |diff| {d:.3e} (scale {sc:.3e})")
