"""Critical path of the ViT-CNN B=64 training step's lane DAG (forward + backward programs).

Pass 1 records the program's launch structure: every C-ABI call with its lane, and the cross-lane
edges (event marks and waits).  Pass 2 (every lane mapped onto one stream) times every call with HIP
events, the GPU held back by a sleep kernel first so that the host has queued everything and the
events measure back-to-back device time (each call's kernels plus its launch gaps).  Both passes issue
the same calls in the same order.  The DAG replayed with those durations gives the critical path of
an ideal lane schedule (no cross-queue costs): its length, the calls on it, and what each lane holds.
usage: python tools/critical_path.py [--top 40]"""
import argparse
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-cnn_amd"))
import torch  # noqa: E402

import knobs  # noqa: F401,E402  (measurement switches: tools/knobs.py)
import vitcnn_amd.model as M  # noqa: E402
from vitcnn_amd import AdamW, CrossEntropyLoss, Multimodality_Mamba, fused_train_step  # noqa: E402


class _Wrapped:
    def __init__(self, L, prog, tracer):
        self._L, self._prog, self._t = L, prog, tracer

    def __getattr__(self, name):
        fn = getattr(self._L, name)
        if not name.startswith("vc_") or name.endswith("_floats"):
            return fn

        def call(*args):
            return self._t.call(name, self._prog, fn, args)
        return call


class Tracer:
    def __init__(self, timing):
        self.timing = timing
        self.nodes = []             # (name, lane, [dep node indices])
        self.last = defaultdict(lambda: -1)   # lane -> last node index
        self.pending = defaultdict(list)      # lane -> events waited since its last node
        self.marks = {}             # id(event) -> node index it follows
        self.ev = []

    def wrap(self, L, prog):
        return _Wrapped(L, prog, self)

    def mark(self, e, lane):
        self.marks[id(e)] = self.last[lane]

    def wait(self, e, lane):
        self.pending[lane].append(self.marks.get(id(e), -1))

    def call(self, name, prog, fn, args):
        lane = prog.cur
        deps = [d for d in self.pending.pop(lane, []) if d >= 0]
        if self.last[lane] >= 0:
            deps.append(self.last[lane])
        if self.timing:   # one event per call boundary: call i spans ev[i] .. ev[i + 1]
            st = prog.streams[lane]
            if not self.ev:
                self.ev.append(torch.cuda.Event(enable_timing=True))
                self.ev[0].record(st)
            r = fn(*args)
            self.ev.append(torch.cuda.Event(enable_timing=True))
            self.ev[-1].record(st)
        else:
            r = fn(*args)
        self.last[lane] = len(self.nodes)
        self.nodes.append((name, lane, deps))
        return r


def setup(dev):
    torch.manual_seed(0)
    m = Multimodality_Mamba(9, 1, 1, 144, 1, 32, 16).to(dev).train()
    opt = AdamW(m.parameters(), lr=8e-4)
    w = torch.ones(16)
    w[0] = 0.0
    crit = CrossEntropyLoss(weight=w.to(dev))
    g = torch.Generator().manual_seed(1000)
    hsi = torch.rand(64, 144, 9, 9, generator=g).to(dev)
    lidar = torch.rand(64, 1, 9, 9, generator=g).to(dev)
    tgt = torch.randint(1, 16, (64,), generator=g).to(dev)
    return m, opt, crit, hsi, lidar, tgt


def run(m, opt, crit, hsi, lidar, tgt, tracer, one_stream):
    """one step; one_stream: every lane mapped onto the current stream (the same calls in the same
    order as with lanes, serialised)"""
    M._TRACER = tracer
    orig = m._side_lanes
    if one_stream:
        m._side_lanes = lambda dev: [(torch.cuda.current_stream(dev), t) for _, t in orig(dev)]
    try:
        opt.zero_grad(set_to_none=True)
        if tracer is not None and tracer.timing:
            torch.cuda._sleep(200_000_000)   # ~0.1 s: the host queues the whole step behind it
        fused_train_step(m, crit, hsi, lidar, tgt, optimizer=opt)
        torch.cuda.synchronize()
    finally:
        M._TRACER = None
        m._side_lanes = orig


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    m, opt, crit, hsi, lidar, tgt = setup(dev)
    for _ in range(3):
        run(m, opt, crit, hsi, lidar, tgt, None, False)
    struct = Tracer(False)
    run(m, opt, crit, hsi, lidar, tgt, struct, False)
    timed = Tracer(True)
    run(m, opt, crit, hsi, lidar, tgt, timed, True)
    names_s = [n[0] for n in struct.nodes]
    names_t = [n[0] for n in timed.nodes]
    if names_s != names_t:
        raise SystemExit(f"call sequences differ: {len(names_s)} vs {len(names_t)}")
    dur = [timed.ev[i].elapsed_time(timed.ev[i + 1]) * 1e3 for i in range(len(timed.ev) - 1)]   # us
    n = len(dur)
    fin = [0.0] * n
    crit_pred = [-1] * n
    for i, (name, lane, deps) in enumerate(struct.nodes):
        start, pred = 0.0, -1
        for d in deps:
            if fin[d] > start:
                start, pred = fin[d], d
        fin[i] = start + dur[i]
        crit_pred[i] = pred
    end = max(range(n), key=lambda i: fin[i])
    path = []
    i = end
    while i >= 0:
        path.append(i)
        i = crit_pred[i]
    path.reverse()
    lanes = defaultdict(float)
    for i, (_, lane, _) in enumerate(struct.nodes):
        lanes[lane] += dur[i]
    print(f"calls {n}  serial sum {sum(dur):.1f} us  critical path {fin[end]:.1f} us over {len(path)} calls")
    print("per-lane sums: " + "  ".join(f"lane {k}: {v:.1f} us" for k, v in sorted(lanes.items())))
    on = defaultdict(lambda: [0, 0.0])
    for i in path:
        on[struct.nodes[i][0]][0] += 1
        on[struct.nodes[i][0]][1] += dur[i]
    print(f"\non the critical path, by entry point ({'calls':>5s}, us):")
    for k, (c, s) in sorted(on.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"  {k:28s} {c:5d} {s:8.1f}")
    print("\ncritical path, in order (lane, us, entry point):")
    for i in path:
        print(f"  {i:4d} L{struct.nodes[i][1]} {dur[i]:7.1f}  {struct.nodes[i][0]}")


if __name__ == "__main__":
    main()
