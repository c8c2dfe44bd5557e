"""Per-step kernel timeline from a rocprofv3 --kernel-trace database: the last `adamw`-terminated
step, each dispatch's duration, grid and the idle gap before it.

With several lanes (side streams) kernels overlap: `busy` is the union of the dispatch intervals (time
at least one kernel runs), `sum` the summed durations, and the concurrency histogram says how much of
the span ran 0 / 1 / 2 / 3+ kernels at once.  `--summary` prints only the totals and a per-kernel-name
table (count, summed us) — the launch census of one step.
usage: step_timeline.py DB_OR_DIR [--summary]"""
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]


def main():
    p = sys.argv[1]
    summary = "--summary" in sys.argv
    if os.path.isdir(p):
        p = glob.glob(os.path.join(p, "**", "*.db"), recursive=True)[0]
    con = sqlite3.connect(p)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    qcol = next((c for c in ("queue_id", "stream_id") if c in cols), None)
    sel = "name, start, end, grid_x, grid_y, grid_z, workgroup_x, lds_size, vgpr_count, accum_vgpr_count, scratch_size"
    if qcol:
        sel += ", " + qcol
    rows = con.execute(f"select {sel} from kernels order by start").fetchall()
    ends = [i for i, r in enumerate(rows) if "adamw(" in r[0]]
    if len(ends) < 2:
        raise SystemExit("need two steps")
    a, b = ends[-2] + 1, ends[-1] + 1
    step = rows[a:b]
    t0 = step[0][1]
    span = max(r[2] for r in step) - t0
    total = sum(r[2] - r[1] for r in step)
    # union of intervals + concurrency histogram (sweep over start / end events)
    ev = sorted([(r[1], 1) for r in step] + [(r[2], -1) for r in step])
    hist = defaultdict(float)
    level, last = 0, t0
    for t, d in ev:
        hist[min(level, 3)] += t - last
        level += d
        last = t
    busy = span - hist[0]
    queues = sorted({r[-1] for r in step}) if qcol else []
    print(f"dispatches {len(step)}  span {span/1e3:.1f} us  busy(union) {busy/1e3:.1f} us  "
          f"sum {total/1e3:.1f} us  idle {hist[0]/1e3:.1f} us  queues {len(queues)}")
    print("concurrency: " + "  ".join(f"{k}{'+' if k == 3 else ''}: {hist[k]/1e3:.1f} us" for k in range(4)))
    if summary:
        agg = defaultdict(lambda: [0, 0.0])
        for r in step:
            n = short(r[0])
            agg[n][0] += 1
            agg[n][1] += (r[2] - r[1]) / 1e3
        print(f"{'kernel':48s} {'count':>5s} {'sum us':>8s} {'avg us':>7s}")
        for n, (c, s) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            print(f"{n:48s} {c:5d} {s:8.1f} {s / c:7.1f}")
        return
    prev = t0
    for r in step:
        blocks = r[3] * r[4] * r[5] // max(r[6], 1)
        q = f" q{queues.index(r[-1])}" if qcol else ""
        print(f"{(r[1]-t0)/1e3:8.1f} gap {(r[1]-prev)/1e3:5.1f} dur {(r[2]-r[1])/1e3:7.1f}  blk {blocks:6d} "
              f"lds {r[7]:6d} vgpr {r[8]:3d}/{r[9]:3d} scr {r[10]:4d}{q}  {short(r[0])}")
        prev = max(prev, r[2])


if __name__ == "__main__":
    main()
