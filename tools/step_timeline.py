"""Per-step kernel timeline from a rocprofv3 --kernel-trace database: the last `adamw`-terminated
step, each dispatch's duration, grid and the idle gap before it.  usage: step_timeline.py DB_OR_DIR"""
import glob
import os
import sqlite3
import sys


def main():
    p = sys.argv[1]
    if os.path.isdir(p):
        p = glob.glob(os.path.join(p, "**", "*.db"), recursive=True)[0]
    con = sqlite3.connect(p)
    rows = con.execute("select name, start, end, grid_x, grid_y, grid_z, workgroup_x, lds_size, vgpr_count, "
                       "accum_vgpr_count, scratch_size from kernels order by start").fetchall()
    ends = [i for i, r in enumerate(rows) if "adamw(" in r[0]]
    if len(ends) < 2:
        raise SystemExit("need two steps")
    a, b = ends[-2] + 1, ends[-1] + 1
    step = rows[a:b]
    t0 = step[0][1]
    busy = sum(r[2] - r[1] for r in step)
    span = step[-1][2] - t0
    print(f"dispatches {len(step)}  span {span/1e3:.1f} us  busy {busy/1e3:.1f} us  idle {(span-busy)/1e3:.1f} us")
    prev = t0
    for r in step:
        name = r[0].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]
        blocks = r[3] * r[4] * r[5] // max(r[6], 1)
        print(f"{(r[1]-t0)/1e3:8.1f} gap {(r[1]-prev)/1e3:5.1f} dur {(r[2]-r[1])/1e3:7.1f}  blk {blocks:6d} "
              f"lds {r[7]:6d} vgpr {r[8]:3d}/{r[9]:3d} scr {r[10]:4d}  {name}")
        prev = r[2]


if __name__ == "__main__":
    main()
