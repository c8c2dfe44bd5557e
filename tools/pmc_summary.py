"""Per-kernel PMC counter values per dispatch from rocprofv3 --pmc databases (counters_collection).
usage: pmc_summary.py DIR [DIR...] [--filter NAME]
Groups dispatches by (kernel, grid size); prints the mean per-dispatch value of every counter."""
import argparse
import glob
import os
import sqlite3
from collections import defaultdict


def load(d, flt):
    out = defaultdict(lambda: defaultdict(list))   # (kernel, grid) -> counter -> [per-dispatch values]
    dur = defaultdict(list)
    for db in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        con = sqlite3.connect(db)
        rows = con.execute("select dispatch_id, kernel_name, grid_size, counter_name, value, duration "
                           "from counters_collection").fetchall()
        per = defaultdict(float)
        meta = {}
        for disp, name, grid, ctr, val, du in rows:
            if flt and flt not in name:
                continue
            per[(disp, ctr)] += val
            meta[disp] = (name, grid, du)
        for (disp, ctr), v in per.items():
            name, grid, du = meta[disp]
            short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            out[(short, grid)][ctr].append(v)
        for disp, (name, grid, du) in meta.items():
            short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            dur[(short, grid)].append(du)
    return out, dur


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    merged = defaultdict(dict)
    durs = {}
    for d in a.dirs:
        out, dur = load(d, a.filter)
        for k, v in out.items():
            for c, vals in v.items():
                merged[k][c] = sum(vals) / len(vals)
        for k, v in dur.items():
            durs[k] = sum(v) / len(v)
    for k in sorted(merged, key=lambda k: -durs.get(k, 0)):
        print(f"{k[0]}  grid={k[1]}  avg duration {durs.get(k, 0) / 1e3:.1f} us")
        for c, v in sorted(merged[k].items()):
            print(f"    {c:24s} {v:.6g}")


if __name__ == "__main__":
    main()
