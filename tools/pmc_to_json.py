"""Fold the FETCH_SIZE / WRITE_SIZE passes of tools/pmc_collect.sh into profiles/r01_pmc.json:
per kernel (name<template>, largest grid = the hsi1 launch for the scan kernels) the mean per-launch
counter values and HBM bytes.  rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KB (derived from
TCC_EA0_RDREQ / _WRREQ).  MI355X_MICROARCH.md: FETCH_SIZE counts half of the bytes of 16-B/lane
streaming reads; the same factor holds here for coalesced 4-B/lane reads (calibrated on this run:
sum_bc_chunks streams 33.2 MB of split slabs and reports 16.2 MB; adamw's 16-B reads of p,g,m,v
(26.6 MB) report 13.3 MB while its writes report exactly 19.9 MB).  hbm_bytes_per_launch is
therefore 2 x FETCH_SIZE + WRITE_SIZE (in bytes).
usage: pmc_to_json.py FETCH_DIR WRITE_DIR OUT.json"""
import glob
import json
import os
import sqlite3
import sys
from collections import defaultdict


def per_launch(d, counter):
    vals = defaultdict(lambda: defaultdict(float))
    dur = {}
    for db in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        con = sqlite3.connect(db)
        for disp, name, grid, ctr, val, du in con.execute(
                "select dispatch_id, kernel_name, grid_size, counter_name, value, duration from counters_collection"):
            if ctr != counter:
                continue
            short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            vals[(short, grid)][disp] += val
            dur[(short, grid, disp)] = du
    out = {}
    for (short, grid), per in vals.items():
        v = list(per.values())
        out[(short, grid)] = (sum(v) / len(v), len(v))
    return out


def main():
    fd, wd, outp = sys.argv[1:4]
    fetch, write = per_launch(fd, "FETCH_SIZE"), per_launch(wd, "WRITE_SIZE")
    best = {}
    for (short, grid) in set(fetch) | set(write):
        cur = best.get(short)
        if cur is None or grid > cur:
            best[short] = grid
    res = {}
    for short, grid in best.items():
        f = fetch.get((short, grid), (None, 0))[0]
        w = write.get((short, grid), (None, 0))[0]
        res[short] = {"grid_threads": grid, "FETCH_SIZE_kB": f, "WRITE_SIZE_kB": w,
                      "hbm_bytes_per_launch": (2 * f + w) * 1024 if f is not None and w is not None else None}
    doc = {"source": "rocprofv3 --kernel-trace --pmc FETCH_SIZE | WRITE_SIZE (separate passes) over "
                     "tools/run_steps.py 3 (B=64 training steps), MI355X", "kernels": res}
    with open(outp, "w") as fo:
        json.dump(doc, fo, indent=1, sort_keys=True)
    for k in sorted(res, key=lambda k: -(res[k]["hbm_bytes_per_launch"] or 0))[:15]:
        print(k, res[k])


if __name__ == "__main__":
    main()
