"""Fold a tools/pmc_summary.py text summary (tools/pmc_step.sh output: SQ / FETCH_SIZE / WRITE_SIZE
passes over the same training steps) into the JSON bench.py reads: per kernel (name<template>, the
largest grid = the hsi1 launch for the scan kernels) the mean per-launch counters, the HBM bytes
(2 x FETCH_SIZE + WRITE_SIZE, in bytes: the round-1 calibration of FETCH_SIZE for coalesced streaming
reads, tools/pmc_to_json.py) and the VALU-issue lower bound on the launch time
(SQ_INSTS_VALU x 4 cycles / 1024 SIMDs at the 2.4 GHz peak clock: a wave64 VALU instruction holds its
SIMD for 4 cycles).
usage: pmc_summary_json.py SUMMARY.txt OUT.json [SOURCE-DESCRIPTION]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_table import parse  # noqa: E402

CLOCK_HZ = 2.4e9
SIMDS = 1024


def main():
    src, outp = sys.argv[1:3]
    desc = sys.argv[3] if len(sys.argv) > 3 else "rocprofv3 --pmc, tools/pmc_step.sh"
    best = {}
    for r in parse(src):
        name = r["name"]
        if name not in best or r["grid"] > best[name]["grid"]:
            best[name] = r
    kernels = {}
    for name, r in best.items():
        c = r["c"]
        k = {"grid_threads": r["grid"], "avg_us_under_pmc": r["us"]}
        for key in ("FETCH_SIZE", "WRITE_SIZE"):
            if key in c:
                k[key + "_kB"] = c[key]
        for key in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_ACTIVE_INST_VALU",
                    "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"):
            if key in c:
                k[key] = c[key]
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            k["hbm_bytes_per_launch"] = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
        if "SQ_INSTS_VALU" in c:
            k["valu_issue_bound_us"] = c["SQ_INSTS_VALU"] * 4 / SIMDS / CLOCK_HZ * 1e6
        kernels[name] = k
    with open(outp, "w") as f:
        json.dump({"source": desc, "kernels": kernels}, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
