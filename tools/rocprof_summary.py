"""Summarise a rocprofv3 --kernel-trace database (or kernel_stats.csv) into per-kernel totals.

usage: python tools/rocprof_summary.py <run_results.db | dir> [--steps N] [--out profiles/x.md]
"""
import argparse
import glob
import os
import sqlite3


def load(path):
    if os.path.isdir(path):
        dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
        if not dbs:
            raise SystemExit(f"no .db under {path}")
        path = dbs[0]
    con = sqlite3.connect(path)
    rows = con.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                       "from kernels group by name order by sum(duration) desc").fetchall()
    return path, rows


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0] if "(" in name else name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=0, help="steps in the trace, for per-step numbers")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    path, rows = load(a.path)
    tot = sum(r[2] for r in rows)
    lines = [f"# rocprofv3 --kernel-trace --stats summary ({os.path.basename(path)})", "",
             f"total kernel time {tot / 1e6:.3f} ms over {sum(r[1] for r in rows)} dispatches"
             + (f"; per step {tot / 1e6 / a.steps:.3f} ms, {sum(r[1] for r in rows) / a.steps:.0f} dispatches"
                if a.steps else ""), "",
             "| kernel | calls | total ms | avg us | min us | max us | % |", "|---|---|---|---|---|---|---|"]
    for n, c, s, av, mn, mx in rows:
        lines.append(f"| `{short(n)}` | {c} | {s / 1e6:.3f} | {av / 1e3:.2f} | {mn / 1e3:.2f} | {mx / 1e3:.2f} | "
                     f"{100 * s / tot:.1f} |")
    text = "\n".join(lines) + "\n"
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)
    print(text)


if __name__ == "__main__":
    main()
