"""Average PMC counter values per kernel (name, grid) from rocprofv3 run_results.db files.
usage: python tools/pmc_db.py DIR [DIR ...]"""
import collections
import re
import sqlite3
import sys


def _short(k):
    m = re.search(r"(\w+<[^<>]*>)\(", k) or re.search(r"(\w+)\(", k)
    return m.group(1) if m else k[:40]


def main():
    rows = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[1:]:
        db = sqlite3.connect(f"{d}/run_results.db")
        cols = [r[1] for r in db.execute("pragma table_info(counters_collection)")]
        cn = "counter_name" if "counter_name" in cols else None
        q = ("select kernel_name, grid_size_x, grid_size_y, grid_size_z, dispatch_id, "
             "counter_name, value, duration from counters_collection")
        per = collections.defaultdict(float)
        for k, gx, gy, gz, disp, c, v, du in db.execute(q):
            per[(_short(k), gx // 256, gy, gz, disp, "duration_us")] = du / 1e3
            per[(_short(k), gx // 256, gy, gz, disp, c)] += v
        for (k, gx, gy, gz, disp, c), v in per.items():
            rows[(k, gx, gy, gz)][c].append(v)
    for key, ctrs in rows.items():
        print(key)
        for c, vs in sorted(ctrs.items()):
            print(f"   {c:28s} {sum(vs) / len(vs):14.4g}  (n={len(vs)})")


if __name__ == "__main__":
    main()
