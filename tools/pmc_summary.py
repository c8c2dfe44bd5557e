"""Per-kernel PMC counter averages from a rocprofv3 --pmc database.  usage: pmc_summary.py DIR [name-filter]"""
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    for db in dbs:
        con = sqlite3.connect(db)
        tabs = [r[0] for r in con.execute("select name from sqlite_master where type in ('table','view')")]
        pmc = [t for t in tabs if t.startswith("counters") or t == "pmc_events" or "counter" in t.lower()]
        print(db, pmc)
        if "counters" not in tabs:
            continue
        cols = [r[1] for r in con.execute("pragma table_info(counters)")]
        print(cols)
        rows = con.execute("select * from counters").fetchall()
        agg = defaultdict(lambda: defaultdict(list))
        ci = {c: i for i, c in enumerate(cols)}
        for r in rows:
            name = r[ci.get("kernel_name", ci.get("name", 0))]
            if flt and flt not in str(name):
                continue
            agg[str(name).split("(")[0][-40:]][r[ci["counter_name"]]].append(r[ci["value"]])
        for k, v in agg.items():
            print(k)
            for c, vals in sorted(v.items()):
                print("   %-28s mean %.4g  (n=%d)" % (c, sum(vals) / len(vals), len(vals)))


if __name__ == "__main__":
    main()
