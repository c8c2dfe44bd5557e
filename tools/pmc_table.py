"""Per-kernel PMC table of one ViT-CNN training step (tools/pmc_step.sh output) as markdown.

usage: python tools/pmc_table.py gpurun_out/TAG_summary.txt [--steps 3] > profiles/rNN_pmc_step.md

Columns per kernel (grid size distinguishes the launches of one kernel template):
  * MFMA util  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x 256 CUs)   (round-1 normalisation,
                 checked against the flop-rate fraction of the largest FusAtNet GEMM)
  * VALU issue = 4 x SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)   (a wave64 VALU instruction
                 holds its SIMD 4 cycles; GRBM_GUI_ACTIVE is summed over the 8 XCDs)
  * HBM bytes  = FETCH_SIZE + WRITE_SIZE (KB as reported; gfx950 corrections per MI355X_MICROARCH.md
                 are NOT applied here, the raw counters are shown)
"""
import argparse
import re


def parse(path):
    rows = []
    cur = None
    for line in open(path):
        m = re.match(r"^(\S.*?)  grid=(\d+)  avg duration ([\d.]+) us", line)
        if m:
            cur = {"name": m.group(1), "grid": int(m.group(2)), "us": float(m.group(3)), "c": {}}
            rows.append(cur)
            continue
        p = line.split()
        if cur is not None and len(p) == 2:
            try:
                cur["c"][p[0]] = float(p[1])
            except ValueError:
                pass
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("summary")
    ap.add_argument("--top", type=int, default=45)
    a = ap.parse_args()
    rows = sorted(parse(a.summary), key=lambda r: -r["us"])
    print("| kernel | grid (threads) | avg us | MFMA util | VALU issue | FETCH KB | WRITE KB |")
    print("|---|---|---|---|---|---|---|")
    for r in rows[: a.top]:
        c = r["c"]
        gui = c.get("GRBM_GUI_ACTIVE", 0.0)
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        valu = c.get("SQ_INSTS_VALU", 0.0)
        mfu = mf / (gui * 256) if gui else 0.0
        vu = 4 * valu / (gui / 8 * 1024) if gui else 0.0
        print(f"| `{r['name']}` | {r['grid']} | {r['us']:.1f} | {mfu:.3f} | {vu:.3f} | "
              f"{c.get('FETCH_SIZE', 0):.0f} | {c.get('WRITE_SIZE', 0):.0f} |")


if __name__ == "__main__":
    main()
