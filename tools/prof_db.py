"""Per-iteration kernel summary from a rocprofv3 results database (rocpd sqlite).

usage: python tools/prof_db.py <run_results.db> <iterations traced> [--grid] [--md out.md]
  --grid  split rows by launch grid (separates GEMM shapes sharing one kernel symbol)
"""
import sqlite3
import sys
from collections import defaultdict


def main():
    db, iters = sys.argv[1], float(sys.argv[2])
    by_grid = "--grid" in sys.argv
    md = sys.argv[sys.argv.index("--md") + 1] if "--md" in sys.argv else None
    c = sqlite3.connect(db)
    agg = defaultdict(lambda: [0.0, 0])
    for name, dur, gx, gy, gz in c.execute("select name, duration, grid_x, grid_y, grid_z from kernels"):
        key = (name, (gx, gy, gz) if by_grid else None)
        agg[key][0] += dur
        agg[key][1] += 1
    tot = sum(v[0] for v in agg.values())
    rows = sorted(agg.items(), key=lambda kv: -kv[1][0])
    lines = [f"total kernel time {tot / 1e6 / iters:.2f} ms/iteration ({iters:g} iterations traced)", "",
             "| ms/iter | % | calls/iter | avg us | kernel |", "|---:|---:|---:|---:|---|"]
    for (name, grid), (d, n) in rows:
        nm = name if len(name) < 110 else name[:107] + "..."
        if grid:
            nm += f" grid={grid}"
        lines.append(f"| {d / 1e6 / iters:.3f} | {100 * d / tot:.1f} | {n / iters:.1f} | {d / n / 1e3:.1f} | `{nm}` |")
    out = "\n".join(lines)
    print(out)
    if md:
        open(md, "w").write(out + "\n")


if __name__ == "__main__":
    main()
