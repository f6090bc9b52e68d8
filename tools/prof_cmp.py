"""Per-kernel (symbol, grid) time per iteration of two rocprofv3 kernel traces (rocpd databases).
usage: python tools/prof_cmp.py <dir A> <dir B> <iterations traced>"""
import sqlite3
import sys
from collections import defaultdict
from pathlib import Path


def load(d, iters):
    db = next(Path(d).rglob("*.db"))
    agg = defaultdict(lambda: [0.0, 0])
    for name, dur, gx, gy, gz in sqlite3.connect(db).execute("select name, duration, grid_x, grid_y, grid_z from kernels"):
        k = (name[:100], (gx, gy, gz))
        agg[k][0] += dur / iters / 1e3
        agg[k][1] += 1
    return agg


def main():
    a, b, iters = sys.argv[1], sys.argv[2], float(sys.argv[3])
    A, B = load(a, iters), load(b, iters)
    ta, tb = sum(v[0] for v in A.values()), sum(v[0] for v in B.values())
    print(f"total us/iter: A {ta:.1f}  B {tb:.1f}  diff {tb - ta:+.1f}")
    rows = []
    for k in set(A) | set(B):
        va, vb = A.get(k, [0.0, 0]), B.get(k, [0.0, 0])
        rows.append((vb[0] - va[0], va[0], vb[0], va[1], vb[1], k))
    rows.sort(key=lambda r: -abs(r[0]))
    for d, va, vb, na, nb, k in rows[:45]:
        print(f"{d:+9.1f} us  A {va:9.1f} ({na:4d})  B {vb:9.1f} ({nb:4d})  {k[0]} {k[1]}")


if __name__ == "__main__":
    main()
