#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace database (or CSV) per kernel/grid:
count, total ms, average us -- the committed profiles/*.md tables come from this."""
import sqlite3
import sys


def main(path, steps=None):
    c = sqlite3.connect(path)
    rows = c.execute("select name, grid_x, workgroup_x, count(*), sum(duration)/1e6, avg(duration)/1e3, "
                     "min(duration)/1e3, max(duration)/1e3, max(vgpr_count), max(lds_size) from kernels "
                     "group by name, grid_x order by sum(duration) desc").fetchall()
    tot = sum(r[4] for r in rows)
    print(f"| kernel | grid | n | total ms | avg us | min us | max us | vgpr | lds | share |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for r in rows:
        if r[4] < 0.002 * tot:
            continue
        name = r[0]
        if name.startswith("void "):
            name = name[5:]
        name = name.replace("(anonymous namespace)::", "").split("(")[0]
        print(f"| {name[:100]} | {r[1]} | {r[3]} | {r[4]:.2f} | {r[5]:.1f} | {r[6]:.1f} | {r[7]:.1f} | {r[8]} | {r[9]} | {100*r[4]/tot:.1f}% |")
    print(f"\ntotal kernel time {tot:.2f} ms over {sum(r[3] for r in rows)} dispatches")


if __name__ == "__main__":
    main(sys.argv[1])
