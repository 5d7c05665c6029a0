#!/usr/bin/env python3
"""Per-kernel dispatch counts and time over the last N seconds of a rocprofv3
kernel-trace database (one step's launch anatomy).

    python scripts/prof_names.py RESULTS.db --last-s 0.08
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last-s", type=float, required=True)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select start, end, name from kernels order by start").fetchall()
    t_end = max(r[1] for r in rows)
    rows = [r for r in rows if r[0] >= t_end - a.last_s * 1e9]
    n = collections.Counter()
    t = collections.Counter()
    for s, e, name in rows:
        name = name[5:] if name.startswith("void ") else name
        name = name.replace("(anonymous namespace)::", "").split("(")[0][:110]
        n[name] += 1
        t[name] += (e - s) / 1e3
    print(f"{len(rows)} dispatches, {sum(t.values()) / 1e3:.2f} ms kernel time in the last {a.last_s} s")
    print("| kernel | n | total us | avg us |")
    print("|---|---|---|---|")
    for name, k in n.most_common():
        print(f"| {name} | {k} | {t[name]:.0f} | {t[name] / k:.1f} |")


if __name__ == "__main__":
    main()
