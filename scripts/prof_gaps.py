#!/usr/bin/env python3
"""GPU idle time between kernels in a rocprofv3 kernel-trace database: sorts
dispatches by start, reports the busy span, the summed kernel time, the idle
gaps (> --min-us) and the largest ones with the kernels on either side.

    python scripts/prof_gaps.py RESULTS.db [--last-s 2.0] [--min-us 5] [--top 15]
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last-s", type=float, default=0.0, help="only the last N seconds of the trace (0: all)")
    ap.add_argument("--min-us", type=float, default=5.0)
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select start, end, name from kernels order by start").fetchall()
    if a.last_s > 0:
        t_end = max(r[1] for r in rows)
        rows = [r for r in rows if r[0] >= t_end - a.last_s * 1e9]
    busy = 0
    gaps = []
    cur_end = rows[0][1]
    prev_name = rows[0][2]
    busy += rows[0][1] - rows[0][0]
    for s, e, n in rows[1:]:
        busy += e - s
        if s > cur_end:
            g = (s - cur_end) / 1e3
            if g > a.min_us:
                gaps.append((g, prev_name[:60], n[:60]))
        if e > cur_end:
            cur_end = e
            prev_name = n
    span = (rows[-1][1] - rows[0][0]) / 1e6
    tot_gap = sum(g for g, _, _ in gaps) / 1e3
    print(f"dispatches {len(rows)}  span {span:.2f} ms  kernel time {busy / 1e6:.2f} ms  "
          f"idle gaps > {a.min_us} us: {len(gaps)} totalling {tot_gap:.2f} ms")
    for g, p, n in sorted(gaps, reverse=True)[:a.top]:
        print(f"  {g:10.1f} us  after {p}  before {n}")


if __name__ == "__main__":
    main()
