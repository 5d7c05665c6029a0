#!/usr/bin/env python3
"""Per-HW-queue view of a rocprofv3 kernel trace (CSV): launches, busy time,
span, and the gaps between consecutive kernels of each queue -- used on the
overlapped chunk pipeline to see whether the alignment stream's kernels run
slowly or wait.

    python scripts/queue_gaps.py TRACE_DIR [--top 12]
"""
import argparse
import csv
import glob
import os
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    q = defaultdict(list)
    for r in rows:
        q[r.get("Queue_Id", "?")].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    for qid, ks in sorted(q.items(), key=lambda kv: -len(kv[1])):
        ks.sort()
        busy = sum(e - s for s, e, _ in ks) / 1e6
        span = (ks[-1][1] - ks[0][0]) / 1e6
        gaps = [max(0, ks[i + 1][0] - ks[i][1]) / 1e3 for i in range(len(ks) - 1)]
        print(f"queue {qid}: {len(ks)} kernels, busy {busy:.1f} ms, span {span:.1f} ms, "
              f"median gap {statistics.median(gaps) if gaps else 0:.1f} us, mean gap {statistics.mean(gaps) if gaps else 0:.1f} us")
        by = defaultdict(lambda: [0, 0.0])
        for s, e, n in ks:
            n = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:70]
            by[n][0] += 1
            by[n][1] += (e - s) / 1e3
        for n, (c, t) in sorted(by.items(), key=lambda kv: -kv[1][1])[:a.top]:
            print(f"    {n:70s} {c:6d}  {t / 1e3:8.2f} ms  {t / c:8.1f} us avg")


if __name__ == "__main__":
    main()
