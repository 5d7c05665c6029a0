#!/usr/bin/env python3
"""Per-kernel HBM traffic and bandwidth from three rocprofv3 runs of one command
(MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE do not fit one TCC pass):

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d F -- <cmd>
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d W -- <cmd>
    rocprofv3 --kernel-trace --output-format csv -d T -- <cmd>

    python scripts/pmc_kernel_table.py F W T [--match conv_,upsample,dpt] [--out table.md]

For each (kernel, grid): launches, median bytes per launch = 2 x FETCH_SIZE
(gfx950 counts half the bytes of 16-B-per-lane streaming reads) + WRITE_SIZE
(both in KB), average duration from the kernel trace, and the achieved HBM rate
against the ~8 TB/s peak.  Rates from a profiled run read low (DVFS, item 2).
"""
import argparse
import csv
import glob
import os
import statistics
from collections import defaultdict

HBM_PEAK_GBS = 8000.0


def _rows(d, pattern):
    files = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    if not files:
        raise SystemExit(f"no {pattern} under {d}")
    for f in files:
        with open(f) as fh:
            yield from csv.DictReader(fh)


def _get(row, *names):
    for n in names:
        if n in row and row[n] != "":
            return row[n]
    raise KeyError(f"none of {names} in {list(row)}")


def _short(name):
    if name.startswith("void "):
        name = name[5:]
    return name.replace("(anonymous namespace)::", "").split("(")[0]


def counters(d, counter):
    out = defaultdict(list)
    for r in _rows(d, "*counter_collection.csv"):
        if _get(r, "Counter_Name", "counter_name") != counter:
            continue
        key = (_short(_get(r, "Kernel_Name", "kernel_name")),
               int(float(_get(r, "Grid_Size", "grid_size", "Grid_Size_X", "grid_x"))))
        out[key].append(float(_get(r, "Counter_Value", "counter_value")))
    return out


def durations(d):
    out = defaultdict(list)
    for r in _rows(d, "*kernel_trace.csv"):
        key = (_short(_get(r, "Kernel_Name", "kernel_name")),
               int(float(_get(r, "Grid_Size", "grid_size", "Grid_Size_X", "grid_x"))))
        out[key].append(float(_get(r, "End_Timestamp", "end_timestamp")) -
                        float(_get(r, "Start_Timestamp", "start_timestamp")))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("trace_dir")
    ap.add_argument("--match", default="", help="comma-separated substrings of kernel names to keep (default: all)")
    ap.add_argument("--min-ms", type=float, default=0.05, help="drop (kernel, grid) rows with less total time")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    fetch, write, dur = counters(a.fetch_dir, "FETCH_SIZE"), counters(a.write_dir, "WRITE_SIZE"), durations(a.trace_dir)
    keys = [k for k in dur if k in fetch and k in write]
    pats = [p for p in a.match.split(",") if p]
    if pats:
        keys = [k for k in keys if any(p in k[0] for p in pats)]
    rows = []
    for k in keys:
        ns = statistics.mean(dur[k])
        tot_ms = sum(dur[k]) / 1e6
        if tot_ms < a.min_ms:
            continue
        byt = 2.0 * statistics.median(fetch[k]) * 1024 + statistics.median(write[k]) * 1024
        gbs = byt / ns  # bytes per ns = GB/s
        rows.append((tot_ms, k, len(dur[k]), byt, ns, gbs))
    rows.sort(reverse=True)
    lines = ["| kernel | grid | n | total ms | avg us | HBM MB / launch | GB/s | of 8 TB/s |",
             "|---|---|---|---|---|---|---|---|"]
    for tot_ms, (name, grid), n, byt, ns, gbs in rows:
        lines.append(f"| {name[:80]} | {grid} | {n} | {tot_ms:.2f} | {ns / 1e3:.1f} | {byt / 1e6:.1f} | {gbs:.0f} | "
                     f"{gbs / HBM_PEAK_GBS:.2f} |")
    text = "\n".join(lines)
    print(text)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(text + "\n")


if __name__ == "__main__":
    main()
