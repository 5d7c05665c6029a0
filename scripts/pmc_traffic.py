#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 PMC passes (MI355X_MICROARCH.md §HBM):
FETCH_SIZE and WRITE_SIZE are collected in separate passes (they do not fit one
TCC pass); on gfx950 FETCH_SIZE counts half the bytes of 16-B-per-lane streaming
reads, so it is doubled; WRITE_SIZE is taken as is.  Both are reported by
rocprofv3 in KB.

    python scripts/pmc_traffic.py FETCH_DIR WRITE_DIR --kernel attn_fwd_kernel --grid 704512 \
        [--out profiles/attn_traffic.json]

Each DIR is a `rocprofv3 --pmc <COUNTER> --output-format csv -d DIR` output
tree (the *counter_collection.csv file is located recursively).
"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys


def _stamp():
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "large-scale-vit-slam_amd"))
    from aligned_vggt.provenance import stamp
    return stamp()


def _rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no *counter_collection.csv under {d}")
    for f in files:
        with open(f) as fh:
            yield from csv.DictReader(fh)


def _get(row, *names):
    for n in names:
        if n in row and row[n] != "":
            return row[n]
    raise KeyError(f"none of {names} in {list(row)}")


def per_launch(d, counter, kernel, grid):
    vals = []
    for r in _rows(d):
        if _get(r, "Counter_Name", "counter_name") != counter:
            continue
        name = _get(r, "Kernel_Name", "kernel_name")
        g = int(float(_get(r, "Grid_Size", "grid_size", "Grid_Size_X", "grid_x")))
        if kernel in name and (grid is None or g == grid):
            vals.append(float(_get(r, "Counter_Value", "counter_value")))
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel} grid {grid} in {d}")
    return statistics.median(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--kernel", default="attn_fwd_kernel")
    ap.add_argument("--grid", type=int, default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    fetch_kb, nf = per_launch(a.fetch_dir, "FETCH_SIZE", a.kernel, a.grid)
    write_kb, nw = per_launch(a.write_dir, "WRITE_SIZE", a.kernel, a.grid)
    traffic = 2.0 * fetch_kb * 1024 + write_kb * 1024
    res = {"kernel": a.kernel, "grid": a.grid, "fetch_size_kb_raw": fetch_kb, "write_size_kb": write_kb,
           "launches": [nf, nw], "hbm_bytes_per_launch": traffic,
           "correction": "FETCH_SIZE x2 (gfx950 16-B/lane streaming reads), WRITE_SIZE x1",
           **_stamp()}
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
