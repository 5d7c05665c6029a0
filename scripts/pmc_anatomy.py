#!/usr/bin/env python3
"""Per-kernel SQ anatomy from rocprofv3 `--pmc ... --output-format csv` passes
(scripts/kernel_pmc.sh): median counter value per launch of the kernels whose
name contains --kernel, then the derived issue / wait / MFMA-busy fractions.

    python scripts/pmc_anatomy.py DIR [DIR ...] --kernel gemm_ppp_kernel [--out FILE.md]

SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles;
SQ_VALU_MFMA_BUSY_CYCLES and SQ_BUSY_CYCLES count cycles (MI355X_MICROARCH.md
cycle-constants table).  GRBM_GUI_ACTIVE is the sum over the 8 XCDs.
"""
import argparse
import collections
import csv
import glob
import os
import statistics


def rows(d):
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            yield from csv.DictReader(fh)


def get(r, *names):
    for n in names:
        if n in r and r[n] != "":
            return r[n]
    raise KeyError(names)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--grid", type=int, default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    per = collections.defaultdict(list)
    for d in a.dirs:
        # one value per (dispatch, counter): rocprofv3 may emit per-dimension rows
        acc = collections.defaultdict(float)
        for r in rows(d):
            name = get(r, "Kernel_Name", "kernel_name")
            if a.kernel not in name:
                continue
            g = int(float(get(r, "Grid_Size", "grid_size")))
            if a.grid is not None and g != a.grid:
                continue
            disp = get(r, "Dispatch_Id", "dispatch_id", "Correlation_Id", "correlation_id")
            acc[(disp, get(r, "Counter_Name", "counter_name"))] += float(get(r, "Counter_Value", "counter_value"))
        for (disp, c), v in acc.items():
            per[c].append(v)
    med = {c: statistics.median(v) for c, v in per.items()}
    lines = [f"# SQ anatomy of `{a.kernel}` (median per launch)", "", "| counter | value | launches |", "|---|---|---|"]
    for c in sorted(med):
        lines.append(f"| {c} | {med[c]:.4g} | {len(per[c])} |")
    wc = med.get("SQ_WAVE_CYCLES")
    if wc:
        lines += ["", "| share of wave cycles | |", "|---|---|"]
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_MFMA",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC", "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_LDS"):
            if c in med:
                lines.append(f"| {c} | {med[c] / wc:.3f} |")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in med and "SQ_BUSY_CYCLES" in med:
        # MFMA busy is summed over SIMDs; SQ_BUSY_CYCLES over SEs/XCDs
        lines.append(f"| MFMA busy / SQ busy | {med['SQ_VALU_MFMA_BUSY_CYCLES'] / med['SQ_BUSY_CYCLES']:.3f} |")
    if "GRBM_GUI_ACTIVE" in med:
        lines.append(f"| GRBM_GUI_ACTIVE / 8 (cycles per XCD) | {med['GRBM_GUI_ACTIVE'] / 8:.4g} |")
    text = "\n".join(lines) + "\n"
    print(text)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(text)


if __name__ == "__main__":
    main()
