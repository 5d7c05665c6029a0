#!/usr/bin/env python3
"""Counter-based MFMA utilisation of one bench step.

Input: rocprofv3 `--pmc ... --output-format csv` directories of one
`bench.py --steps 1 --warmup 1 --no-cpu-baseline` run each (one counter group
per pass, scripts/gpu_step_pmc.sh).  The timed step is the second half of the
dispatches (the warmup step is the same kernel sequence).  Per pass:

  * SQ_VALU_MFMA_BUSY_CYCLES (summed over the SIMDs) / (SIMDs x GRBM_GUI_ACTIVE / 8)
      = the fraction of SIMD-cycles with the matrix pipe busy, over the step's
        kernel time (GRBM_GUI_ACTIVE is the sum over the 8 XCDs);
  * SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 = bf16 MFMA FLOPs the hardware counted
      (MI355X_MICROARCH.md: MOPS in units of 512 FLOP), cross-checking the
      algorithmic count bench.py reports.

    python scripts/step_pmc.py DIR [DIR ...] --out profiles/step_mfma.json [--simds 1024]
"""
import argparse
import collections
import csv
import glob
import json
import os
import sys


def rows(d):
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            yield from csv.DictReader(fh)


def get(r, *names):
    for n in names:
        if n in r and r[n] != "":
            return r[n]
    raise KeyError(names)


def classify(name):
    if "attn_fwd" in name or "attn16_fwd" in name:
        return "attention"
    if "gemm" in name:
        return "gemm"
    if "norm" in name or "resid_add_ln" in name:
        return "norm"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--out", required=True)
    ap.add_argument("--simds", type=int, default=1024)  # 256 CUs x 4 SIMDs
    a = ap.parse_args()
    tot = collections.defaultdict(float)
    per_cls = collections.defaultdict(lambda: collections.defaultdict(float))
    for d in a.dirs:
        disp = collections.defaultdict(dict)  # dispatch -> counter -> value
        names = {}
        for r in rows(d):
            k = int(float(get(r, "Dispatch_Id", "dispatch_id", "Correlation_Id", "correlation_id")))
            c = get(r, "Counter_Name", "counter_name")
            disp[k][c] = disp[k].get(c, 0.0) + float(get(r, "Counter_Value", "counter_value"))
            names[k] = get(r, "Kernel_Name", "kernel_name")
        ids = sorted(disp)
        # the timed step = the last forward pass: from the last im2col (patch-embed)
        # dispatch on (the warmup pass before it also carries the one-time weight
        # packing copies, so a plain half split would not isolate it)
        marks = [k for k in ids if "im2col" in names[k]]
        step = [k for k in ids if k >= marks[-1]] if marks else ids[len(ids) // 2:]
        for k in step:
            cls = classify(names[k])
            for c, v in disp[k].items():
                key = c if c != "GRBM_GUI_ACTIVE" else f"GRBM_GUI_ACTIVE@{os.path.basename(d.rstrip('/'))}"
                tot[key] += v
                per_cls[cls][key] += v
    out = {"simds": a.simds, "dispatches_per_step": None, "counters": dict(tot)}

    def frac(src, pas):
        g = src.get(f"GRBM_GUI_ACTIVE@{pas}")
        m = src.get("SQ_VALU_MFMA_BUSY_CYCLES")
        return m / (a.simds * g / 8) if g and m is not None else None

    passes = sorted({k.split("@")[1] for k in tot if k.startswith("GRBM_GUI_ACTIVE@")})
    busy_pass = next((p for p in passes if "busy" in p), passes[0] if passes else None)
    out["mfma_busy_frac"] = frac(tot, busy_pass)
    out["mfma_busy_frac_by_class"] = {c: frac(v, busy_pass) for c, v in per_cls.items()}
    if "SQ_INSTS_VALU_MFMA_MOPS_BF16" in tot:
        out["mfma_bf16_tflop_counted"] = tot["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512 / 1e12
    if busy_pass:
        g = tot[f"GRBM_GUI_ACTIVE@{busy_pass}"] / 8
        out["kernel_cycles_per_xcd"] = g
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "large-scale-vit-slam_amd"))
    from aligned_vggt.provenance import stamp
    out.update(stamp())
    print(json.dumps(out, indent=1))
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
