#!/usr/bin/env python3
"""A/B of the 8-wave attention schedules on the global-attention shape
(1 x 16 heads x 21,984 x 21,984 x 64): lockstep variant 33 against the
staggered variants 289-291, interleaved rounds, HIP events over R launches.

    python scripts/attn_stag_bench.py [--reps 20] [--rounds 3] [--variants 33,289,290,291]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "large-scale-vit-slam_amd"))

import torch  # noqa: E402

from aligned_vggt import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="33,289,290,291")
    ap.add_argument("--n", type=int, default=16 * 1374)
    ap.add_argument("--heads", type=int, default=16)
    a = ap.parse_args()
    n, H, D = a.n, a.heads, 64
    C = H * D
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(n, 3 * C, device="cuda", generator=g).to(torch.bfloat16)
    o = torch.empty(n, C, device="cuda", dtype=torch.bfloat16)
    flops = 4.0 * n * n * D * H
    N.tune(N.TUNE_ATTN_WAVES, 8)
    res = {}
    for r in range(a.rounds):
        for var in [int(x) for x in a.variants.split(",")]:
            N.tune(N.TUNE_ATTN_VARIANT, var)
            run = lambda: N.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, 1, H, n, n, D, n, n, n)  # noqa: E731
            run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / a.reps * 1e3
            res.setdefault(var, []).append(round(us, 1))
            print(f"round {r} variant {var}: {us:.1f} us  {flops / us / 1e6:.0f} TF/s  frac {flops / us / 1e6 / 2500:.3f}",
                  flush=True)
    print(json.dumps({"shape": [1, H, n, n, D], "us": res}))


if __name__ == "__main__":
    main()
