"""DPT convolution microbench on the default (pre-split) path: the 3x3 convs of
one 16-frame 518^2 chunk's depth head, plus the 296^2 -> 518^2 bilinear
upsample (+ positional table, split output) that feeds output_conv2.

    python scripts/convbench_pre.py [--reps N] [--only NAME]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "large-scale-vit-slam_amd"))
from aligned_vggt import _native as N  # noqa: E402

SHAPES = {"c148": (16, 148, 256, 256), "c296": (16, 296, 256, 128), "c74": (16, 74, 256, 256),
          "c518": (16, 518, 128, 32)}


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for name, (n, hw, ci, co) in SHAPES.items():
        if a.only and a.only not in name:
            continue
        x = torch.randn(n * hw * hw, ci, device=dev, generator=g)
        wp = torch.zeros((co + 127) // 128 * 128, 9 * ci, device=dev)
        wp[:co] = torch.randn(co, 9 * ci, device=dev, generator=g) * 0.02
        whi, wlo = N.split_bf16x2(wp)
        b = torch.zeros(co, device=dev)
        y = torch.empty(n * hw * hw, co, device=dev)
        xs = N.split_act_bf16x2(x)
        fl = 2 * n * hw * hw * co * 9 * ci
        us = timeit(lambda: N.conv2d_bf16x3_pre(xs[0], xs[1], n, hw, hw, ci, whi, wlo, b, co, 3, 3, 1, 1, y), a.reps)
        print(f"{name}: conv3x3 n={n} hw={hw} ci={ci} co={co}: {us:.1f} us  fp32-eq {fl / us / 1e6:.0f} TF/s  "
              f"bf16 MFMA {3 * fl / us / 1e6:.0f} TF/s ({3 * fl / us / 1e6 / 2500 * 100:.1f}% of peak)", flush=True)
    if not a.only or "up" in a.only:
        n, hi, C, ho = 16, 296, 128, 518
        x = torch.randn(n * hi * hi, C, device=dev, generator=g)
        pos = torch.randn(ho * ho, C, device=dev, generator=g)
        ys = (torch.empty(n * ho * ho, C, device=dev, dtype=torch.bfloat16),
              torch.empty(n * ho * ho, C, device=dev, dtype=torch.bfloat16))
        us = timeit(lambda: N.upsample_bilinear_split(x, n, hi, hi, C, None, ho, ho, pos, y_split=ys), a.reps)
        mb = (n * hi * hi * C * 4 + n * ho * ho * C * 4 + ho * ho * C * 4) / 1e6
        print(f"up: upsample 296->518 x{C} (+pos, split out): {us:.1f} us  {mb / us:.2f} TB/s algorithmic "
              f"({mb:.0f} MB)", flush=True)
    if not a.only or "fused" in a.only:
        from aligned_vggt.backbone.dpt_head import pos_table_sep
        n, hi, C, ho, co = 16, 296, 128, 518, 32
        x = torch.randn(n * hi * hi, C, device=dev, generator=g)
        sep = pos_table_sep(C, ho, ho, ho, ho).to(dev)
        wp = torch.zeros(128, 9 * C, device=dev)
        wp[:co] = torch.randn(co, 9 * C, device=dev, generator=g) * 0.02
        whi, wlo = N.split_bf16x2(wp)
        b = torch.zeros(co, device=dev)
        ys = (torch.empty(n * ho * ho, co, device=dev, dtype=torch.bfloat16),
              torch.empty(n * ho * ho, co, device=dev, dtype=torch.bfloat16))
        us = timeit(lambda: N.conv2d_upsample_bf16x3(x, n, hi, hi, C, sep, ho, ho, whi, wlo, b, co, None,
                                                     relu_out=True, y_split=ys), a.reps)
        fl = 2 * n * ho * ho * co * 9 * C
        print(f"fused: upsample 296->518 + conv3x3 {C}->{co}: {us:.1f} us  bf16 MFMA {3 * fl / us / 1e6:.0f} TF/s",
              flush=True)


if __name__ == "__main__":
    main()
