#!/usr/bin/env python3
"""Time one continuation chunk's align_chunk (the ring's recurrent step) alone
at the configs[3] shape (16 x 154 x 518, overlap 4, 8 memory tokens): HIP
events per call, then --reps calls for a rocprofv3 --kernel-trace summary
(kernels per call = dispatches / reps).  Prints one JSON line."""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "large-scale-vit-slam_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--height", type=int, default=154)
    args = ap.parse_args()
    from aligned_vggt.models.featureAligned_vggt import FeatureAlignedVGGT
    from aligned_vggt.utils.synthetic import condition_pose_outputs_, synthetic_images, synthetic_init_
    dev = torch.device("cuda:0")
    m = FeatureAlignedVGGT(enable_point=False, enable_track=False, num_memory_tokens=8)
    synthetic_init_(m, seed=0)
    condition_pose_outputs_(m)
    m = m.to(dev).eval()
    imgs = synthetic_images(1, 28, args.height, 518, seed=1, device=dev)
    with torch.no_grad():
        e1 = m.encode_chunk(imgs[:, :16], dense=False)
        e2 = m.encode_chunk(imgs[:, 12:28], dense=False)
        ctx = m.align_chunk(e1, 4, None)

        def one():
            c = {k: (list(v) if isinstance(v, list) else v) for k, v in ctx.items()}
            return m.align_chunk(e2, 4, c)

        for _ in range(3):
            one()
        torch.cuda.synchronize()
        ts = []
        s = torch.cuda.current_stream()
        for _ in range(args.reps):
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record(s)
            one()
            b.record(s)
            b.synchronize()
            ts.append(a.elapsed_time(b))
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            for _ in range(10):
                one()
            torch.cuda.synchronize()
    rows = []
    for e in prof.key_averages():
        t = getattr(e, "device_time_total", None)
        if t is None:
            t = e.cuda_time_total
        if t > 0:
            rows.append((t / 10.0, e.count / 10.0, e.key))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows)
    print(f"| kernel | per call | us per call | share |\n|---|---|---|---|")
    for t, n, k in rows[:40]:
        print(f"| {k[:90]} | {n:g} | {t:.1f} | {100 * t / tot:.1f}% |")
    print(f"\nkernel time per call {tot / 1e3:.3f} ms over {sum(r[1] for r in rows):g} launches")
    print(json.dumps({"t_align_ms_median": round(statistics.median(ts), 3), "t_align_ms_min": round(min(ts), 3),
                      "t_align_ms_max": round(max(ts), 3), "reps": args.reps,
                      "kernel_ms_per_call": round(tot / 1e3, 3),
                      "launches_per_call": sum(r[1] for r in rows),
                      "shape": [16, args.height, 518]}), flush=True)


if __name__ == "__main__":
    main()
