#!/usr/bin/env python3
"""Op counts of one continuation chunk's align_chunk (alignment head +
Sim(3)/SE(3) composition) at the 154x518 sequence shape: which torch ops
make up the per-chunk glue launches."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "large-scale-vit-slam_amd"))

import torch  # noqa: E402


def main():
    from aligned_vggt.models.featureAligned_vggt import FeatureAlignedVGGT
    from aligned_vggt.utils.synthetic import condition_pose_outputs_, synthetic_images, synthetic_init_
    dev = torch.device("cuda:0")
    m = FeatureAlignedVGGT(enable_point=False, enable_track=False, num_memory_tokens=8).to(dev).eval()
    synthetic_init_(m, seed=0)
    condition_pose_outputs_(m)
    imgs = synthetic_images(1, 28, 154, 518, seed=1, device=dev)
    with torch.no_grad():
        e1 = m.encode_chunk(imgs[:, :16])
        e2 = m.encode_chunk(imgs[:, 12:28])
        ctx = m.align_chunk(e1, 4, None)
        for _ in range(2):
            c = {k: (list(v) if isinstance(v, list) else v) for k, v in ctx.items()}
            m.align_chunk(e2, 4, c)
        torch.cuda.synchronize()
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            c = {k: (list(v) if isinstance(v, list) else v) for k, v in ctx.items()}
            m.align_chunk(e2, 4, c)
            torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="count", row_limit=40), flush=True)
    print(prof.key_averages(group_by_stack_n=0).table(sort_by="self_cpu_time_total", row_limit=15), flush=True)


if __name__ == "__main__":
    main()
