#!/usr/bin/env python3
"""List the torch copy / fill ops of one steady-state per-chunk
FeatureAlignedVGGT forward (torch.profiler with Python stacks), grouped by the
aligned_vggt frame that issued them, so the blit kernels
(__amd_rocclr_copyBuffer / fillBuffer) in the chunk's kernel table can be
traced to their call sites.  Usage: python scripts/copy_probe.py [--frames 16]"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "large-scale-vit-slam_amd"))
import torch  # noqa: E402

from aligned_vggt.models.featureAligned_vggt import FeatureAlignedVGGT  # noqa: E402
from aligned_vggt.utils.synthetic import condition_pose_outputs_, synthetic_images, synthetic_init_  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=16)
ap.add_argument("--height", type=int, default=518)
args = ap.parse_args()
dev = torch.device("cuda:0")
model = FeatureAlignedVGGT(enable_point=False, enable_track=False, num_memory_tokens=8).to(dev).eval()
synthetic_init_(model, seed=0)
condition_pose_outputs_(model)
imgs = synthetic_images(1, args.frames, args.height, 518, seed=1234, device=dev)
ctx = None
for _ in range(2):
    ctx = model(imgs, 4, ctx)
torch.cuda.synchronize()
OPS = ("aten::copy_", "aten::fill_", "aten::zero_", "aten::cat", "aten::index", "aten::index_put_",
       "aten::nonzero", "aten::masked_select")
with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU], with_stack=True,
                            record_shapes=True) as prof:
    ctx = model(imgs, 4, ctx)
    torch.cuda.synchronize()
sites = collections.Counter()
shapes = {}
for ev in prof.events():
    if ev.name not in OPS:
        continue
    st = [s for s in (ev.stack or []) if "aligned_vggt" in s]
    key = " <- ".join(s.split("aligned_vggt/")[-1] for s in st[:3]) or "(no aligned_vggt frame)"
    sites[(ev.name, key)] += 1
    shapes.setdefault((ev.name, key), str(ev.input_shapes)[:80])
print(f"{sum(sites.values())} copy/fill/cat ops in one chunk forward")
for (name, key), n in sites.most_common(60):
    print(f"{n:4d}  {name:18s} {key}  {shapes[(name, key)]}")
