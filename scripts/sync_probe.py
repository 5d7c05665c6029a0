#!/usr/bin/env python3
"""List the host-synchronising torch calls of one steady-state per-chunk
FeatureAlignedVGGT forward (torch.cuda.set_sync_debug_mode('warn')), with the
Python frame inside aligned_vggt that issued each, so the per-chunk glue can
be kept asynchronous.  Usage: python scripts/sync_probe.py [--frames 16]"""
import argparse
import collections
import os
import sys
import traceback
import warnings

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
sites = collections.Counter()


def show(message, category, filename, lineno, file=None, line=None):
    st = [f for f in traceback.extract_stack() if "aligned_vggt" in f.filename]
    key = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}" for f in reversed(st[-3:]))
    if "prototype feature" in str(message):  # the mode's own notice, not a sync
        return
    sites[(str(message)[:60], key)] += 1


warnings.showwarning = show
warnings.simplefilter("always")
torch.cuda.set_sync_debug_mode("warn")
ctx = model(imgs, 4, ctx)
torch.cuda.set_sync_debug_mode(0)
torch.cuda.synchronize()
print(f"{sum(sites.values())} synchronising calls in one chunk forward")
for (msg, key), n in sites.most_common():
    print(f"{n:4d}  {msg} | {key}")
