#!/usr/bin/env python3
"""Run-to-run determinism of the HIP path: the same small sequence through
apply_sequence_to_model three times (the third after a differently-sized
forward has re-used the workspaces) must give bitwise-identical outputs."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "large-scale-vit-slam_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from aligned_vggt.dist.pipeline import apply_sequence_to_model  # noqa: E402
from aligned_vggt.models.featureAligned_vggt import FeatureAlignedVGGT  # noqa: E402
from aligned_vggt.utils.synthetic import condition_pose_outputs_, synthetic_images, synthetic_init_  # noqa: E402
from tests.test_gpu_model import _synthetic_w2c  # noqa: E402

m = FeatureAlignedVGGT(enable_point=True, enable_track=False, num_memory_tokens=8)
synthetic_init_(m, seed=11)
condition_pose_outputs_(m)
m = m.cuda().eval()
S, w, ov, H, W = 7, 4, 2, 42, 56
imgs = synthetic_images(1, S, H, W, seed=12).cuda()
batch = {"images": imgs, "extrinsics": _synthetic_w2c(S).cuda()}


def run():
    out = apply_sequence_to_model(batch, m, [w], [ov], "chunk_overlap", "scale_from_poses")
    return {k: (v.detach().cpu().clone() if isinstance(v, torch.Tensor) else v) for k, v in out.items()}


a = run()
b = run()
with torch.no_grad():
    m(synthetic_images(1, 6, 70, 84, seed=3).cuda(), 2, None)  # dirty the workspaces
c = run()
for k, v in a.items():
    if isinstance(v, torch.Tensor):
        print(f"{k:28s} a==b {torch.equal(v, b[k])}  a==c {torch.equal(v, c[k])}  "
              f"max|a-c| {(v.float() - c[k].float()).abs().max().item():.3e}")
