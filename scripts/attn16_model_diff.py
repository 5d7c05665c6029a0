"""Forward differences of the small FeatureAlignedVGGT of tests/test_gpu_train.py
(42x56, S=3, two chunks) between the 32x32x16 and 16x16x32 attention forms,
next to the oracle's own bf16-vs-fp32 spread."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "large-scale-vit-slam_amd"))
sys.path.insert(0, ROOT)
from aligned_vggt import _native as N  # noqa: E402
from aligned_vggt.models.featureAligned_vggt import FeatureAlignedVGGT  # noqa: E402
from aligned_vggt.utils.synthetic import condition_pose_outputs_, synthetic_images, synthetic_init_  # noqa: E402
from oracle import vggt_oracle as O  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def main():
    m = FeatureAlignedVGGT(enable_point=False, enable_track=False, num_memory_tokens=8)
    synthetic_init_(m, seed=11)
    condition_pose_outputs_(m)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.cuda().eval()
    S, ov, H, W = 3, 1, 42, 56
    imgs = synthetic_images(1, 2 * S - ov, H, W, seed=5)
    chunks = O.generate_chunks(imgs.shape[1], S, ov)
    outs = {}
    for f in (0, 1):
        N.tune(N.TUNE_ATTN16, f)
        ctx = None
        with torch.no_grad():
            for ids in chunks:
                ctx = m(imgs[:, ids].cuda(), ov, ctx)
            agg, _ = m.aggregator(imgs[:, chunks[0]].cuda())
        outs[f] = (ctx, agg)
    refs = {}
    for tag, bf in (("bf", True), ("32", False)):
        rc = None
        with torch.no_grad():
            for ids in chunks:
                rc = O.feature_aligned_forward(sd, imgs[:, ids], ov, rc, bf16=bf)
        refs[tag] = rc
    a0, a1 = outs[0][1], outs[1][1]
    for i in (0, len(a0) // 2, len(a0) - 1):
        print(f"aggregator layer {i}: rel(16 vs 32) {rel(a1[i], a0[i]):.3e}")
    for k in ("chunk_sim3_alignment_enc", "frame_se3_alignment_enc"):
        print(f"{k}: rel(16 vs 32) {rel(outs[1][0][k], outs[0][0][k]):.3e}  rel(32 vs oracle bf16) "
              f"{rel(outs[0][0][k], refs['bf'][k]):.3e}  rel(16 vs oracle bf16) {rel(outs[1][0][k], refs['bf'][k]):.3e}  "
              f"oracle bf16 vs fp32 {rel(refs['bf'][k], refs['32'][k]):.3e}")
    for k in ("pose_enc", "depth"):
        for c in range(len(chunks)):
            print(f"{k}[{c}]: rel(16 vs 32) {rel(outs[1][0][k][c], outs[0][0][k][c]):.3e}  rel(32 vs bf16 oracle) "
                  f"{rel(outs[0][0][k][c], refs['bf'][k][c]):.3e}  rel(16 vs bf16 oracle) "
                  f"{rel(outs[1][0][k][c], refs['bf'][k][c]):.3e}  oracle bf16 vs fp32 "
                  f"{rel(refs['bf'][k][c], refs['32'][k][c]):.3e}")


if __name__ == "__main__":
    main()
