"""A/B of DPT head variants in one process (interleaved rounds): the depth
head on one 16-frame 518^2 chunk of synthetic kept-layer tokens.

    python scripts/dpt_ab.py [--rounds R] [--frames S]
Variants: module attributes of aligned_vggt.backbone.dpt_head toggled between
rounds (REORDER_OUT_CONV, FUSE_UPSAMPLE_CONV when present).
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "large-scale-vit-slam_amd"))
from aligned_vggt.backbone import dpt_head as D  # noqa: E402
from aligned_vggt.utils.synthetic import synthetic_init_  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    head = D.DPTHead(dim_in=2048, output_dim=2, activation="exp", conf_activation="expp1",
                     intermediate_layer_idx=range(4))
    synthetic_init_(head, seed=1)
    head = head.to(dev).eval()
    S, H, W = a.frames, 518, 518
    P = 5 + 37 * 37
    g = torch.Generator(device=dev).manual_seed(0)
    toks = [torch.randn(1, S, P, 2048, device=dev, generator=g) for _ in range(4)]
    imgs = torch.rand(1, S, 3, H, W, device=dev, generator=g)
    variants = {"reference_order": {"REORDER_OUT_CONV": False, "SEPARABLE_POS": False},
                "reordered": {"REORDER_OUT_CONV": True, "SEPARABLE_POS": False},
                "reordered+sep_pos": {"REORDER_OUT_CONV": True, "SEPARABLE_POS": True}}
    if hasattr(D, "FUSE_UPSAMPLE_CONV"):
        variants["reordered+sep_pos+fused_up"] = {"REORDER_OUT_CONV": True, "SEPARABLE_POS": True,
                                                  "FUSE_UPSAMPLE_CONV": True}
        for v in variants.values():
            v.setdefault("FUSE_UPSAMPLE_CONV", False)
    outs, times = {}, {k: [] for k in variants}
    for r in range(a.rounds):
        for name, attrs in variants.items():
            for k, v in attrs.items():
                setattr(D, k, v)
            head(toks, images=imgs, patch_start_idx=5)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                o = head(toks, images=imgs, patch_start_idx=5)
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / a.reps)
            outs[name] = [t.clone() for t in o]
    ref = outs["reference_order"]
    for name in variants:
        errs = [((x - y).norm() / y.norm()).item() for x, y in zip(outs[name], ref)]
        print(f"{name}: median {statistics.median(times[name]):.3f} ms  min {min(times[name]):.3f} ms  "
              f"rel-L2 vs reference order depth {errs[0]:.2e} conf {errs[1]:.2e}", flush=True)


if __name__ == "__main__":
    main()
