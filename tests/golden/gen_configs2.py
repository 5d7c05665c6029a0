"""Oracle outputs at BASELINE configs[2]'s size, committed as fixtures so the
GPU test (tests/test_gpu_fullsize.py) compares against them without spending
minutes of the GPU box's CPU on the oracle.

  * ``configs2_seq.npz``: FeatureAlignedVGGT with a reduced-depth aggregator
    (depth 4, DINOv2 depth 1, kept layers 0-3), memory 8, depth head on, 28
    synthetic 518x518 frames, chunk 16 / overlap 4 (two chunks: frames 0-15
    and 12-27), through the oracle's chunk loop (featureAligned_vggt.py:48-225)
    in the bf16-mixed tier and in fp32;
  * ``configs2_head.npz``: the AlignmentHead alone at P = 1374 (518^2 frames,
    1375 tokens per frame inside the head) on seeded N(0, 1) tokens, a first
    chunk and a continuation chunk (overlap tokens + memory), both tiers
    (alignment_head.py:224-345, cross_attention.py:47-78).

Weights come from ``synthetic_init_`` (per-name seeded CPU generators) and the
inputs from seeded CPU generators, so the GPU test rebuilds them exactly; only
outputs are stored (large maps strided: depth every 7th pixel, overlap tokens
every 25th token).  The oracle is this repository's own CPU restatement
(oracle/vggt_oracle.py), i.e. the same computation the GPU tests otherwise run
on the box.  Usage: python tests/golden/gen_configs2.py [--threads N]"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "large-scale-vit-slam_amd"))
sys.path.insert(0, ROOT)

# shared with the test
SEQ = dict(N=28, w=16, ov=4, H=518, W=518, seed_w=17, seed_img=41, depth=4, dino_depth=1)
HEAD = dict(S=16, H=518, W=518, ov=4, seed_w=23, seed_tok=5)
DEPTH_STRIDE = 7
TOK_STRIDE = 25


def seq_model():
    from aligned_vggt.backbone.aggregator import Aggregator
    from aligned_vggt.models import featureAligned_vggt as FAmod
    from aligned_vggt.models.featureAligned_vggt import FeatureAlignedVGGT
    from aligned_vggt.utils.synthetic import condition_pose_outputs_, synthetic_init_
    orig = FAmod.Aggregator
    FAmod.Aggregator = lambda **kw: Aggregator(depth=SEQ["depth"], dino_depth=SEQ["dino_depth"], **kw)
    try:
        m = FeatureAlignedVGGT(enable_point=False, enable_track=False, num_memory_tokens=8)
    finally:
        FAmod.Aggregator = orig
    m.intermediate_layer_indices = [0, 1, 2, 3]
    synthetic_init_(m, seed=SEQ["seed_w"])
    condition_pose_outputs_(m)
    return m


def seq_images():
    from aligned_vggt.utils.synthetic import synthetic_images
    return synthetic_images(1, SEQ["N"], SEQ["H"], SEQ["W"], seed=SEQ["seed_img"])


def head_model():
    from aligned_vggt.heads.alignment_head import AlignmentHead
    from aligned_vggt.utils.synthetic import synthetic_init_
    h = AlignmentHead(in_dim=2048, num_memory_tokens=8)
    synthetic_init_(h, seed=HEAD["seed_w"])
    for dec in (h.chunk_sim3_decoder, h.frame_se3_decoder):  # condition_pose_outputs_ on the bare head
        with torch.no_grad():
            dec.fc2.bias.zero_()
            dec.fc2.bias[6] = 1.0
    return h


def head_inputs():
    S, P = HEAD["S"], 5 + (HEAD["H"] // 14) * (HEAD["W"] // 14)
    g = torch.Generator().manual_seed(HEAD["seed_tok"])
    tok0 = torch.randn(1, S, P, 2048, generator=g)
    tok1 = torch.randn(1, S, P, 2048, generator=g)
    return tok0, tok1


def merged(ctx, ov, key):
    return torch.cat([p[:, (ov if i else 0):] for i, p in enumerate(ctx[key])], 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--only", choices=["seq", "head"], default=None)
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    from oracle import vggt_oracle as O
    if args.only in (None, "head"):
        h = head_model()
        sd = {"alignment_head." + k: v.detach().clone() for k, v in h.state_dict().items()}
        tok0, tok1 = head_inputs()
        out = {}
        for tier, bf16 in (("bf16", True), ("fp32", False)):
            t0 = time.time()
            with torch.no_grad():
                cs0, fs0, m0, o0 = O.alignment_head(sd, tok0, (HEAD["H"], HEAD["W"]), HEAD["ov"], None, None, bf16=bf16)
                cs1, fs1, m1, o1 = O.alignment_head(sd, tok1, (HEAD["H"], HEAD["W"]), HEAD["ov"], o0, m0, bf16=bf16)
            for k, v in (("cs0", cs0), ("fs0", fs0), ("mem0", m0), ("cs1", cs1), ("fs1", fs1), ("mem1", m1)):
                out[f"{tier}_{k}"] = v.numpy()
            out[f"{tier}_ov0"] = o0[:, :, ::TOK_STRIDE].contiguous().numpy()
            out[f"{tier}_ov1"] = o1[:, :, ::TOK_STRIDE].contiguous().numpy()
            print(f"head {tier}: {time.time() - t0:.1f} s", flush=True)
        np.savez_compressed(os.path.join(HERE, "configs2_head.npz"), **out)
    if args.only in (None, "seq"):
        m = seq_model()
        sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
        imgs = seq_images()
        chunks = O.generate_chunks(SEQ["N"], SEQ["w"], SEQ["ov"])
        assert [len(c) for c in chunks] == [16, 16]
        agg_kw = {"keep": (0, 1, 2, 3), "depth": SEQ["depth"], "dino_depth": SEQ["dino_depth"]}
        out = {}
        for tier, bf16 in (("bf16", True), ("fp32", False)):
            t0 = time.time()
            ctx = None
            with torch.no_grad():
                for ids in chunks:
                    ctx = O.feature_aligned_forward(sd, imgs[:, ids], SEQ["ov"], ctx, bf16=bf16, agg_kwargs=agg_kw)
                    print(f"  chunk {ids[0]}-{ids[-1]} {tier}: {time.time() - t0:.1f} s", flush=True)
            ov = SEQ["ov"]
            out[f"{tier}_chunk_sim3"] = ctx["chunk_sim3_alignment_enc"].numpy()
            out[f"{tier}_frame_se3"] = ctx["frame_se3_alignment_enc"].numpy()
            out[f"{tier}_pose_enc"] = merged(ctx, ov, "pose_enc").numpy()
            out[f"{tier}_depth"] = merged(ctx, ov, "depth")[:, :, ::DEPTH_STRIDE, ::DEPTH_STRIDE].contiguous().numpy()
            out[f"{tier}_depth_conf"] = merged(ctx, ov, "depth_conf")[:, :, ::DEPTH_STRIDE,
                                                                      ::DEPTH_STRIDE].contiguous().numpy()
            out[f"{tier}_memory"] = torch.stack(ctx["memory_tokens"]).numpy()
            out[f"{tier}_overlap"] = ctx["overlap_tokens"][:, :, ::TOK_STRIDE].contiguous().numpy()
        np.savez_compressed(os.path.join(HERE, "configs2_seq.npz"), **out)


if __name__ == "__main__":
    main()
