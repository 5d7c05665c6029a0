#!/usr/bin/env python3
"""Golden fixture for the headline config at full depth and full size
(BASELINE configs[1]: one 16-frame 518x518 chunk through the whole VGGT
aggregator -- DINOv2 ViT-L/14 x 24 + 24 frame / 24 global blocks -- layers
4/11/17/23 kept, featureAligned_vggt.py:24, :78-82).

TEST INFRASTRUCTURE: runs the CPU oracle (``oracle/vggt_oracle.aggregator``)
twice on the same input -- ``bf16=True`` (the reference's bf16-mixed autocast
rounding points) and ``bf16=False`` (plain fp32) -- and stores a strided
subsample of every kept layer of both tiers in ``tests/golden/configs1_full.npz``:

  weights  ``synthetic_init_(Aggregator(), seed=0)`` (per-name CPU generators:
           identical on any host)
  images   ``synthetic_images(1, 16, 518, 518, seed=1234)``
  sample   frames (0, 8, 15) x every 11th token x every 4th channel of the
           (1, 16, 1374, 2048) outputs, fp32 -> (4, 3, 125, 512) per tier

Resumable: each tier's full kept layers are written to ``--work`` (default
``scratch/configs1_full``) when it finishes and reused on the next call, so a
killed run only repeats the unfinished tier.  One tier takes ~15-25 min on 8
cores.  ``tests/test_gpu_fullsize.py::test_aggregator_headline_chunk_full_depth``
compares the HIP ``Aggregator()`` on the GPU against this fixture.

  python tests/golden/gen_configs1_full.py [--threads N] [--work DIR]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "large-scale-vit-slam_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

FRAMES = (0, 8, 15)
TOKEN_STRIDE = 11
CHANNEL_STRIDE = 4
KEEP = (4, 11, 17, 23)
WEIGHT_SEED = 0
IMAGE_SEED = 1234


def subsample(x: torch.Tensor) -> np.ndarray:
    """(1, 16, 1374, 2048) -> (3, 125, 512) fp32."""
    return x[0, list(FRAMES), ::TOKEN_STRIDE, ::CHANNEL_STRIDE].float().numpy().copy()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--work", default=os.path.join(ROOT, "scratch", "configs1_full"))
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden", "configs1_full.npz"))
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    os.makedirs(a.work, exist_ok=True)

    from oracle import vggt_oracle as O
    from aligned_vggt.backbone.aggregator import Aggregator
    from aligned_vggt.utils.synthetic import synthetic_images, synthetic_init_

    agg = Aggregator()
    synthetic_init_(agg, seed=WEIGHT_SEED)
    sd = {"aggregator." + k: v.detach() for k, v in agg.state_dict().items()}
    del agg
    img = synthetic_images(1, 16, 518, 518, seed=IMAGE_SEED)

    timings = {}
    samples = {}
    for tier, bf16 in (("bf16", True), ("fp32", False)):
        path = os.path.join(a.work, f"{tier}.pt")
        if os.path.exists(path):
            saved = torch.load(path, weights_only=True)  # our own file
            outs, timings[tier] = saved["outs"], float(saved["seconds"])
            print(f"{tier}: reusing {path}", flush=True)
        else:
            t0 = time.perf_counter()
            with torch.no_grad():
                outs, psi = O.aggregator(sd, img, bf16=bf16, keep=KEEP)
            assert psi == 5
            timings[tier] = time.perf_counter() - t0
            torch.save({"outs": outs, "seconds": timings[tier]}, path)
            print(f"{tier}: {timings[tier]:.1f} s at {a.threads} threads", flush=True)
        assert len(outs) == len(KEEP) and all(o.shape == (1, 16, 1374, 2048) for o in outs)
        samples[tier] = np.stack([subsample(o) for o in outs])
        # full-tensor spread is recorded too: the test's bars use the subsample's, this shows it is representative
        samples[tier + "_full_norm"] = np.array([o.float().norm().item() for o in outs], np.float64)
        if tier == "fp32":
            full_bf16 = torch.load(os.path.join(a.work, "bf16.pt"), weights_only=True)["outs"]
            samples["spread_full"] = np.array(
                [((b - f).norm() / f.norm()).item() for b, f in zip(full_bf16, outs)], np.float64)

    spread_sample = np.array([np.linalg.norm(b - f) / np.linalg.norm(f)
                              for b, f in zip(samples["bf16"], samples["fp32"])])
    np.savez(a.out, bf16=samples["bf16"], fp32=samples["fp32"], keep=np.array(KEEP), frames=np.array(FRAMES),
             token_stride=TOKEN_STRIDE, channel_stride=CHANNEL_STRIDE, weight_seed=WEIGHT_SEED,
             image_seed=IMAGE_SEED, spread_sample=spread_sample, spread_full=samples["spread_full"],
             seconds=np.array([timings["bf16"], timings["fp32"]]), threads=a.threads)
    print("bf16-vs-fp32 spread per kept layer (sample):", spread_sample)
    print("bf16-vs-fp32 spread per kept layer (full):  ", samples["spread_full"])
    print("wrote", a.out, os.path.getsize(a.out), "bytes")


if __name__ == "__main__":
    main()
