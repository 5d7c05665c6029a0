#!/usr/bin/env python3
"""BASELINE.md §3 row C3 on the host cores: one 64-frame synthetic 518^2
sequence, chunk 16 / overlap 4 (5 chunks), through the oracle's FULL
FeatureAlignedVGGT (aggregator 24 + 24 + DINOv2 24, camera head, depth DPT
head, alignment head with memory 8, Sim(3) composition; featureAligned_vggt.py:
48-225 chained through ``context`` as training_metrics.py:643-652 does), fp32
(the reference's numerics), random-init weights.

A whole sequence takes longer than one GPU-box call may run, so the run is
resumable: after every chunk the state (chunk times so far + the context the
next chunk needs: overlap tokens, memory, the last pose encoding, the merged
Sim(3) / SE(3) lists) is saved to --state, and a later call continues from it
(each call does its own reduced-depth warm-up first).  When the last chunk is
done the row "C3_t<threads>" (per-chunk seconds, the sequence total, chunks/s)
is merged into --out.

  python scripts/cpu_baseline_c3.py --threads 16 --state gpurun_out/c3cpu/state.pt \
      --out gpurun_out/c3cpu/cpu_baseline_full.json [--max-seconds 1000]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "large-scale-vit-slam_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

SEQ, W, OV = 64, 16, 4
KEEP_CTX = ("overlap_tokens", "chunk_sim3_alignment_enc", "frame_se3_alignment_enc")


def _heartbeat(state):
    while not state["done"]:
        time.sleep(60)
        if not state["done"]:
            print(f"[c3cpu] chunk {state['chunk']} running {time.time() - state['t0']:.0f} s", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--state", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--max-seconds", type=float, default=1e9, help="start no chunk after this many seconds")
    ap.add_argument("--chunk-estimate", type=float, default=600.0)
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    from oracle import vggt_oracle as O
    from aligned_vggt.models.featureAligned_vggt import FeatureAlignedVGGT
    from aligned_vggt.utils.synthetic import condition_pose_outputs_, synthetic_images, synthetic_init_
    t_start = time.time()
    m = FeatureAlignedVGGT(enable_point=False, enable_track=False, num_memory_tokens=8)
    synthetic_init_(m, seed=0)
    condition_pose_outputs_(m)
    sd = {k: v.detach() for k, v in m.state_dict().items()}
    del m
    imgs = synthetic_images(1, SEQ, 518, 518, seed=1234)
    chunks = O.generate_chunks(SEQ, W, OV)
    assert len(chunks) == 5
    st = {"next": 0, "chunk_s": [], "ctx": None}
    if os.path.exists(a.state):
        st = torch.load(a.state, weights_only=True)  # written by this script
    print(f"[c3cpu] resume at chunk {st['next']} with {st['chunk_s']}", flush=True)
    with torch.no_grad():  # warm-up: reduced depth, 2 frames
        t0 = time.time()
        O.feature_aligned_forward(sd, imgs[:, :2], 1, None, agg_kwargs={"keep": (0, 1, 2, 3), "depth": 4,
                                                                      "dino_depth": 1})
        warm = time.time() - t0
    hb = {"done": False, "chunk": st["next"], "t0": time.time()}
    threading.Thread(target=_heartbeat, args=(hb,), daemon=True).start()
    while st["next"] < len(chunks):
        if time.time() - t_start + a.chunk_estimate > a.max_seconds:
            print(f"[c3cpu] stopping before chunk {st['next']} (budget)", flush=True)
            break
        i = st["next"]
        ctx = st["ctx"]
        hb["chunk"], hb["t0"] = i, time.time()
        t0 = time.perf_counter()
        with torch.no_grad():
            out = O.feature_aligned_forward(sd, imgs[:, chunks[i]], OV, ctx, bf16=False)
        dt = time.perf_counter() - t0
        st["chunk_s"].append(round(dt, 2))
        st["next"] = i + 1
        # what the next chunk reads (featureAligned_vggt.py:84-94, :122-137): the rest of the
        # per-chunk lists (depth maps, images) is output, not recurrence state
        nxt = {k: out[k] for k in KEEP_CTX}
        nxt["memory_tokens"] = [out["memory_tokens"][-1]]
        nxt["pose_enc"] = [out["pose_enc"][-1]]
        st["ctx"] = nxt
        os.makedirs(os.path.dirname(os.path.abspath(a.state)), exist_ok=True)
        torch.save(st, a.state)
        print(f"[c3cpu] chunk {i}: {dt:.1f} s (warm-up {warm:.1f} s)", flush=True)
    hb["done"] = True
    if st["next"] == len(chunks):
        total = sum(st["chunk_s"])
        try:
            with open(a.out) as fh:
                full = json.load(fh)
        except (OSError, ValueError):
            full = {"rows": {}}
        full.setdefault("rows", {})[f"C3_t{a.threads}"] = {
            "row": "C3", "threads": a.threads,
            "workload": "FeatureAlignedVGGT full (aggregator + camera + depth DPT + alignment head, memory 8), "
                        "64 x 518^2 frames, chunk 16 / overlap 4 = 5 chunks, fp32 oracle",
            "chunk_s": st["chunk_s"], "sequence_s": round(total, 2), "chunks_per_s": round(5 / total, 6),
            "procedure": "one whole sequence, chunks timed one after another (resumable across calls: the "
                         "context the next chunk reads is saved after each chunk; each call warms up first)"}
        with open(a.out, "w") as fh:
            json.dump(full, fh, indent=1)
        print(f"[c3cpu] sequence {total:.1f} s -> {5 / total:.5f} chunks/s", flush=True)


if __name__ == "__main__":
    main()
