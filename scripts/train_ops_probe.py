#!/usr/bin/env python3
"""Where the alignment-head training step's launches come from: host enqueue
time vs device time per step, and a torch.profiler table of the ops by launch
count (the step of bench.py --workload train).

    python scripts/train_ops_probe.py [--frames 16] [--height 518]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "large-scale-vit-slam_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--height", type=int, default=518)
    ap.add_argument("--rows", type=int, default=45)
    args = ap.parse_args()
    from aligned_vggt.heads.alignment_head import AlignmentHead
    from aligned_vggt.utils.synthetic import synthetic_init_
    dev = torch.device("cuda:0")
    H, W, S, ov = args.height, 518, args.frames, 4
    P = 5 + (H // 14) * (W // 14)
    head = AlignmentHead(in_dim=2048, num_memory_tokens=8).to(dev).train()
    synthetic_init_(head, seed=0)
    opt = torch.optim.AdamW(head.parameters(), lr=5e-5, weight_decay=0.05, fused=True)
    g = torch.Generator(device=dev).manual_seed(1234)
    toks = [torch.randn(1, S, P, 2048, device=dev, generator=g) for _ in range(2)]
    wcs = torch.randn(1, 1, 8, device=dev, generator=g)
    wfs = torch.randn(1, S - 1, 7, device=dev, generator=g)

    def step():
        cs1, fs1, m1, o1 = head(toks[0], (H, W), ov)
        cs2, fs2, m2, _ = head(toks[1], (H, W), ov, overlap_tokens=o1, memory_tokens=m1)
        loss = ((cs1 + cs2) * wcs).sum() + ((fs1 + fs2) * wfs).sum() + m2.square().sum()
        opt.zero_grad(set_to_none=True)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(head.parameters(), 1.0)
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    for _ in range(3):
        t0 = time.perf_counter()
        step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"host enqueue {1e3 * (t1 - t0):.1f} ms, step {1e3 * (t2 - t0):.1f} ms", flush=True)
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        step()
        torch.cuda.synchronize()
    ka = prof.key_averages()
    print(ka.table(sort_by="count", row_limit=args.rows), flush=True)
    print(ka.table(sort_by="self_cpu_time_total", row_limit=25), flush=True)


if __name__ == "__main__":
    main()
