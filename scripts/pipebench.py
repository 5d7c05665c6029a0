#!/usr/bin/env python3
"""A/B of the persistent GEMM's DMA placement (VGGT_TUNE_GEMM_PIPE values) at the
aggregator's shapes, in one process, rounds alternating the order of the values.

    python scripts/pipebench.py [--pipes 0,1,2,3] [--rounds 3] [--reps 40]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "large-scale-vit-slam_amd"))

import torch  # noqa: E402

from aligned_vggt import _native as N  # noqa: E402


def timeit(fn, reps):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pipes", default="0,1,2,3")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--tokens", type=int, default=16 * 1374)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    M = args.tokens
    x = (torch.rand(M, 4096, device=dev) * 2 - 1).bfloat16()
    cases = []
    for name, Nn, K, epi in (("qkv", 3072, 1024, N.EPI_BF16), ("fc1_gelu", 4096, 1024, N.EPI_GELU_BF16),
                             ("fc1", 4096, 1024, N.EPI_BF16), ("fc2", 1024, 4096, N.EPI_BF16),
                             ("proj", 1024, 1024, N.EPI_BF16)):
        a = x[:, :K].contiguous()
        w = ((torch.rand(Nn, K, device=dev) * 2 - 1) * K ** -0.5).bfloat16()
        bias = torch.randn(Nn, device=dev) * 0.1
        o = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
        cases.append((name, 2.0 * M * Nn * K, (lambda a=a, w=w, bias=bias, o=o, epi=epi: N.gemm_bf16(a, w, bias, o, epi)), o))
    # the fused q/k-norm + RoPE-2D qkv GEMM (the half-K main loop)
    H, D = 16, 64
    a = x[:, :1024].contiguous()
    wqkv = ((torch.rand(3 * H * D, 1024, device=dev) * 2 - 1) * 1024 ** -0.5).bfloat16()
    bq = torch.randn(3 * H * D, device=dev) * 0.1
    lw, lb = torch.rand(D, device=dev) + 0.5, torch.randn(D, device=dev) * 0.1
    hw = 37 * 37
    yy, xx = torch.meshgrid(torch.arange(37), torch.arange(37), indexing="ij")
    pos = torch.cat([torch.zeros(5, 2, dtype=torch.long), torch.stack([yy.reshape(-1), xx.reshape(-1)], -1) + 1])
    pos = pos.to(torch.int32).contiguous().to(dev)
    inv = 1.0 / (100.0 ** (torch.arange(0, D // 2, 2).float() / (D // 2)))
    ang = torch.outer(torch.arange(39).float(), inv)
    ang = torch.cat([ang, ang], -1)
    cs, sn = ang.cos().contiguous().to(dev), ang.sin().contiguous().to(dev)
    oq = torch.empty(M, 3 * H * D, device=dev, dtype=torch.bfloat16)
    qkv_fn = lambda: N.gemm_qkv(a, wqkv, bq, oq, H, D, lw, lb, lw, lb, 1e-5, N.ROPE_2D, pos, hw + 5, cs, sn)  # noqa: E731
    cases.append(("qkv_fused", 2.0 * M * 3 * H * D * 1024, qkv_fn))
    pipes = [int(p) for p in args.pipes.split(",")]
    # correctness: every pipe value gives the same bits as pipe 0
    ref = {}
    for p in pipes:
        N.tune(N.TUNE_GEMM_PIPE, p)
        for c in cases:
            name, fn = c[0], c[2]
            o = c[3] if len(c) > 3 else oq
            fn()
            torch.cuda.synchronize()
            if name in ref:
                same = torch.equal(ref[name], o)
                print(f"bitwise pipe {p} {name}: {same}", flush=True)
                if not same:
                    sys.exit(1)
            else:
                ref[name] = o.clone()
    t_end = time.time() + 3.0
    while time.time() < t_end:
        cases[1][2]()
        torch.cuda.synchronize()
    res = {}
    for r in range(args.rounds):
        order = pipes if r % 2 == 0 else pipes[::-1]
        for p in order:
            N.tune(N.TUNE_GEMM_PIPE, p)
            for c in cases:
                us = timeit(c[2], args.reps)
                res.setdefault((c[0], p), []).append(us)
    for name, *_ in cases:
        print(name, "  ".join(f"pipe{p}: " + "/".join(f"{u:.1f}" for u in res[(name, p)]) for p in pipes), flush=True)


if __name__ == "__main__":
    main()
