#!/usr/bin/env python3
"""Per-kernel microbenchmark on the aggregator's production shapes (one
16-frame 518x518 chunk: M = 16 x 1374 = 21984 token rows, C = 1024, 16 heads
of 64).  Each kernel is timed with HIP events over R back-to-back launches on
the current stream.  Used to iterate on single kernels between full bench runs.

    python scripts/kbench.py [--reps 20] [--only gemm,norm,attn]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "large-scale-vit-slam_amd"))

import torch  # noqa: E402

from aligned_vggt import _native as N  # noqa: E402
from aligned_vggt.backbone.layers import RopeTables  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="gemm,norm,attn")
    ap.add_argument("--gemm-modes", default="0,1,2")
    ap.add_argument("--attn-waves", default="4,8")
    ap.add_argument("--attn-variants", default="0")
    ap.add_argument("--rounds", type=int, default=1, help="repeat the attention sweep (A/B alternation)")
    ap.add_argument("--warm-s", type=float, default=3.0)
    ap.add_argument("--tokens", type=int, default=16 * 1374,
                    help="token rows M (6592 = the 154x518 sequence chunk, 16 x 412)")
    args = ap.parse_args()
    only = set(args.only.split(","))
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    M, C, H, D = args.tokens, 1024, 16, 64
    res = {}
    if "gemm" in only:
        x = (torch.randn(M, 4096, device=dev) * 0.5).bfloat16()
        # clocks / power to the steady state before the first measured shape
        wq = (torch.randn(3 * C, C, device=dev) * C ** -0.5).bfloat16()
        oq = torch.empty(M, 3 * C, device=dev, dtype=torch.bfloat16)
        t_end = time.time() + args.warm_s
        while time.time() < t_end:
            N.gemm_bf16(x[:, :C], wq, torch.zeros(3 * C, device=dev), oq, N.EPI_BF16)
            torch.cuda.synchronize()
        for mode, (name, Nn, K, epi) in [(md, sh) for md in map(int, args.gemm_modes.split(",")) for sh in (
                ("qkv", 3 * C, C, N.EPI_BF16), ("proj", C, C, N.EPI_RESID_F32), ("fc1", 4 * C, C, N.EPI_GELU_BF16),
                ("fc1_plain", 4 * C, C, N.EPI_BF16), ("fc2", C, 4 * C, N.EPI_RESID_F32),
                ("fc2_plain", C, 4 * C, N.EPI_BF16), ("proj_plain", C, C, N.EPI_BF16))]:
            N.tune(N.TUNE_GEMM_TILE, mode)
            w = (torch.randn(Nn, K, device=dev) * K ** -0.5).bfloat16()
            bias = torch.randn(Nn, device=dev) * 0.1
            a = x[:, :K]
            if epi == N.EPI_RESID_F32:
                out = torch.randn(M, Nn, device=dev)
                gamma = torch.rand(Nn, device=dev)
            else:
                out = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
                gamma = None
            us = timeit(lambda: N.gemm_bf16(a, w, bias, out, epi, gamma=gamma), args.reps)
            res[f"{name}/tile{mode}"] = {"us": round(us, 1), "tflops": round(2 * M * Nn * K / us / 1e6, 1)}
            print(f"{name}/tile{mode}", res[f"{name}/tile{mode}"], flush=True)
            if name == "qkv":  # the production form: q/k LayerNorm + RoPE2D in the epilogue
                yy, xx = torch.meshgrid(torch.arange(37), torch.arange(37), indexing="ij")
                pos = torch.cat([torch.zeros(5, 2, dtype=torch.long),
                                 torch.stack([yy.reshape(-1), xx.reshape(-1)], -1) + 1], 0)
                rp = RopeTables(pos, D, 100.0, dev)
                qw, qb, kw, kb = (torch.rand(D, device=dev) for _ in range(4))
                us = timeit(lambda: N.gemm_qkv(a, w, bias, out, H, D, qw, qb, kw, kb, 1e-5, rp.mode, rp.pos, rp.period,
                                               rp.cos, rp.sin), args.reps)
                res[f"qkv_fused/tile{mode}"] = {"us": round(us, 1), "tflops": round(2 * M * Nn * K / us / 1e6, 1)}
                print(f"qkv_fused/tile{mode}", res[f"qkv_fused/tile{mode}"], flush=True)
    if "norm" in only:
        xf = torch.randn(M, C, device=dev)
        y = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
        w, b = torch.rand(C, device=dev), torch.rand(C, device=dev)
        us = timeit(lambda: N.layernorm(xf, w, b, 1e-5, y), args.reps)
        res["layernorm"] = {"us": round(us, 1), "gbs": round(M * C * 6 / us / 1e3, 1)}
        qkv = torch.randn(M, 3 * C, device=dev).bfloat16()
        qw, qb, kw, kb = (torch.rand(D, device=dev) for _ in range(4))
        yy, xx = torch.meshgrid(torch.arange(37), torch.arange(37), indexing="ij")
        pos = torch.stack([yy.reshape(-1), xx.reshape(-1)], -1) + 1
        pos = torch.cat([torch.zeros(5, 2, dtype=pos.dtype), pos], 0)
        rp = RopeTables(pos, D, 100.0, dev)
        us = timeit(lambda: N.qknorm_rope(qkv, H, D, qw, qb, kw, kb, 1e-5, rp.mode, rp.pos, rp.period, rp.cos, rp.sin),
                    args.reps)
        res["qknorm_rope"] = {"us": round(us, 1), "gbs": round(M * 2 * C * 4 / us / 1e3, 1)}
    if "attn" in only:
        qkv = (torch.randn(M, 3 * C, device=dev)).bfloat16()
        o = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
        q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
        # bring clocks / power to the steady state first (the first ~2 s of a
        # cold box measure 5-20% slow)
        t_end = time.time() + args.warm_s
        while time.time() < t_end:
            N.attention(q, k, v, o, 1, H, M, M, D, M, M, M)
            torch.cuda.synchronize()
        for rnd, var, nw, (name, batch, n) in [(r_, v_, w_, sh) for r_ in range(args.rounds)
                                          for v_ in map(int, args.attn_variants.split(","))
                                          for w_ in map(int, args.attn_waves.split(","))
                                          for sh in (("global_attn", 1, M), ("frame_attn", 16, M // 16))]:
            N.tune(N.TUNE_ATTN_WAVES, nw)
            N.tune(N.TUNE_ATTN_VARIANT, var)
            us = timeit(lambda: N.attention(q, k, v, o, batch, H, n, n, D, n, n, n),
                        max(3, args.reps // 4))
            key = f"{name}/w{nw}/v{var}" + (f"/r{rnd}" if args.rounds > 1 else "")
            res[key] = {"us": round(us, 1), "tflops": round(4 * batch * H * n * n * D / us / 1e6, 1)}
            print(key, res[key], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
