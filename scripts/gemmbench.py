#!/usr/bin/env python3
"""GEMM anatomy sweep at the aggregator's shapes: our kernels (per tile mode)
vs torch.matmul (hipBLASLt) on the same operands, plain and with the fused
epilogues, plus long-K variants that separate the per-tile fixed cost
(prologue / epilogue) from the main loop.

    python scripts/gemmbench.py [--modes -1,0,7] [--reps 30] [--tokens 21984]
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
    ap.add_argument("--modes", default="-1,0,7")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--tokens", type=int, default=16 * 1374)
    ap.add_argument("--warm-s", type=float, default=3.0)
    ap.add_argument("--shapes", default="qkv,proj,fc1,fc2,fc1_k4096")
    ap.add_argument("--epis", default="torch,plain,gelu,resid")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    M = args.tokens
    x = (torch.rand(M, 4096, device=dev) * 2 - 1).bfloat16()
    shapes = {"qkv": (3072, 1024), "proj": (1024, 1024), "fc1": (4096, 1024), "fc2": (1024, 4096),
              "fc1_k4096": (4096, 4096), "qkv_k4096": (3072, 4096), "dx_k3072": (1024, 3072),
              "fc1_k64": (4096, 64), "fc1_k128": (4096, 128), "fc1_k256": (4096, 256), "fc2_k64": (1024, 64)}
    wq = (torch.randn(3072, 1024, device=dev) * 0.03).bfloat16()
    oq = torch.empty(M, 3072, device=dev, dtype=torch.bfloat16)
    t_end = time.time() + args.warm_s
    while time.time() < t_end:
        N.gemm_bf16(x[:, :1024], wq, torch.zeros(3072, device=dev), oq, N.EPI_BF16)
        torch.cuda.synchronize()
    res = {}
    for name in args.shapes.split(","):
        Nn, K = shapes[name]
        a = x[:, :K].contiguous()
        w = ((torch.rand(Nn, K, device=dev) * 2 - 1) * K ** -0.5).bfloat16()
        bias = torch.randn(Nn, device=dev) * 0.1
        fl = 2.0 * M * Nn * K
        ob = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
        if "torch" in args.epis.split(","):
            us = timeit(lambda: torch.matmul(a, w.t(), out=ob), args.reps)
            res[f"{name}/torch"] = {"us": round(us, 1), "tflops": round(fl / us / 1e6, 1)}
            print(f"{name}/torch", res[f"{name}/torch"], flush=True)
        xr = torch.randn(M, Nn, device=dev)
        gamma = torch.rand(Nn, device=dev)
        for mode in map(int, args.modes.split(",")):
            prev = N.tune(N.TUNE_GEMM_TILE, mode)
            try:
                for epi, en in ((N.EPI_BF16, "plain"), (N.EPI_GELU_BF16, "gelu"), (N.EPI_RESID_F32, "resid")):
                    if en not in args.epis.split(","):
                        continue
                    if epi == N.EPI_RESID_F32:
                        fn = lambda: N.gemm_bf16(a, w, bias, xr, epi, gamma=gamma)  # noqa: E731
                    else:
                        fn = lambda: N.gemm_bf16(a, w, bias, ob, epi)  # noqa: E731
                    us = timeit(fn, args.reps)
                    key = f"{name}/{en}/tile{mode}"
                    res[key] = {"us": round(us, 1), "tflops": round(fl / us / 1e6, 1)}
                    print(key, res[key], flush=True)
            finally:
                N.tune(N.TUNE_GEMM_TILE, prev)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
