#!/usr/bin/env python3
"""Time vggt_wgrad_bf16 at the alignment head's training shapes (22,000 tokens):
fc1 / fc2 / qkv / proj weight gradients.  VGGT_WGRAD_DMA selects the staging (1 LDS-DMA, 0 registers)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "large-scale-vit-slam_amd"))

import torch  # noqa: E402

from aligned_vggt import _native as N  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    M = 22000
    g = torch.Generator(device=dev).manual_seed(0)
    for name, Nn, K in (("fc1", 4096, 1024), ("fc2", 1024, 4096), ("qkv", 3072, 1024), ("proj", 1024, 1024)):
        dy = torch.randn(M, Nn, device=dev, generator=g).bfloat16()
        x = torch.randn(M, K, device=dev, generator=g).bfloat16()
        dw = torch.empty(Nn, K, device=dev)
        for _ in range(3):
            N.wgrad_bf16(dy, x, dw, False)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            N.wgrad_bf16(dy, x, dw, False)
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) / 20 * 1e3
        ref = (dy.float().t() @ x.float())
        err = ((dw - ref).norm() / ref.norm()).item()
        print(f"dma={os.environ.get('VGGT_WGRAD_DMA', '1')} {name} {us:.1f} us {2 * M * Nn * K / us / 1e6:.0f} TF/s rel {err:.1e}",
              flush=True)


if __name__ == "__main__":
    main()
