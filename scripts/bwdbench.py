#!/usr/bin/env python3
"""Flash-attention backward microbenchmark at the alignment head's frame-block
shape (16 frames x 8 heads x 1,375 tokens x 128; alignment_head.py:347-366):
forward with LSE, then vggt_attention_bwd (dq + dk/dv launches) timed with
HIP events.  Prints TF/s over the 5 products (S twice, dP twice, dQ, dK, dV
counted as 7 x 2 n^2 d per (frame, head) incl. the recomputes)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "large-scale-vit-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import torch  # noqa: E402

from aligned_vggt import _native as N  # noqa: E402
from kbench import timeit  # noqa: E402

B, H, n, D = 16, 8, 1375, 128
C = H * D
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
qkv = torch.randn(B * n, 3 * C, device=dev, generator=g).bfloat16()
q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
o = torch.empty(B * n, C, device=dev, dtype=torch.bfloat16)
lse = torch.empty(B * H * n, device=dev)
N.attention_fwd_lse(q, k, v, o, lse, B, H, n, n, D, n, n, n)
do = torch.randn(B * n, C, device=dev, generator=g).bfloat16()
dqkv = torch.empty(B * n, 3 * C, device=dev, dtype=torch.bfloat16)
fn = lambda: N.attention_bwd(q, k, v, o, do, lse, dqkv[:, :C], dqkv[:, C:2 * C], dqkv[:, 2 * C:], B, H, n, n, D,
                             n, n, n)
for _ in range(3):
    us = timeit(fn, 20)
    print(f"attention_bwd {us:8.1f} us  {7 * 2 * B * H * n * n * D / us / 1e6:7.1f} TF/s", flush=True)
