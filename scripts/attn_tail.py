#!/usr/bin/env python3
"""Workgroup-quantisation probe for the global attention: time the production
kernel at nk = 21,984 keys for query counts that give whole and partial
dispatch rounds (4 workgroups of 128 query rows per CU x 256 CUs = 1024
slots), and report the time per query row."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "large-scale-vit-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import torch  # noqa: E402

from aligned_vggt import _native as N  # noqa: E402
from kbench import timeit  # noqa: E402

dev = torch.device("cuda:0")
M, C, H, D = 21984, 1024, 16, 64
qkv = torch.randn(M + 8192, 3 * C, device=dev).bfloat16()
o = torch.empty(M + 8192, C, device=dev, dtype=torch.bfloat16)
k, v = qkv[:M, C:2 * C], qkv[:M, 2 * C:]
t_end = time.time() + 3
while time.time() < t_end:
    N.attention(qkv[:M, :C], k, v, o, 1, H, M, M, D, M, M, M)
    torch.cuda.synchronize()
for rnd in range(2):
    for nq in (128 * 64, 128 * 128, 128 * 160, 21984, 128 * 176, 128 * 192, 128 * 224):
        us = timeit(lambda: N.attention(qkv[:nq, :C], k, v, o[:nq], 1, H, nq, M, D, nq + 8192, M, nq + 8192), 6)
        wg = -(-nq // 128) * H
        print(f"r{rnd} nq={nq:6d} wg={wg:5d} rounds={wg / 1024:5.2f} us={us:8.1f} ns/row={us * 1e3 / nq:7.2f} "
              f"TF/s={4 * H * nq * M * D / us / 1e6:7.1f}", flush=True)
