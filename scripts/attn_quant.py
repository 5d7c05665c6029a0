#!/usr/bin/env python3
"""Global attention's round quantisation: attn_fwd (16 heads, D 64, nk = 21,984
keys) at query counts whose workgroup count (256 rows each, 16 heads) fills
a whole number of rounds of 512 resident workgroups (2 per CU) or not.
TF/s per nq; HIP events over back-to-back launches.  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "large-scale-vit-slam_amd"))

import torch  # noqa: E402

from aligned_vggt import _native as N  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    H, D, NK = 16, 64, 21984
    C = H * D
    nqs = [int(x) for x in os.environ.get("NQS", "16384,21984,24576").split(",")]
    reps = int(os.environ.get("REPS", "10"))
    k = (torch.randn(NK, C, device=dev) * 0.5).bfloat16()
    v = (torch.randn(NK, C, device=dev) * 0.5).bfloat16()
    qa = (torch.randn(max(nqs), C, device=dev) * 0.5).bfloat16()
    o = torch.empty(max(nqs), C, device=dev, dtype=torch.bfloat16)
    t_end = time.time() + 2.0
    while time.time() < t_end:
        N.attention(qa[:NK], k, v, o[:NK], 1, H, NK, NK, D, NK, NK, NK)
        torch.cuda.synchronize()
    res = {}
    for _ in range(2):
        for nq in nqs:
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(reps):
                N.attention(qa[:nq], k, v, o[:nq], 1, H, nq, NK, D, nq, NK, nq)
            b.record()
            b.synchronize()
            ms = a.elapsed_time(b) / reps
            fl = 4.0 * nq * NK * D * H
            wgs = -(-nq // 256) * H
            res[str(nq)] = {"ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1), "workgroups": wgs,
                            "rounds_of_512": round(wgs / 512, 3)}
            print(nq, res[str(nq)], flush=True)
    # the 21,984-row launch as two: whole rounds of 8-wave workgroups, then the tail on
    # narrower workgroups (same rows per wave, finer per-CU balance)
    nq = NK
    for split in (16384, 12288):
        for tail_w in (4, 2, 40):  # 40: 4-wave tail on the 32x32x16 form (bitwise the 8-wave rows)
            ts = []
            for _ in range(2):
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(reps):
                    N.attention(qa[:split], k, v, o[:split], 1, H, split, NK, D, split, NK, split)
                    prev = N.tune(N.TUNE_ATTN_WAVES, 4 if tail_w == 40 else tail_w)
                    p16 = N.tune(N.TUNE_ATTN16, 0) if tail_w == 40 else None
                    N.attention(qa[split:nq], k, v, o[split:nq], 1, H, nq - split, NK, D, nq - split, NK, nq - split)
                    N.tune(N.TUNE_ATTN_WAVES, prev)
                    if p16 is not None:
                        N.tune(N.TUNE_ATTN16, p16)
                b.record()
                b.synchronize()
                ts.append(a.elapsed_time(b) / reps)
            ms = min(ts)
            key = f"py_split{split}_tail{tail_w}w"
            res[key] = {"ms": round(ms, 4), "tflops": round(4.0 * nq * NK * D * H / ms / 1e9, 1)}
            print(key, res[key], flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
