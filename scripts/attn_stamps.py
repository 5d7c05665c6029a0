#!/usr/bin/env python3
"""Where the global attention's wave cycles go (split the
waits by cause).  Runs vggt_attention_stamps -- the default forward (variant
33, 8-wave workgroups at the headline shape) with s_memtime stamps at every
tile boundary -- on random bf16 q/k/v of the configs[1] global attention
(1 x 16 heads x 21,984 tokens x 64), after the plain kernel has held the
clock for a few seconds, and prints per tile and wave: the tile's work (DMA
issue, QK^T, softmax, P.V issue, to its last LDS read), the end-of-tile
vmcnt(0) wait for the next tile's LDS-DMA, and the barrier.  Also times the
stamped and the plain kernel with HIP events (the instrumentation's cost).

    python scripts/attn_stamps.py [--tokens 21984] [--heads 16] [--out profiles/r11/attn_stamps.json]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "large-scale-vit-slam_amd"))

import torch  # noqa: E402

from aligned_vggt import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16 * 1374)
    ap.add_argument("--heads", type=int, default=16)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--warm-s", type=float, default=3.0)
    ap.add_argument("--variant", type=int, default=33, help="VGGT_TUNE_ATTN_VARIANT: 33 (default), 2081, 4129")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    N.tune(N.TUNE_ATTN_VARIANT, a.variant)
    dev = torch.device("cuda:0")
    n, H, B, D = a.tokens, a.heads, a.batch, 64
    C = H * D
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B * n, 3 * C, device=dev, generator=g).to(torch.bfloat16)
    o = torch.empty(B * n, C, device=dev, dtype=torch.bfloat16)
    q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
    plain = lambda: N.attention(q, k, v, o, B, H, n, n, D, n, n, n)  # noqa: E731
    stamped = lambda: N.attention_stamps(q, k, v, o, B, H, n, n, n, n, n)  # noqa: E731
    t_end = time.time() + a.warm_s
    while time.time() < t_end:
        plain()
        torch.cuda.synchronize()

    def ev(fn, reps=10):
        ts = []
        for _ in range(reps):
            x, y = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            x.record()
            r = fn()
            y.record()
            y.synchronize()
            ts.append(x.elapsed_time(y) * 1e3)
        return statistics.median(ts), r

    us_plain, _ = ev(plain)
    us_stamp, st = ev(stamped)
    o_ref = o.clone()
    plain()
    torch.cuda.synchronize()
    same = bool(torch.equal(o, o_ref))
    st = st.cpu().double()
    nt = -(-n // 64)
    work, vm, bar = st[:, 2], st[:, 3], st[:, 4]
    tot = work + vm + bar
    nw = 8 if n >= 4096 else 4
    flops = 4.0 * B * H * n * n * D
    res = {"variant": a.variant, "shape": {"batch": B, "heads": H, "tokens": n, "D": D, "waves_per_workgroup": nw, "tiles_per_wave": nt},
           "us_plain": round(us_plain, 1), "us_stamped": round(us_stamp, 1),
           "tflops_plain": round(flops / us_plain / 1e6, 1), "outputs_bitwise_equal": same,
           "cycles_per_tile": {"work": round(work.mean().item() / nt, 1), "vmcnt_wait": round(vm.mean().item() / nt, 1),
                               "barrier": round(bar.mean().item() / nt, 1), "total": round(tot.mean().item() / nt, 1)},
           "share": {"work": round((work.sum() / tot.sum()).item(), 4), "vmcnt_wait": round((vm.sum() / tot.sum()).item(), 4),
                     "barrier": round((bar.sum() / tot.sum()).item(), 4)},
           "barrier_by_wave_slot": [round((bar.view(-1, nw)[:, w].mean() / nt).item(), 1) for w in range(nw)],
           "work_by_wave_slot": [round((work.view(-1, nw)[:, w].mean() / nt).item(), 1) for w in range(nw)],
           "mfma_cycles_per_tile_per_wave": 16 * 32,
           "note": "s_memtime cycles (shader clock) per wave summed over its tiles; work = DMA issue + QK^T + "
                   "softmax + P.V issue up to the tile's last LDS read (lgkmcnt(0) in the stamp); 4 waves share a "
                   "SIMD, so a wave's cycles per tile are ~4x its own issue time"}
    print(json.dumps(res, indent=1))
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
