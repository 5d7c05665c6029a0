#!/usr/bin/env python3
"""BASELINE.md §3 CPU rows measured on whole chunks (not extrapolated):

  C1  one 8-frame 518^2 chunk through the oracle's point-aligned VGGT
      (pointAligned_wrapped_vggt.py:34-157: aggregator, point / depth DPT heads,
      camera head), fp32, random-init weights;
  C2  one 16-frame 518^2 chunk through the oracle's aggregator (the CPU side
      of the configs[1] headline), fp32.

Each row: 1 warm-up (a reduced-depth pass of the same code) + N timed whole
chunks, median, at the listed thread counts (default: the per-GPU share, 16,
and os.cpu_count()).  The oracle is the reference's numerics restated in fp32
torch (the reference's own Python cannot run without the absent vggt package,
SURVEY.md §8c).  Writes one JSON (default profiles/cpu_baseline_full.json),
which bench.py attaches to its cpu_baseline.

  python scripts/cpu_baseline_full.py [--rows C1,C2] [--threads 16,0] [--runs 3] [--out PATH] [--append]
      (--threads 0 = os.cpu_count(); --append adds this call's timed runs to a row's earlier ones, so a
      slow row can be measured over several bounded calls -- each call still does its own warm-up)
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "large-scale-vit-slam_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def row_c1(runs: int):
    from oracle import alignment_oracle as AO
    from aligned_vggt.models.pointAligned_wrapped_vggt import VGGT
    from aligned_vggt.utils.synthetic import condition_pose_outputs_, synthetic_images, synthetic_init_
    m = VGGT(enable_track=False)
    synthetic_init_(m, seed=0)
    condition_pose_outputs_(m)
    sd = {k: v.detach() for k, v in m.state_dict().items()}
    del m
    imgs = synthetic_images(1, 8, 518, 518, seed=1234)
    warm = lambda: AO.point_aligned_forward(sd, imgs[:, :2], 0, None,  # noqa: E731
                                            agg_kwargs={"keep": (0, 1, 2, 3), "depth": 4, "dino_depth": 1})
    full = lambda: AO.point_aligned_forward(sd, imgs, 0, None)  # noqa: E731
    return warm, full, "point-aligned VGGT, 1 x 8 x 518^2 (aggregator + point/depth DPT + camera head)"


def row_c2(runs: int):
    from oracle import vggt_oracle as O
    from aligned_vggt.backbone.aggregator import Aggregator
    from aligned_vggt.utils.synthetic import synthetic_images, synthetic_init_
    agg = Aggregator()
    synthetic_init_(agg, seed=0)
    sd = {"aggregator." + k: v.detach() for k, v in agg.state_dict().items()}
    del agg
    imgs = synthetic_images(1, 16, 518, 518, seed=1234)
    warm = lambda: O.aggregator(sd, imgs[:, :2], keep=(1,), depth=2, dino_depth=1)  # noqa: E731
    full = lambda: O.aggregator(sd, imgs, keep=(4, 11, 17, 23))  # noqa: E731
    return warm, full, "VGGT aggregator, 1 x 16 x 518^2 (DINOv2 + 24 frame/global blocks, layers 4/11/17/23)"


def _heartbeat(state: dict) -> None:
    """A progress line every minute (a GPU-box command that prints nothing for
    3 minutes is taken to be hung; one C2 chunk at 16 threads takes ~8)."""
    import threading

    def beat():
        while not state.get("done"):
            time.sleep(60)
            if not state.get("done"):
                print(f"[{time.strftime('%H:%M:%S')}] still running: {state.get('what')}", flush=True)

    threading.Thread(target=beat, daemon=True).start()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="C1,C2")
    ap.add_argument("--threads", default="16,0")
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "cpu_baseline_full.json"))
    ap.add_argument("--append", action="store_true", help="add rows to an existing --out file")
    a = ap.parse_args()
    res = {"host_cpu": _cpu_model(), "host_logical_cpus": os.cpu_count(), "torch": torch.__version__,
           "procedure": "1 warm-up (reduced-depth pass) + N timed whole chunks, median; oracle fp32 "
                        "(reference numerics), random-init weights, synthetic uniform frames", "rows": {}}
    if a.append and os.path.exists(a.out):
        with open(a.out) as f:
            res["rows"] = json.load(f).get("rows", {})
    state = {"what": "setup"}
    _heartbeat(state)
    for row in a.rows.split(","):
        state["what"] = f"{row} setup"
        warm, full, what = {"C1": row_c1, "C2": row_c2}[row](a.runs)
        for th in (int(x) for x in a.threads.split(",")):
            th = th or (os.cpu_count() or 1)
            torch.set_num_threads(th)
            with torch.no_grad():
                t0 = time.perf_counter()
                warm()
                tw = time.perf_counter() - t0
                ts = []
                for i in range(a.runs):
                    state["what"] = f"{row} threads={th} run {i}"
                    t0 = time.perf_counter()
                    full()
                    ts.append(time.perf_counter() - t0)
                    print(f"[{time.strftime('%H:%M:%S')}] {row} threads={th} run {i}: {ts[-1]:.1f} s", flush=True)
            key = f"{row}_t{th}"
            prev = res["rows"].get(key, {}).get("runs_s", []) if a.append else []
            allr = prev + [round(x, 2) for x in ts]  # --append: runs of earlier calls (one GPU-box lease each) kept
            med = statistics.median(allr)
            res["rows"][key] = {"row": row, "workload": what, "threads": th, "runs": len(allr),
                                "warmup_s": round(tw, 2), "runs_s": allr, "median_s_per_chunk": round(med, 2),
                                "chunks_per_s": round(1.0 / med, 6)}
            with open(a.out, "w") as f:  # after every row: a killed run keeps what it measured
                json.dump(res, f, indent=1)
    state["done"] = True
    print(json.dumps(res))


if __name__ == "__main__":
    main()
