#!/usr/bin/env python3
"""BASELINE.md §3 row C2 (the oracle, i.e. the reference's numerics in fp32
torch on CPU, on one 16 x 518^2 aggregator chunk) as a thread-scaling curve:
bench.py's bounded per-block sample (patch embed, one DINOv2 / frame / global
block at full size, x24) at 4, 8 and 16 threads on the GPU box host.  16 is
the per-GPU CPU share the box grants one command (its OMP_NUM_THREADS); a
whole-host row would take other jobs' cores, so the curve shows how the CPU
baseline scales up to that share instead.  Writes one JSON.

    python scripts/cpu_thread_scaling.py [--threads 4,8,16] [--out profiles/r11/cpu_thread_scaling.json]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="4,8,16")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r11", "cpu_thread_scaling.json"))
    a = ap.parse_args()
    try:
        lscpu = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
    except (OSError, subprocess.SubprocessError):
        lscpu = ""
    keep = ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core", "CPU(s)", "NUMA node(s)",
            "CPU max MHz")
    res = {"lscpu": {ln.split(":", 1)[0].strip(): ln.split(":", 1)[1].strip() for ln in lscpu.splitlines()
                     if ":" in ln and ln.split(":", 1)[0].strip() in keep},
           "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"), "rows": []}
    for th in (int(x) for x in a.threads.split(",")):
        r = bench.cpu_baseline(th)
        r.pop("committed_whole_chunk_row", None)
        r["s_per_chunk"] = round(1.0 / r["value"], 1)
        res["rows"].append(r)
        print(f"threads={th}: {r['s_per_chunk']} s per 16 x 518^2 chunk ({r['value']:.5f} chunks/s)", flush=True)
    base = res["rows"][0]
    for r in res["rows"]:
        r["speedup_vs_first"] = round(r["value"] / base["value"], 2)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
