#!/usr/bin/env python3
"""Headline benchmark: chunks/sec of the VGGT encoder (Aggregator: DINOv2
ViT-L/14-reg + 24 frame + 24 global alternating-attention blocks) forward on
one 16-frame 518x518 synthetic chunk (BASELINE.json configs[1]), bf16 MFMA,
random-init weights.

  python bench.py [--gpus N --steps K --warmup W] [--workload aggregator|chunk|sequence|train]
  python bench.py --config 3 --gpus 8     (BASELINE configs[3]: 512 frames 154x518, chunk 16 / overlap 4)

N > 1: one process per GPU (torch.distributed over RCCL).  Run as is, bench.py
starts ``python -m torch.distributed.run --nproc-per-node N`` itself (before
touching the GPU) and relays rank 0's line; under an external torchrun it
reads RANK / WORLD_SIZE.  aggregator / chunk / train: every rank runs its own
independent chunks (replicas, weak scaling), value = all ranks' chunks /
max-over-ranks time; sequence: the ranks share one sequence through the
ChunkPipeline baton ring (strong scaling).  Prints ONE JSON line on rank 0 with the roofline of
the dominant kernel (global attention) measured with HIP events on the
stream it is launched on, and the CPU baseline (the oracle's fp32 path on a
bounded sample of the same workload).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "large-scale-vit-slam_amd"))
sys.path.insert(0, ROOT)

# kernel arguments in device memory (see aligned_vggt/__init__.py), set before
# the HIP runtime initialises
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
os.environ.setdefault("GPU_STREAMOPS_CP_WAIT", "1")  # the encode gate's wait on the CP (aligned_vggt/__init__.py)
import torch  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
H_IMG = W_IMG = 518
S_FRAMES = 16


def agg_flops(S=S_FRAMES, H=H_IMG, W=W_IMG, C=1024, depth=24, dino_depth=24):
    """Algorithmic FLOPs of one aggregator forward (BASELINE.md §2 counting:
    2MNK per GEMM, 4*Nq*Nk*d per attention)."""
    hw = (H // 14) * (W // 14)
    P = 5 + hw
    T = S * P
    lin_per_block = 24 * T * C * C  # qkv 6, proj 2, fc1 8, fc2 8 (x T C^2)
    frame_attn = 4 * S * P * P * C
    global_attn = 4 * T * T * C
    patch = 2 * S * hw * 3 * 14 * 14 * C
    total = (depth * 2 + dino_depth) * lin_per_block + (dino_depth + depth) * frame_attn + depth * global_attn + patch
    return {"total": total, "global_attn_launch": global_attn, "global_attn": depth * global_attn,
            "attn": depth * global_attn + (dino_depth + depth) * frame_attn}


def cpu_baseline(threads: int):
    """Time the oracle (reference numerics, fp32, CPU) on a bounded sample of
    the SAME workload at the full 16x518x518 chunk shape (~20 s): the DINOv2
    patch embed + final LayerNorm, one DINOv2 block, one frame block, one
    global block and the four kept-layer concats, after a small warm-up pass;
    the cheap blocks are timed 3 times (median), the global block (most of the
    sample) once.  The whole chunk = patch embed + 24 x each block kind +
    concats.  Threads: the GPU box's per-GPU CPU share (16), not the whole host
    (os.cpu_count() reports every CPU of the machine, shared with other jobs).
    The full-chunk measurements of scripts/cpu_baseline_full.py (1 warm-up +
    3 timed whole chunks, median, at 16 and at os.cpu_count() threads;
    BASELINE.md §3 rows C1 / C2) are attached from profiles/cpu_baseline_full.json."""
    import statistics
    from oracle import vggt_oracle as O
    from aligned_vggt.backbone.aggregator import Aggregator
    from aligned_vggt.utils.synthetic import synthetic_images, synthetic_init_
    torch.set_num_threads(threads)
    agg = Aggregator(depth=1, dino_depth=1)
    synthetic_init_(agg)
    sd = {"aggregator." + k: v for k, v in agg.state_dict().items()}
    hw = (H_IMG // 14) * (W_IMG // 14)
    P = 5 + hw
    g = torch.Generator().manual_seed(0)
    x = torch.randn(S_FRAMES, P, 1024, generator=g)
    imgs = synthetic_images(1, S_FRAMES, H_IMG, W_IMG)[0]
    pos = O.position_grid(S_FRAMES, H_IMG // 14, W_IMG // 14, 5)

    def timed(fn, n=1):
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return statistics.median(ts)

    with torch.no_grad():
        t0 = time.perf_counter()
        O.block(sd, "aggregator.frame_blocks.0.", x[:2], 16, pos[:2], "2d", True)  # warm-up
        warm = time.perf_counter() - t0
        t_patch = timed(lambda: O.dinov2(sd, "aggregator.patch_embed.", imgs, False, depth=0))
        t_dino = timed(lambda: O.block(sd, "aggregator.patch_embed.blocks.0.", x, 16, eps=1e-6), 3)
        t_frame = timed(lambda: O.block(sd, "aggregator.frame_blocks.0.", x, 16, pos, "2d", True), 3)
        t_glob = timed(lambda: O.block(sd, "aggregator.global_blocks.0.", x.view(1, S_FRAMES * P, 1024), 16,
                                       pos.view(1, -1, 2), "2d", True))
        t_cat = timed(lambda: [torch.cat([x, x], dim=-1) for _ in range(4)])
    sec_chunk = t_patch + 24 * (t_dino + t_frame + t_glob) + t_cat
    out = {"value": 1.0 / sec_chunk, "unit": "chunks/s", "cores": threads, "kind": "port",
           "host_cpu": _cpu_model(), "host_logical_cpus": os.cpu_count(),
           "sample": f"oracle fp32 CPU (reference numerics) at 16x518x518 after a {warm:.1f} s warm-up: patch embed "
                     f"+ final LN {t_patch:.2f} s, DINOv2 block {t_dino:.2f} s and frame block {t_frame:.2f} s "
                     f"(median of 3 each), global block {t_glob:.2f} s, 4 kept-layer concats; blocks scaled x24 "
                     f"each to a full aggregator chunk ({sec_chunk:.1f} s/chunk)"}
    # the value is this run's own bounded sample (on this host, now); the whole-chunk rows
    # of BASELINE.md §3 measured earlier on a GPU-box host (scripts/cpu_baseline_full.py,
    # committed in profiles/cpu_baseline_full.json) ride along, labelled as such
    committed = _measured_row("C2", threads)
    if committed is not None:
        out["committed_whole_chunk_row"] = committed
    # the same sample at 4 / 8 / 16 threads on a GPU-box host (scripts/cpu_thread_scaling.py):
    # how the CPU baseline scales up to the per-command share of 16 threads
    try:
        with open(os.path.join(ROOT, "profiles", "r11", "cpu_thread_scaling.json")) as fh:
            sc = json.load(fh)
        out["committed_thread_scaling"] = {
            "host": sc.get("lscpu", {}).get("Model name"),
            "s_per_chunk_by_threads": {str(r["cores"]): r["s_per_chunk"] for r in sc.get("rows", [])},
            "source": "profiles/r11/cpu_thread_scaling.json"}
    except (OSError, ValueError, KeyError):
        pass
    return out


def _measured_row(row: str, threads: int):
    """A BASELINE.md §3 CPU row measured on whole chunks by scripts/cpu_baseline_full.py
    (1 warm-up + >= 3 timed runs, median; profiles/cpu_baseline_full.json), or None."""
    try:
        with open(os.path.join(ROOT, "profiles", "cpu_baseline_full.json")) as fh:
            full = json.load(fh)
    except (OSError, ValueError):
        return None
    r = full.get("rows", {}).get(f"{row}_t{threads}")
    if not r:
        return None
    if "sequence_s" in r:  # C3: one whole sequence
        return {"value": r["chunks_per_s"], "unit": "chunks/s", "cores": threads, "kind": "port",
                "host_cpu": full.get("host_cpu"), "host_logical_cpus": full.get("host_logical_cpus"),
                "measured": "earlier, on a GPU-box host (profiles/cpu_baseline_full.json)",
                "sample": f"oracle fp32 CPU (reference numerics), {r['workload']}: chunks {r['chunk_s']} s, "
                          f"sequence {r['sequence_s']} s"}
    if r.get("runs", 0) < 3:
        return None
    return {"value": r["chunks_per_s"], "unit": "chunks/s", "cores": threads, "kind": "port",
            "host_cpu": full.get("host_cpu"), "host_logical_cpus": full.get("host_logical_cpus"),
            "measured": "earlier, on a GPU-box host (profiles/cpu_baseline_full.json)",
            "sample": f"oracle fp32 CPU (reference numerics), {r['workload']}: {r['runs']} timed whole chunks "
                      f"{r['runs_s']} s after a warm-up, median {r['median_s_per_chunk']} s/chunk"}


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _launch(args) -> int:
    """--gpus N > 1 without a torchrun environment: start N ranks with
    torch.distributed.run as a CHILD process (the parent never touches the
    GPU, so no exec after HIP init) and return its exit code; rank 0's JSON
    line reaches stdout through it."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


# BASELINE.json configs as presets: (workload, seq_frames, height, frames, overlap, memory tokens)
CONFIGS = {0: ("point", None, 518, 8, 0, 0), 1: ("aggregator", None, 518, 16, 4, 8), 2: ("sequence", 64, 518, 16, 4, 8),
           3: ("sequence", 512, 154, 16, 4, 0), 4: ("sequence", 512, 154, 16, 4, 8)}


class EventTimer:
    """HIP-event timing of tagged native launches on the launching stream."""

    def __init__(self, tags):
        self.tags = set(tags)
        self.pairs = []
        self.active = False

    def __call__(self, tag, fn):
        if not self.active or tag not in self.tags:
            return fn()
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        st = torch.cuda.current_stream()
        s.record(st)
        r = fn()
        e.record(st)
        self.pairs.append((s, e))
        return r

    def mean_ms(self):
        torch.cuda.synchronize()
        if not self.pairs:
            return None
        return sum(s.elapsed_time(e) for s, e in self.pairs) / len(self.pairs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=None, choices=sorted(CONFIGS),
                    help="BASELINE.json configs[i] preset (sets workload / frames / size / memory)")
    ap.add_argument("--memory-tokens", type=int, default=8, help="alignment-head memory tokens (0: no memory)")
    ap.add_argument("--workload", default="aggregator",
                    choices=["aggregator", "point", "chunk", "sequence", "train", "selftest"],
                    help="aggregator: BASELINE configs[1] headline (default); point: configs[0], one 8-frame "
                         "518^2 chunk through the point-aligned VGGT (aggregator + point / depth / camera heads); "
                         "chunk: full FeatureAlignedVGGT "
                         "per-chunk forward (encoder + alignment head + camera/depth heads); sequence: configs[2..4] "
                         "chunk pipeline over --seq-frames frames (RCCL baton ring at N>1); train: one alignment-head "
                         "training step (two chunks with memory recurrence, forward + backward + AdamW) on resident "
                         "synthetic aggregator tokens (SURVEY §8f row 4); selftest: the multi-rank launcher and "
                         "baton ring on CPU / gloo with a toy model (no GPU)")
    ap.add_argument("--seq-frames", type=int, default=64)
    ap.add_argument("--height", type=int, default=H_IMG)
    ap.add_argument("--overlap", type=int, default=4)
    ap.add_argument("--frames", type=int, default=S_FRAMES)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--cpu-runs", type=int, default=1,
                    help="point workload: timed full-chunk CPU runs after the warm-up (BASELINE.md §3 asks for 3)")
    args = ap.parse_args()
    if args.config is not None:
        args.workload, seq, args.height, args.frames, args.overlap, args.memory_tokens = CONFIGS[args.config]
        if seq is not None:
            args.seq_frames = seq

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_launch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}; using the launcher's {world} ranks",
              file=sys.stderr)
    if args.workload == "selftest":
        return bench_selftest(args, world, rank)
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from aligned_vggt import _native
    from aligned_vggt.backbone.aggregator import Aggregator
    from aligned_vggt.utils.synthetic import synthetic_images, synthetic_init_

    if args.workload == "train":
        return bench_train(args, world, rank, dev)
    if args.workload == "point":
        return bench_point(args, world, rank, dev)
    if args.workload != "aggregator":
        return bench_full(args, world, rank, dev)

    agg = Aggregator().to(dev)
    synthetic_init_(agg, seed=0)
    agg.eval()
    imgs = synthetic_images(1, args.frames, H_IMG, W_IMG, seed=1234 + rank, device=dev)
    keep = (4, 11, 17, 23)

    timer = EventTimer({"global_attn"})
    _native.EVENT_HOOK = timer

    def step():
        outs, _ = agg(imgs, keep_layers=keep)
        return outs

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    timer.active = True
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    timer.active = False
    attn_ms = timer.mean_ms()
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()

    fl = agg_flops(S=args.frames)
    chunks = args.steps * world
    value = chunks / dt
    ms_step = dt / args.steps * 1e3
    if rank == 0:
        attn_tflops = fl["global_attn_launch"] / (attn_ms * 1e-3) / 1e12 if attn_ms else None
        line = {
            "metric": "chunks/sec (16-frame 518x518) + ViT MFMA util%",
            "value": round(value, 4),
            "unit": "chunks/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (uniform [0,1) frames, random-init weights)",
            "config": {"workload": "VGGT aggregator forward (DINOv2-L/14-reg + 24x frame/global AA blocks), "
                                   "1 chunk of %d frames 518x518, layers 4/11/17/23 emitted" % args.frames,
                       "frames": args.frames, "tokens_per_chunk": args.frames * (5 + 37 * 37),
                       "parallelism": "replicas x%d" % world},
            "mfma_util_whole_step": round(fl["total"] * value / world / (PEAK_BF16_TFLOPS * 1e12), 4),
            "mfma_util_pmc": _step_pmc(),
            "tflops_per_gpu": round(fl["total"] * value / world / 1e12, 1),
            "roofline": {"bound": "mfma", "kernel": "attn_fwd_kernel<64> (global attention, 1x16 heads x 21984^2 x 64)",
                         "achieved": round(attn_tflops, 1) if attn_tflops else None, "peak": PEAK_BF16_TFLOPS,
                         "unit": "TFLOP/s",
                         "frac": round(attn_tflops / PEAK_BF16_TFLOPS, 4) if attn_tflops else None,
                         "avg_launch_ms": round(attn_ms, 4) if attn_ms else None,
                         "flops_per_launch": fl["global_attn_launch"], "traffic": _pmc_traffic(),
                         "traffic_provenance": _counter_provenance("attn_traffic.json")},
            "mfma_util_pmc_provenance": _counter_provenance("step_mfma.json"),
        }
        if os.environ.get("VGGT_MFMA_PROBE", "1") != "0":
            # the peak the roofline is priced against, measured on this device after the timed
            # region: back-to-back 32x32x16 bf16 MFMAs, sustained TF/s + clock
            line["mfma_peak_measured"] = {"random_operands": _native.mfma_probe(random=True),
                                          "zero_operands": _native.mfma_probe(random=False)}
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(args.cpu_threads)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _pmc_traffic():
    """HBM bytes per global-attention launch from the committed PMC summary
    (profiles/attn_traffic.json, written by scripts/pmc_traffic.py from two
    separate `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes of this
    same bench command; FETCH_SIZE x2 per the gfx950 correction), or None."""
    d = _committed_counters("attn_traffic.json")
    return None if d is None else d.get("hbm_bytes_per_launch")


def _committed_counters(name: str):
    """A committed counter file (profiles/<name>) if it was measured on these
    sources (aligned_vggt.provenance: same source fingerprint), else None --
    a stale counter is never reported as current."""
    from aligned_vggt.provenance import source_fingerprint
    try:
        with open(os.path.join(ROOT, "profiles", name)) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None
    if d.get("source_fingerprint") != source_fingerprint():
        return None
    return d


def _counter_provenance(name: str) -> dict:
    try:
        with open(os.path.join(ROOT, "profiles", name)) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return {"file": "profiles/" + name, "status": "missing"}
    from aligned_vggt.provenance import source_fingerprint
    fp = source_fingerprint()
    return {"file": "profiles/" + name, "git_head": d.get("git_head"), "source_fingerprint": d.get("source_fingerprint"),
            "status": "current" if d.get("source_fingerprint") == fp else "stale (measured on other sources: not used)"}


def _step_pmc():
    """Counter-based MFMA utilisation of the aggregator step from the committed
    summary (profiles/step_mfma.json, scripts/gpu_step_pmc.sh: rocprofv3 --pmc
    SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE over one step of this bench,
    and SQ_INSTS_VALU_MFMA_MOPS_BF16), or None."""
    d = _committed_counters("step_mfma.json")
    if d is None:
        return None
    out = {"mfma_busy_frac": d.get("mfma_busy_frac"), "by_class": d.get("mfma_busy_frac_by_class"),
           "source": "profiles/step_mfma.json", "git_head": d.get("git_head")}
    if d.get("mfma_bf16_tflop_counted") is not None:
        out["bf16_tflop_counted_per_step"] = round(d["mfma_bf16_tflop_counted"], 3)
    return out


def bench_full(args, world, rank, dev):
    """Full per-chunk model (configs[2..4]): 'chunk' = one FeatureAlignedVGGT
    forward per rank per step (context threaded step to step); 'sequence' =
    one ChunkPipeline pass over a synthetic --seq-frames sequence per step."""
    import torch.distributed as dist
    from aligned_vggt.dist.pipeline import ChunkPipeline
    from aligned_vggt.models.featureAligned_vggt import FeatureAlignedVGGT
    from aligned_vggt.utils.data import generate_chunks
    from aligned_vggt.utils.synthetic import condition_pose_outputs_, synthetic_images, synthetic_init_
    nm = args.memory_tokens
    model = FeatureAlignedVGGT(enable_point=False, enable_track=False, num_memory_tokens=nm).to(dev).eval()
    synthetic_init_(model, seed=0)
    condition_pose_outputs_(model)
    H, W = args.height, W_IMG
    S, ov = args.frames, args.overlap
    if args.workload == "chunk":
        imgs = synthetic_images(1, S, H, W, seed=1234 + rank, device=dev)
        ctx = {"c": None}

        def step():
            ctx["c"] = model(imgs, ov, ctx["c"])
            for k in ("depth", "depth_conf", "images", "pose_enc", "memory_tokens"):
                if k in ctx["c"] and isinstance(ctx["c"][k], list) and len(ctx["c"][k]) > 2:
                    del ctx["c"][k][0]
        n_chunks_step = world
    else:
        # the sequence resident in HBM before the timed region (the bench contract);
        # the pipeline also overlaps host-to-device transfers when given host frames
        seq = synthetic_images(1, args.seq_frames, H, W, seed=1234, device="cpu").to(dev)
        pipe = ChunkPipeline(model, device=dev)
        P1 = 6 + (H // 14) * (W // 14)

        def step():
            pipe.run(seq, S, ov, token_dims=(P1, 1024), memory_shape=(1, nm, 512) if nm > 0 else None)
        n_chunks_step = len(generate_chunks(args.seq_frames, "chunk_overlap", S, ov))
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    recurrence = ring_model = None
    if args.workload == "sequence" and os.environ.get("VGGT_RECURRENCE_PROBE", "1") != "0":
        recurrence = _recurrence_probe(pipe, step, lambda: pipe.prepare(seq, S, ov), n_chunks_step,
                                       dt / args.steps * 1e3, world)
        if world == 1:
            ring_model = _ring_model(model, pipe, seq, S, ov, recurrence, dt / args.steps * 1e3)
    if world > 1:
        dist.destroy_process_group()
    if rank == 0:
        value = n_chunks_step * args.steps / dt
        print(json.dumps({
            "metric": "chunks/sec (%d-frame %dx%d) full per-chunk FeatureAlignedVGGT" % (S, H, W),
            "value": round(value, 4), "unit": "chunks/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak" if args.workload == "chunk" else "strong", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic", "config": {"workload": args.workload, "baseline_config": args.config,
                                            "frames": S, "overlap": ov,
                                            "seq_frames": args.seq_frames if args.workload == "sequence" else None,
                                            "image": [H, W], "heads": "camera+depth+alignment(memory %d)" % nm,
                                            "parallelism": ("chunk pipeline x%d (RCCL baton ring)" % world
                                                            if args.workload == "sequence" else
                                                            "replicas x%d" % world)},
            "recurrence": recurrence, "ring_model": ring_model,
            # BASELINE.md §3 row C3 (configs[2]'s sequence through the fp32 oracle at 16 threads: 2,350 s, too
            # long to re-time inside a bench run) as measured on a GPU-box host, labelled as such
            "cpu_baseline": (_measured_row("C3", args.cpu_threads)
                             if (args.config == 2 and world == 1 and not args.no_cpu_baseline) else None)}),
              flush=True)


def _recurrence_probe(pipe, step, prepare, n_chunks, t1_ms, world):
    """The alignment recurrence's critical path: chunk i's
    alignment needs chunk i-1's post-head tokens, so with W ranks a sequence
    takes at least n_chunks x t_align (+ W-1 .. n-1 baton hops) whatever the
    encodes do.  Measured after the timed region with HIP events around every
    align_chunk on its own stream: (a) the sequential schedule (align between
    encodes on the compute stream: t_align alone) and (b) the ring's schedule
    (align on the side stream while the next encode group runs: t_align under
    load, the regime of every W > 1 rank).  At W = 1 (b) is the W = 1 ring
    schedule (overlap_align), whose sequence time is reported beside: with the
    ring's defaults (the encode gated while an alignment runs, persistent
    GEMMs), gated with short-workgroup streams, ungated short-workgroup, ungated
    persistent (the round-3 schedule) and, for VGGT_PROBE_RESERVE=r,..., with
    the encodes masked off r CUs.  chain_lower_bound_frac_* (a lower bound only) =
    n_chunks x t_align over the overlapped sequence time / 8: the 8-rank ring's
    critical path against its encode share (<= 1: the encodes bound it)."""
    import statistics
    pipe.time_align = True
    out = {"n_chunks": n_chunks}
    # (name, overlap_align, reserve_cus, short_workgroups, gate_encode); None = the pipeline's setting
    rsvs = [int(x) for x in os.environ.get("VGGT_PROBE_RESERVE", "").split(",") if x]
    modes = ((("alone", False, 0, None, None), ("under_load", True, 0, None, None),
              ("under_load_gated_short", True, 0, True, True), ("under_load_ungated_short", True, 0, True, False),
              ("under_load_ungated", True, 0, False, False))
             + tuple(("under_load_reserved%d" % r, True, r, True, False) for r in rsvs)
             if world == 1 else (("under_load", None, None, None, None),))
    for name, ov_mode, rsv, short, gate in modes:
        keep = (pipe.overlap_align, pipe.reserve_cus, pipe.short_workgroups, pipe.gate_encode)
        if ov_mode is not None:
            pipe.overlap_align = ov_mode
        if rsv is not None:
            pipe.reserve_cus = rsv
        if short is not None:
            pipe.short_workgroups = short
        if gate is not None:
            pipe.gate_encode = gate
        keep_gates = pipe.plan_gates
        pipe.plan_gates = (pipe.gate_encode,)  # the mode's gate on every rank, not the planner's choice
        prepare()  # the planner's host-side search outside the timed call
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        pipe.overlap_align, pipe.reserve_cus, pipe.short_workgroups, pipe.gate_encode = keep
        pipe.plan_gates = keep_gates
        ms = pipe.align_ms()
        out["t_align_ms_%s_median" % name] = round(statistics.median(ms), 3) if ms else None
        out["t_align_ms_%s_max" % name] = round(max(ms), 3) if ms else None
        out["sequence_ms_%s" % name] = round(wall, 1)
    pipe.time_align = False
    t_load = out.get("t_align_ms_under_load_median")
    if t_load and world == 1:
        # a LOWER BOUND only: the recurrence alone (n_chunks x t_align), ignoring the
        # pipeline fill, each rank's encode work and the baton hops -- ring_model is the
        # prediction of the 8-rank sequence time
        out["T8_chain_lower_bound_ms"] = round(n_chunks * t_load, 1)
        out["T1_over_8_ms"] = round(t1_ms / 8, 1)
        out["chain_lower_bound_frac_of_T1_over_8"] = round(n_chunks * t_load / (t1_ms / 8), 3)
        for name, ov_mode, r, _, _ in modes:
            t = out.get("t_align_ms_%s_median" % name)
            if ov_mode and t:
                out["chain_lower_bound_frac_%s" % name] = round(n_chunks * t / (out["sequence_ms_%s" % name] / 8), 3)
    return out


def _ring_model(model, pipe, seq, S, ov, rec, t1_ms):
    """The W-rank ring's sequence time predicted by the discrete-event model
    of aligned_vggt/dist/schedule.py from costs measured here on one GPU:
    core / dense encode jobs of g = 1..cap chunks (and the tail chunk), HIP
    events on one stream, median of 3 after a warm-up; t_align alone / beside
    a gated encode / ungated from the recurrence probe; the encode time one
    alignment costs its rank (t_pause) from the W = 1 overlapped sequences
    minus their plan's job time.  The baton hop and a moved alignment's ship
    are not measurable on one GPU: they are priced from their bytes at an
    assumed link rate, reported under ``assumed``.  T1 = this run's measured
    single-rank sequence."""
    import statistics
    from aligned_vggt.dist import schedule as SC
    from aligned_vggt.utils.data import generate_chunks
    chunks = generate_chunks(seq.shape[1], "chunk_overlap", S, ov)
    lengths = [len(c) for c in chunks]
    cap = pipe._group_cap(chunks, seq)
    cur = torch.cuda.current_stream()

    def timed(fn, reps=3):
        fn()
        ts = []
        for _ in range(reps):
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record(cur)
            r = fn()
            b.record(cur)
            b.synchronize()
            ts.append(a.elapsed_time(b))
        return statistics.median(ts), r

    core, dense = {}, {}
    shapes = [(lengths[0], g) for g in range(1, cap + 1)]
    if lengths[-1] != lengths[0]:
        shapes.append((lengths[-1], 1))
    with torch.no_grad():
        for fr, g in shapes:
            idx = [i for i, c in enumerate(chunks) if len(c) == fr][:g]
            x = torch.cat([seq[:, chunks[i]] for i in idx], 0)
            core[(fr, g)], enc = timed(lambda: model.encode_chunk(x, dense=False))
            dense[(fr, g)], _ = timed(lambda: model.encode_dense(dict(enc)))
            del enc
    # the two point-to-point transfers the model cannot measure on one GPU, priced from
    # their bytes: the baton (post-head overlap tokens (ov+1) x (P+1) x 1024 fp32, memory
    # tokens, last pose encoding) and a moved alignment's ship (the prefix rows S x (P+1)
    # x 1024 fp32 + the camera pose encoding), at an assumed effective 100 GB/s on one
    # xGMI link (153 GB/s peak) + 20 us per transfer
    H_img, W_img = seq.shape[-2:]
    P1 = (H_img // 14) * (W_img // 14) + 6
    nm = model.alignment_head.num_memory_tokens if getattr(model, "enable_memory", False) else 0
    baton_b = (ov + 1) * P1 * 1024 * 4 + nm * 512 * 4 + S * 9 * 4
    ship_b = S * P1 * 1024 * 4 + S * 9 * 4
    link = lambda b: round(b / 100e9 * 1e3 + 0.02, 3)  # noqa: E731
    costs = SC.RingCosts(core={k: round(v, 3) for k, v in core.items()},
                         dense={k: round(v, 3) for k, v in dense.items()},
                         t_align=rec["t_align_ms_under_load_median"] or 0.0,
                         t_align_alone=rec["t_align_ms_alone_median"] or 0.0, t_pause=0.0,
                         t_align_ungated=rec["t_align_ms_under_load_ungated_median"] or 0.0,
                         hop=link(baton_b), ship=link(ship_b),
                         source="bench.py --workload sequence on one MI355X (this line); hop / ship from "
                                "%.1f / %.1f MB at 100 GB/s + 20 us" % (baton_b / 1e6, ship_b / 1e6))
    # t_pause: what the overlapped W = 1 sequences spent beyond their plans' job time, per alignment
    n = len(lengths)
    for gated, seq_key in ((True, "sequence_ms_under_load"), (False, "sequence_ms_under_load_ungated")):
        plans, _ = SC.plan_ring(lengths, 1, costs, cap, pipe.plan_policies, (gated,))
        jobs_ms = sum(costs.job_ms(k, lengths[g[0]], len(g)) for k, g in plans[0].jobs)
        tp = max(0.0, (rec[seq_key] - costs.gather - jobs_ms) / n)
        if gated:
            costs.t_pause = round(tp, 3)
        else:
            costs.t_pause_ungated = round(tp, 3)
    pred = SC.predict_scaling(lengths, costs, offload=pipe.plan_offload)
    for W, d in pred.items():
        d["T1_over_TW"] = round(t1_ms / d["T_ms"], 2)
    w1, _ = SC.plan_ring(lengths, 1, costs, cap, pipe.plan_policies, (True,))
    return {"costs": costs.to_json(), "T1_measured_ms": round(t1_ms, 1), "predicted": pred,
            # NOT measured: the two point-to-point transfers, priced from their bytes (the first
            # 8-GPU run recalibrates them: VGGT_RING_COSTS=<its line> with measured hop / ship)
            "assumed": {"hop_ms": costs.hop, "baton_bytes": baton_b, "ship_ms": costs.ship, "ship_bytes": ship_b,
                        "link_GB_per_s": 100.0, "per_transfer_us": 20.0,
                        "offload_default": pipe.plan_offload},
            "check_w1_overlapped_gated": {"predicted_ms": round(SC.simulate(lengths, 1, w1, costs).total_ms, 1),
                                          "measured_ms": rec["sequence_ms_under_load"],
                                          "note": "t_pause is calibrated on this run, so this agrees by construction "
                                                  "up to the plan and alone-time terms"}}


def bench_point(args, world, rank, dev):
    """BASELINE configs[0]: one 8-frame 518 x 518 synthetic chunk through the
    point-aligned VGGT (pointAligned_wrapped_vggt.py:34-157: aggregator,
    point / depth DPT heads, camera head; a first chunk, so the Sim(3) is the
    identity, :96-98), random-init weights, per rank per step (replicas)."""
    import torch.distributed as dist
    from aligned_vggt import _native
    from aligned_vggt.models.pointAligned_wrapped_vggt import VGGT
    from aligned_vggt.utils.synthetic import condition_pose_outputs_, synthetic_images, synthetic_init_
    S, H, W = args.frames, args.height, W_IMG
    model = VGGT(enable_track=False)
    synthetic_init_(model, seed=0)
    condition_pose_outputs_(model)
    cpu_sd = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    model = model.to(dev).eval()
    imgs = synthetic_images(1, S, H, W, seed=1234 + rank, device=dev)
    timer = EventTimer({"global_attn"})
    _native.EVENT_HOOK = timer

    def step():
        return model(imgs, 0, None)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    timer.active = True
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    timer.active = False
    attn_ms = timer.mean_ms()
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
        dist.destroy_process_group()
    if rank != 0:
        return
    fl = agg_flops(S=S, H=H, W=W)
    value = args.steps * world / dt
    attn_tf = fl["global_attn_launch"] / (attn_ms * 1e-3) / 1e12 if attn_ms else None
    line = {
        "metric": "chunks/sec (%d-frame %dx%d) point-aligned VGGT chunk" % (S, H, W),
        "value": round(value, 4), "unit": "chunks/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (uniform [0,1) frames, random-init weights)",
        "config": {"workload": "point-aligned VGGT (aggregator bf16 + point / depth DPT heads + camera head fp32), "
                               "1 chunk of %d frames %dx%d" % (S, H, W), "baseline_config": 0, "frames": S,
                   "parallelism": "replicas x%d" % world},
        "tflops_per_gpu_aggregator": round(fl["total"] * value / world / 1e12, 1),
        "roofline": {"bound": "mfma", "kernel": "attn_fwd_kernel<64> (global attention, 1x16 heads x %d^2 x 64)"
                     % (S * (5 + (H // 14) * (W // 14))),
                     "achieved": round(attn_tf, 1) if attn_tf else None, "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(attn_tf / PEAK_BF16_TFLOPS, 4) if attn_tf else None,
                     "avg_launch_ms": round(attn_ms, 4) if attn_ms else None,
                     "flops_per_launch": fl["global_attn_launch"], "traffic": None},
    }
    if cpu_sd is not None:
        if args.cpu_runs > 0 and os.environ.get("VGGT_CPU_FULL_CHUNK") == "1":  # a whole chunk (~2 min)
            line["cpu_baseline"] = cpu_baseline_point(cpu_sd, S, H, W, args.cpu_threads, args.cpu_runs)
        else:
            line["cpu_baseline"] = cpu_baseline_point_sample(cpu_sd, S, H, W, args.cpu_threads)
        measured = _measured_row("C1", args.cpu_threads) if (S, H, W) == (8, 518, 518) else None
        if measured is not None:
            line["cpu_baseline"]["committed_whole_chunk_row"] = measured
    print(json.dumps(line), flush=True)


def cpu_baseline_point_sample(sd, S, H, W, threads: int):
    """BASELINE.md §3 row C1 as a bounded live sample (~20-30 s): the oracle's
    fp32 point-aligned VGGT pieces at the full chunk shape -- patch embed, one
    DINOv2 / frame / global block (each x24), the point and depth DPT heads on
    2 of the S frames (the DPT convolutions are per frame: x S/2), the camera
    head -- summed to one chunk."""
    import statistics
    from oracle import vggt_oracle as O
    from aligned_vggt.utils.synthetic import synthetic_images
    torch.set_num_threads(threads)
    hw = (H // 14) * (W // 14)
    P = 5 + hw
    g = torch.Generator().manual_seed(0)
    imgs = synthetic_images(1, S, H, W, seed=1234)
    x = torch.randn(S, P, 1024, generator=g)
    pos = O.position_grid(S, H // 14, W // 14, 5)
    toks = [torch.randn(1, S, P, 2048, generator=g) for _ in range(4)]

    def timed(fn, n=1):
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return statistics.median(ts)

    with torch.no_grad():
        O.block(sd, "aggregator.frame_blocks.0.", x[:2], 16, pos[:2], "2d", True)  # warm-up
        t_patch = timed(lambda: O.dinov2(sd, "aggregator.patch_embed.", imgs[0], False, depth=0))
        t_dino = timed(lambda: O.block(sd, "aggregator.patch_embed.blocks.0.", x, 16, eps=1e-6))
        t_frame = timed(lambda: O.block(sd, "aggregator.frame_blocks.0.", x, 16, pos, "2d", True))
        t_glob = timed(lambda: O.block(sd, "aggregator.global_blocks.0.", x.view(1, S * P, 1024), 16,
                                       pos.view(1, -1, 2), "2d", True))
        t2 = [t[:, :2] for t in toks]
        t_pt = timed(lambda: O.dpt_head(sd, "point_head.", t2, imgs[:, :2], 5, "inv_log"))
        t_dp = timed(lambda: O.dpt_head(sd, "depth_head.", t2, imgs[:, :2], 5, "exp"))
        t_cam = timed(lambda: O.camera_head(sd, toks))
    sec = t_patch + 24 * (t_dino + t_frame + t_glob) + (S / 2) * (t_pt + t_dp) + t_cam
    return {"value": 1.0 / sec, "unit": "chunks/s", "cores": threads, "kind": "port", "host_cpu": _cpu_model(),
            "host_logical_cpus": os.cpu_count(),
            "sample": f"oracle fp32 CPU point-aligned VGGT at {S}x{H}x{W}: patch embed {t_patch:.2f} s, DINOv2 / "
                      f"frame / global block {t_dino:.2f} / {t_frame:.2f} / {t_glob:.2f} s (x24 each), point / "
                      f"depth DPT heads on 2 frames {t_pt:.2f} / {t_dp:.2f} s (x{S / 2:g}), camera head "
                      f"{t_cam:.2f} s -> {sec:.1f} s per chunk"}


def cpu_baseline_point(sd, S, H, W, threads: int, runs: int):
    """the oracle's fp32 point-aligned VGGT (reference
    numerics) on one full 8-frame 518^2 chunk on the host cores: one warm-up
    pass at reduced depth (page-in, thread pool), then ``runs`` timed full
    chunks, median."""
    import statistics
    from oracle import alignment_oracle as AO
    from aligned_vggt.utils.synthetic import synthetic_images
    torch.set_num_threads(threads)
    imgs = synthetic_images(1, S, H, W, seed=1234)
    ts = []
    with torch.no_grad():
        t0 = time.perf_counter()
        AO.point_aligned_forward(sd, imgs[:, :2], 0, None,
                                 agg_kwargs={"keep": (0, 1, 2, 3), "depth": 4, "dino_depth": 1})
        warm = time.perf_counter() - t0
        for _ in range(max(1, runs)):
            t0 = time.perf_counter()
            AO.point_aligned_forward(sd, imgs, 0, None)
            ts.append(time.perf_counter() - t0)
    med = statistics.median(ts)
    return {"value": 1.0 / med, "unit": "chunks/s", "cores": threads, "kind": "port", "host_cpu": _cpu_model(),
            "host_logical_cpus": os.cpu_count(),
            "sample": f"oracle fp32 CPU point-aligned VGGT, one full {S}-frame {H}x{W} chunk (aggregator 24+24+24 "
                      f"blocks, point + depth DPT heads, camera head): warm-up {warm:.1f} s (2 frames, reduced depth), "
                      f"{len(ts)} timed run(s) {[round(x, 1) for x in ts]} s, median {med:.1f} s/chunk"}


def bench_train(args, world, rank, dev):
    """Alignment-head training step (train_featureAlignedVGGT_vkitti.yaml: only
    alignment_head.* trains, aggregator / camera / depth frozen): chunk 1
    (first chunk) and chunk 2 (overlap tokens + memory from chunk 1) through
    the head, a loss on both chunks' Sim(3) / SE(3) outputs and chunk 2's
    memory, backward through the HIP training kernels, AdamW step.  The frozen
    encoders' outputs (layer-23 tokens, (1, S, P, 2048) fp32) are synthetic and
    resident in HBM.  Data-parallel over ranks (gradient all-reduce over RCCL
    at N > 1, as Lightning DDP does)."""
    import torch.distributed as dist
    from aligned_vggt.heads.alignment_head import AlignmentHead
    from aligned_vggt.utils.synthetic import synthetic_init_
    H, W = args.height, W_IMG
    S, ov = args.frames, args.overlap
    P = 5 + (H // 14) * (W // 14)
    head = AlignmentHead(in_dim=2048, num_memory_tokens=8).to(dev).train()
    synthetic_init_(head, seed=0)
    # fused AdamW (one multi-tensor kernel per step instead of torch's foreach
    # chain); VGGT_ADAMW_FUSED=0 selects the foreach implementation for A/B
    fused = os.environ.get("VGGT_ADAMW_FUSED", "1") != "0"
    opt = torch.optim.AdamW(head.parameters(), lr=5e-5, weight_decay=0.05, fused=fused)
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    toks = [torch.randn(1, S, P, 2048, device=dev, generator=g) for _ in range(2)]
    wcs = torch.randn(1, 1, 8, device=dev, generator=g)
    wfs = torch.randn(1, S - 1, 7, device=dev, generator=g)

    def fwd_bwd():
        cs1, fs1, m1, o1 = head(toks[0], (H, W), ov)
        cs2, fs2, m2, _ = head(toks[1], (H, W), ov, overlap_tokens=o1, memory_tokens=m1)
        loss = ((cs1 + cs2) * wcs).sum() + ((fs1 + fs2) * wfs).sum() + m2.square().sum()
        opt.zero_grad(set_to_none=True)
        loss.backward()
        return loss

    # VGGT_TRAIN_GRAPH=1: the ~2,000-launch forward + backward as one HIP graph
    # (runtime.GraphedStep; all-reduce, clipping and the fused AdamW eager between
    # replays).  Off by default: 79.4 ms graphed vs 78.7 ms eager per step
    # (profiles/r6a) -- the gaps between the step's kernels are device-side
    graphed = os.environ.get("VGGT_TRAIN_GRAPH", "0") == "1"
    if graphed:
        from aligned_vggt.runtime import GraphedStep
        fwd_bwd = GraphedStep(fwd_bwd, modules=[head], warmup=2, device=dev)

    def step():
        fwd_bwd()
        if world > 1:  # one bucketed all-reduce of every gradient over RCCL (DDP semantics: mean)
            grads = [p.grad for p in head.parameters() if p.grad is not None]
            flat = torch.cat([g.reshape(-1) for g in grads])
            dist.all_reduce(flat)
            flat /= world
            off = 0
            for g_ in grads:
                g_.copy_(flat[off:off + g_.numel()].view_as(g_))
                off += g_.numel()
        torch.nn.utils.clip_grad_norm_(head.parameters(), 1.0)
        opt.step()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
        dist.destroy_process_group()
    if rank == 0:
        value = 2 * world * args.steps / dt
        print(json.dumps({
            "metric": "chunks/sec (%d-frame %dx%d) alignment-head training (fwd+bwd+AdamW)" % (S, H, W),
            "value": round(value, 4), "unit": "chunks/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic (resident encoder tokens)",
            "config": {"workload": "train", "frames": S, "overlap": ov, "image": [H, W],
                       "chunks_per_step": 2, "parallelism": "dp%d" % world, "hip_graph": graphed}}), flush=True)


def bench_selftest(args, world, rank):
    """CPU / gloo check of the multi-rank path end to end (launcher ->
    torch.distributed.run -> N ranks -> ChunkPipeline baton ring ->
    max-over-ranks timing -> one JSON line from rank 0) with the toy model of
    tests/toy_model.py; no GPU is touched."""
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from toy_model import C, DEC, NMEM, P1, ToyAlignModel
    from aligned_vggt.dist.pipeline import ChunkPipeline
    from aligned_vggt.utils.data import generate_chunks
    if world > 1:
        dist.init_process_group("gloo")
    g = torch.Generator().manual_seed(0)
    seq = torch.rand(2, args.seq_frames, 3, 4, 5, generator=g)
    pipe = ChunkPipeline(ToyAlignModel(), device=torch.device("cpu"), gather_dense=True)
    run = lambda: pipe.run(seq, args.frames, args.overlap, token_dims=(P1, C), memory_shape=(2, NMEM, DEC))  # noqa
    for _ in range(args.warmup):
        run()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = run()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
        dist.destroy_process_group()
    if rank == 0:
        n = len(generate_chunks(args.seq_frames, "chunk_overlap", args.frames, args.overlap))
        print(json.dumps({"metric": "selftest chunks/sec (toy model, CPU gloo)", "value": round(n * args.steps / dt, 4),
                          "unit": "chunks/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
                          "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
                          "config": {"workload": "selftest", "seq_frames": args.seq_frames, "frames": args.frames,
                                     "overlap": args.overlap},
                          "checksum": {k: round(float(v.double().sum()), 6) for k, v in out.items()}}), flush=True)


if __name__ == "__main__":
    main()
