"""The multi-GPU chunk pipeline's W > 1 ring (dist/pipeline.py ``_run_ring``)
carrying the real HIP model: two (or four) ranks on the one GPU of the test box (gloo
process group; each baton and the end-of-sequence all-gather are staged
through host memory, the rest -- encodes on the compute stream, alignment on
the high-priority side stream, graphs, per-stream workspaces -- is the RCCL
path's); also four ranks with the planner's offload placement.  Every rank
must return the single-process chunk loop's results
(training_metrics.py:616-659)."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

N_FRAMES, W_CHUNK, OV, H, W = 40, 8, 2, 56, 70


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model():
    from aligned_vggt.backbone.aggregator import Aggregator
    from aligned_vggt.models.featureAligned_vggt import FeatureAlignedVGGT
    from aligned_vggt.utils.synthetic import condition_pose_outputs_, synthetic_init_
    m = FeatureAlignedVGGT(enable_point=False, enable_track=False, num_memory_tokens=8)
    m.aggregator = Aggregator(depth=4, dino_depth=1)
    m.intermediate_layer_indices = [0, 1, 2, 3]
    synthetic_init_(m, seed=23)
    condition_pose_outputs_(m)
    return m.cuda().eval()


def _worker(rank, world, port, q, shift=None, offload=False):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "large-scale-vit-slam_amd")]
    import torch.distributed as dist
    from aligned_vggt.dist.pipeline import ChunkPipeline
    from aligned_vggt.utils.synthetic import synthetic_images
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = _model()
        imgs = synthetic_images(1, N_FRAMES, H, W, seed=4).cuda()
        pipe = ChunkPipeline(m, device=torch.device("cuda"), gather_dense=True, time_align=True)
        pipe.plan_offload = offload  # the planner's own placement of moved alignments (VGGT_RING_OFFLOAD=1)
        if shift is not None:  # every alignment away from its owner: the shipped prefix rows path
            from aligned_vggt.utils.data import generate_chunks
            n = len(generate_chunks(N_FRAMES, "chunk_overlap", W_CHUNK, OV))
            pipe.align_rank_override = tuple((i + shift) % world for i in range(n))
        P1 = 6 + (H // 14) * (W // 14)
        out = pipe.run(imgs, W_CHUNK, OV, token_dims=(P1, 1024), memory_shape=(1, 8, 512))
        torch.cuda.synchronize()
        ar = tuple(pipe._last_plans[0].align_rank) if pipe.__dict__.get("_last_plans") else ()
        q.put((rank, {k: v.cpu().numpy().copy() for k, v in out.items()}, pipe.align_ms(), ar))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,shift,offload", [(2, None, False), (2, 1, False), (4, None, True)])
def test_ring_two_ranks_real_model_matches_loop(world, shift, offload):
    """shift 1: every chunk's alignment runs on the other rank (its encode's
    alignment-head prefix rows and camera pose encoding shipped there, the
    depth maps scaled by the owner after the gather).  world 4 + offload
    (ADVICE r5): four ranks with the planner's OWN placement of moved
    alignments (7 chunks: 5 alignments move), so ships and batons between
    the same rank pairs interleave as they would on a node."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import torch.multiprocessing as mp
    from aligned_vggt.dist.pipeline import apply_sequence_to_model
    from aligned_vggt.utils.synthetic import synthetic_images
    m = _model()
    imgs = synthetic_images(1, N_FRAMES, H, W, seed=4).cuda()
    ref = apply_sequence_to_model({"images": imgs}, m, [W_CHUNK], [OV], "chunk_overlap", None)
    ref = {k: ref[k].cpu() for k in ("pose_enc", "chunk_sim3_alignment_enc", "frame_se3_alignment_enc", "depth")}
    del m
    torch.cuda.synchronize()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, shift, offload)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ars = {ar for _, _, _, ar in got}
    assert len(ars) == 1, ars  # every rank planned the same placement
    ar = ars.pop()
    if offload:
        moved = [i for i, a in enumerate(ar) if a != i % world]
        print("alignments moved off their owner:", moved, "placement", ar)
        assert moved, ar
    for rank, out, ms, _ in got:
        print(f"rank {rank}: align ms per own chunk {[round(x, 2) for x in ms]}")
        for k, b in ref.items():
            a = torch.from_numpy(out[k])
            assert a.shape == b.shape, (rank, k)
            e = ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
            print(f"rank {rank} {k}: rel-L2 vs the single-process loop {e:.2e}")
            assert e < 1e-5, (rank, k, e)
