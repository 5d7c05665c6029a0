"""Multi-process (gloo, CPU) tests of the multi-GPU chunk pipeline: the
distributed schedule (chunk i encoded on rank i % W, alignment baton passed
rank to rank) must reproduce the single-process reference chunk loop
(training_metrics.py:616-659) exactly.  A small deterministic stand-in model
with the same encode/align/context protocol replaces the HIP model (which
needs a GPU)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from aligned_vggt.dist.pipeline import ChunkPipeline, apply_sequence_to_model
from aligned_vggt.dist.schedule import enqueue_order
from aligned_vggt.utils.data import generate_chunks
from toy_model import C, DEC, NMEM, P1, ToyAlignModel


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, Nf, w, ov, q, group=None, policies=None, shift=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(0)
        images = torch.rand(2, Nf, 3, 4, 5, generator=g)
        pipe = ChunkPipeline(ToyAlignModel(), device=torch.device("cpu"), gather_dense=True, encode_group=group)
        if policies is not None:
            pipe.plan_policies = policies
        if shift is not None:  # every alignment on another rank than its chunk's owner
            n = len(generate_chunks(Nf, "chunk_overlap", w, ov))
            pipe.align_rank_override = tuple((i + shift) % world for i in range(n))
        out = pipe.run(images, w, ov, token_dims=(P1, C), memory_shape=(2, NMEM, DEC))
        # the host's issue order against the plan's (dist/schedule.py enqueue_order)
        chunks = generate_chunks(Nf, "chunk_overlap", w, ov)
        plan = pipe.plans(chunks, images, False)[rank]
        expect = [("job",) + tuple(plan.jobs[a]) if k == "job" else (k, a[0])
                  for k, a in enqueue_order(plan, list(range(rank, len(chunks), world)), rank)]
        res = {k: v.numpy().copy() for k, v in out.items()}
        res["_order_ok"] = pipe.enqueue_log == expect
        res["_policies"] = sorted({kind for kind, _ in plan.jobs})
        res["_ships"] = sum(1 for e in pipe.enqueue_log if e[0] == "ship")
        # the end-of-sequence all-gather leaves the merged outputs on every rank
        q.put((rank, res))  # by value: the worker may exit first
    finally:
        dist.destroy_process_group()


def _sequential(Nf, w, ov):
    g = torch.Generator().manual_seed(0)
    images = torch.rand(2, Nf, 3, 4, 5, generator=g)
    return apply_sequence_to_model({"images": images}, ToyAlignModel(), [w, w], [ov, ov])


@pytest.mark.parametrize("world,Nf,w,ov,group", [(2, 14, 5, 1, None), (2, 64, 16, 4, None), (3, 23, 6, 2, None),
                                                 (4, 40, 8, 3, None), (2, 44, 6, 2, 1), (2, 44, 6, 2, 2),
                                                 (3, 60, 6, 2, 3), (5, 9, 5, 1, None),
                                                 # BASELINE configs[3]/[4] chunking: 512 frames, w16 / ov4 ->
                                                 # 43 chunks (a tail of 8) over 8 ranks
                                                 (8, 512, 16, 4, None)])
def test_pipeline_matches_sequential_loop(world, Nf, w, ov, group):
    """W ranks (isend/irecv baton ring, alignment on its own stream on GPUs,
    all_gather_into_tensor at the end), incl. grouped encodes of each rank's
    own consecutive chunks and a world larger than the chunk count."""
    _run_world(world, Nf, w, ov, group, None)


@pytest.mark.parametrize("world,policy", [(2, "with"), (2, "lag"), (2, "end"), (3, "lag"), (3, "end"), (8, "end")])
def test_pipeline_plan_policies(world, policy):
    """Every DPT placement of the ring's planner (with the encode, one group
    behind, all at the end -- the depth maps then scaled by the chunk Sim(3)
    after the alignment) gives the loop's results bitwise, and each rank
    issues its work exactly in the plan's enqueue order."""
    outs = _run_world(world, 512 if world == 8 else 44, 16 if world == 8 else 6, 4 if world == 8 else 2, None,
                      (policy,))
    for r, got in outs.items():
        assert got["_order_ok"], r
        assert got["_policies"] == (["enc"] if policy == "with" else ["core", "dense"]), (r, got["_policies"])


@pytest.mark.parametrize("world,Nf,w,ov,shift,policy", [(2, 44, 6, 2, 1, "end"), (3, 60, 6, 2, 1, "with"),
                                                      (3, 60, 6, 2, 2, "lag"), (4, 40, 8, 3, 1, "end")])
def test_pipeline_offloaded_alignments(world, Nf, w, ov, shift, policy):
    """Alignments away from their chunk's owner (dist/schedule.py offload): the
    owner ships the alignment's inputs on the ship process group, batons go
    between the aligning ranks, the depth maps are scaled by the owner after
    the small gather -- bitwise the loop's results, in the plan's issue order."""
    outs = _run_world(world, Nf, w, ov, None, (policy,), shift)
    assert sum(o["_ships"] for o in outs.values()) > 0


def _run_world(world, Nf, w, ov, group, policies, shift=None):
    ref = _sequential(Nf, w, ov)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, Nf, w, ov, q, group, policies, shift))
             for r in range(world)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert sorted(outs) == list(range(world))
    for r, got in outs.items():
        assert got["_order_ok"], r
        for k in ("pose_enc", "chunk_sim3_alignment_enc", "frame_se3_alignment_enc", "depth", "depth_conf"):
            assert got[k].shape == tuple(ref[k].shape), (r, k)
            torch.testing.assert_close(torch.from_numpy(got[k]), ref[k], rtol=0, atol=0)
    return outs


def test_pipeline_single_rank_matches_sequential_loop():
    ref = _sequential(20, 6, 2)
    g = torch.Generator().manual_seed(0)
    images = torch.rand(2, 20, 3, 4, 5, generator=g)
    got = ChunkPipeline(ToyAlignModel(), device=torch.device("cpu")).run(images, 6, 2, token_dims=(P1, C),
                                                                          memory_shape=(2, NMEM, DEC))
    for k in ("pose_enc", "chunk_sim3_alignment_enc", "frame_se3_alignment_enc", "depth"):
        torch.testing.assert_close(got[k], ref[k], rtol=0, atol=0)


@pytest.mark.parametrize("policy", ["with", "lag", "end"])
def test_pipeline_single_rank_overlapped_schedule_matches_sequential_loop(policy):
    """W = 1 with the ring's schedule (align on the side stream while the next
    encode job runs, baton kept locally): same results as the loop."""
    ref = _sequential(23, 6, 2)
    g = torch.Generator().manual_seed(0)
    images = torch.rand(2, 23, 3, 4, 5, generator=g)
    pipe = ChunkPipeline(ToyAlignModel(), device=torch.device("cpu"), gather_dense=True, encode_group=2,
                         overlap_align=True)
    pipe.plan_policies = (policy,)
    got = pipe.run(images, 6, 2, token_dims=(P1, C), memory_shape=(2, NMEM, DEC))
    for k in ("pose_enc", "chunk_sim3_alignment_enc", "frame_se3_alignment_enc", "depth", "depth_conf"):
        torch.testing.assert_close(got[k], ref[k], rtol=0, atol=0)


@pytest.mark.parametrize("group", [1, 2, 3, 5])
def test_pipeline_encode_groups_match_sequential_loop(group):
    """Grouped encode (consecutive equal-length chunks batched through
    encode_chunk) incl. a shorter tail chunk: bitwise equal to the loop."""
    ref = _sequential(23, 6, 2)
    g = torch.Generator().manual_seed(0)
    images = torch.rand(2, 23, 3, 4, 5, generator=g)
    got = ChunkPipeline(ToyAlignModel(), device=torch.device("cpu"), gather_dense=True, encode_group=group).run(
        images, 6, 2, token_dims=(P1, C), memory_shape=(2, NMEM, DEC))
    for k in ("pose_enc", "chunk_sim3_alignment_enc", "frame_se3_alignment_enc", "depth", "depth_conf"):
        torch.testing.assert_close(got[k], ref[k], rtol=0, atol=0)
