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
from aligned_vggt.models.featureAligned_vggt import merge_results

P1, C, NMEM, DEC = 7, 16, 3, 8


class ToyAlignModel:
    """Same protocol as FeatureAlignedVGGT (encode_chunk / align_chunk /
    forward + reference context semantics), tiny CPU arithmetic with a real
    dependence on the previous chunk's overlap tokens, memory and poses."""

    def encode_chunk(self, images):
        B, S = images.shape[:2]
        f = images.mean(dim=(2, 3, 4))  # (B, S)
        tok = f[:, :, None, None] * torch.arange(1, P1 * C + 1, dtype=torch.float32).view(1, 1, P1, C) / 100
        return {"images": images, "tok": tok, "depth": images[:, :, :1].permute(0, 1, 3, 4, 2) * 2,
                "depth_conf": images[:, :, 1] + 1}

    def align_chunk(self, enc, num_overlap, context=None):
        tok = enc["tok"].clone()
        B, S = tok.shape[:2]
        ov = num_overlap if S > num_overlap else S - 1
        if context is not None:
            prev = context["overlap_tokens"]
            tok = tok + prev.mean(dim=1, keepdim=True) * 0.5
            mem = context["memory_tokens"][-1] * 0.9 + tok.mean() * 0.1
            base = context["pose_enc"][-1][:, -ov:].mean(dim=1, keepdim=True)
        else:
            mem = torch.ones(B, NMEM, DEC)
            base = torch.zeros(B, 1, 9)
        pose = base + tok.mean(dim=(2, 3))[..., None] * torch.arange(9, dtype=torch.float32)
        sim3 = tok.mean(dim=(1, 2, 3))[:, None, None].expand(B, 1, 8).clone()
        fse3 = tok[:, 1:].mean(dim=(2, 3))[..., None].expand(B, S - 1, 7).clone()
        scale = sim3[..., -1]
        depth = enc["depth"] * scale.view(B, 1, 1, 1, 1)
        pred = {"overlap_tokens": torch.cat([tok[:, :1], tok[:, -ov:]], 1).contiguous()}
        if context is None:
            pred.update(pose_enc=[pose], chunk_sim3_alignment_enc=sim3, frame_se3_alignment_enc=fse3,
                        memory_tokens=[mem], depth=[depth], depth_conf=[enc["depth_conf"]])
        else:
            context.setdefault("pose_enc", []).append(pose)
            pred["pose_enc"] = context["pose_enc"]
            pred["chunk_sim3_alignment_enc"] = merge_results(context["chunk_sim3_alignment_enc"], sim3)
            pred["frame_se3_alignment_enc"] = merge_results(context["frame_se3_alignment_enc"], fse3)
            context.setdefault("memory_tokens", []).append(mem)
            pred["memory_tokens"] = context["memory_tokens"]
            for k, v in (("depth", depth), ("depth_conf", enc["depth_conf"])):
                context.setdefault(k, []).append(v)
                pred[k] = context[k]
        return pred

    def __call__(self, images, num_overlap, context=None, gt_poses=None):
        return self.align_chunk(self.encode_chunk(images), num_overlap, context)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, Nf, w, ov, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(0)
        images = torch.rand(2, Nf, 3, 4, 5, generator=g)
        out = ChunkPipeline(ToyAlignModel(), device=torch.device("cpu"), gather_dense=True).run(
            images, w, ov, token_dims=(P1, C), memory_shape=(2, NMEM, DEC))
        if rank == 0:
            q.put({k: v.clone() for k, v in out.items()})
        else:
            assert out is None
    finally:
        dist.destroy_process_group()


def _sequential(Nf, w, ov):
    g = torch.Generator().manual_seed(0)
    images = torch.rand(2, Nf, 3, 4, 5, generator=g)
    return apply_sequence_to_model({"images": images}, ToyAlignModel(), [w, w], [ov, ov])


@pytest.mark.parametrize("world,Nf,w,ov", [(2, 14, 5, 1), (2, 64, 16, 4), (3, 23, 6, 2), (4, 40, 8, 3)])
def test_pipeline_matches_sequential_loop(world, Nf, w, ov):
    ref = _sequential(Nf, w, ov)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, Nf, w, ov, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for k in ("pose_enc", "chunk_sim3_alignment_enc", "frame_se3_alignment_enc", "depth", "depth_conf"):
        assert got[k].shape == ref[k].shape, k
        torch.testing.assert_close(got[k], ref[k], rtol=0, atol=0)


def test_pipeline_single_rank_matches_sequential_loop():
    ref = _sequential(20, 6, 2)
    g = torch.Generator().manual_seed(0)
    images = torch.rand(2, 20, 3, 4, 5, generator=g)
    got = ChunkPipeline(ToyAlignModel(), device=torch.device("cpu")).run(images, 6, 2, token_dims=(P1, C),
                                                                          memory_shape=(2, NMEM, DEC))
    for k in ("pose_enc", "chunk_sim3_alignment_enc", "frame_se3_alignment_enc", "depth"):
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
