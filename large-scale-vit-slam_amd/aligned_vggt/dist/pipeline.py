"""Sequence drivers: the reference's single-process chunk loop and a
multi-GPU chunk pipeline.

``apply_sequence_to_model`` restates training_metrics.py:616-659: chunk the
sequence (data.py:155), run the model chunk by chunk threading ``context``,
offload older chunk outputs to host memory, merge the per-chunk lists with
overlap removal (data.py:54-87).

``ChunkPipeline`` is the MI355X-native multi-GPU form (one process per GPU,
torch.distributed; backend "nccl" = RCCL over xGMI on ROCm, "gloo" for CPU
tests).  The per-chunk work splits into

  * ``encode_chunk``: aggregator + camera/depth/point heads -- ~99% of the
    FLOPs and independent of every other chunk; chunk i is encoded on rank
    i % world, all ranks in parallel;
  * ``align_chunk``: alignment head + Sim(3) composition -- a strict
    recurrence (chunk i consumes chunk i-1's post-head overlap tokens, memory
    tokens and aligned poses, featureAligned_vggt.py:88-90,126).

The recurrence state (the "baton": overlap tokens (B, ov+1, P+1, 1024) fp32
~28 MB, memory (B, 8, 512), last pose encoding (B, S, 9)) travels rank to rank
with point-to-point send/recv: one hop per chunk boundary over one xGMI link
(~0.2 ms), hidden behind the next chunk's encode.  Each rank interleaves
encode(own chunk k) -> align(own chunk k) so that, with align << encode, the
baton ring never stalls an encode.  At the end the small per-chunk outputs
(pose encodings, Sim(3)/SE(3) alignments) reach every rank through one
fixed-shape ``all_gather_into_tensor`` (RCCL over xGMI); dense depth maps stay
on the rank that produced them unless ``gather_dense`` (a second all-gather).
"""
from __future__ import annotations

import contextlib
import os
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..utils.data import alignAndConvertOutputs, chunk_batch, generate_chunks, moveDictListItemToCPU, wait_host_copies


def apply_sequence_to_model(batch: dict, model, chunk_width, num_overlap, sample_mode: str = "chunk_overlap",
                            alignment_type: Optional[str] = None) -> dict:
    """training_metrics.py:616-659 (no_grad inference chunk loop): chunk the
    sequence, thread ``context`` through the model, offload older chunk
    outputs to host memory, then align (GT-based, optional) and merge the
    per-chunk lists into overlap-free tensors in place (data.py:108-153).
    ``batch`` gains the merged ground-truth tensors, as in the reference."""
    S = batch["images"].shape[1]
    chunk_width = chunk_width[0] if isinstance(chunk_width, (list, tuple)) else chunk_width
    num_overlap = num_overlap[0] if isinstance(num_overlap, (list, tuple)) else num_overlap
    indices = generate_chunks(S, sample_mode, chunk_width, num_overlap)
    chunked = chunk_batch(batch, indices)
    predictions = None
    pending: list = []  # host copies in flight (pinned, side stream), waited for before the merge
    # forward == align_chunk(encode_chunk(.)) (featureAligned_vggt.py): consecutive
    # equal-length chunks share one encode, as in ChunkPipeline (same results);
    # VGGT_ENCODE_GROUP=1 keeps the reference's plain per-chunk model(...) call
    encode_group = int(os.environ.get("VGGT_ENCODE_GROUP", "3"))
    grouped = encode_group > 1 and hasattr(model, "encode_chunk") and hasattr(model, "align_chunk") \
        and torch.is_tensor(batch["images"]) and batch["images"].is_cuda
    if grouped and hasattr(model, "_check_frozen") and model.alignment_head.trainable():
        model._check_frozen()  # forward()'s guard, which this path bypasses
    groups = _encode_groups([len(c) for c in indices], batch["images"], model, encode_group) if grouped else []
    encs: dict = {}
    gi = 0
    for i in range(len(indices)):
        gt = chunked["extrinsics"][i] if sample_mode in ("chunk_gt", "two_chunks") else None
        with torch.no_grad():
            if not grouped:
                predictions = model(chunked["images"][i], num_overlap, predictions, gt_poses=gt)
            else:
                if i not in encs:
                    g = groups[gi]
                    gi += 1
                    if len(g) == 1:
                        encs[i] = model.encode_chunk(chunked["images"][i])
                    else:
                        B = chunked["images"][i].shape[0]
                        xs = torch.cat([chunked["images"][j] for j in g], 0)
                        encs.update(zip(g, _split_batch(model.encode_chunk(xs), B, len(g))))
                predictions = model.align_chunk(encs.pop(i), num_overlap, predictions, gt_poses=gt)
        moveDictListItemToCPU(predictions, -2, pending)
    moveDictListItemToCPU(predictions, -1, pending)
    wait_host_copies(pending)
    alignAndConvertOutputs(predictions, batch, chunked, alignment_type, chunk_width, num_overlap)
    return predictions


# token rows per grouped encode (VGGT_GROUP_TOKENS for A/B): 2 chunks of 16 x 518^2
# frames (configs[2] 683 -> 644 ms per 5 chunks, profiles/r4/encode_groups.md) or
# encode_group (3) chunks of 16 x 154x518
GROUP_TOKENS = int(os.environ.get("VGGT_GROUP_TOKENS", "49152"))


def _encode_groups(lengths: List[int], images: torch.Tensor, model, encode_group: Optional[int] = None
                   ) -> List[List[int]]:
    """Runs of consecutive equal-length chunks encoded together (at most
    encode_group chunks and GROUP_TOKENS token rows per encode)."""
    if encode_group is None:
        encode_group = int(os.environ.get("VGGT_ENCODE_GROUP", "3"))
    B, H, W = images.shape[0], images.shape[-2], images.shape[-1]
    agg = getattr(model, "aggregator", None)
    ps = getattr(agg, "patch_size", 14)
    ps = ps[0] if isinstance(ps, (tuple, list)) else int(ps)
    P = (H // ps) * (W // ps) + int(getattr(agg, "patch_start_idx", 5))  # + camera and register tokens
    groups: List[List[int]] = []
    for i, n in enumerate(lengths):
        cap = min(max(1, encode_group), max(1, GROUP_TOKENS // (B * n * P)))
        if groups and len(groups[-1]) < cap and lengths[groups[-1][-1]] == n:
            groups[-1].append(i)
        else:
            groups.append([i])
    return groups


def _split_batch(enc: dict, B: int, n: int) -> List[dict]:
    """Split an encode_chunk result over n chunks stacked along the batch
    dimension (n * B) back into n per-chunk results (views)."""
    outs: List[dict] = [{} for _ in range(n)]
    for k, v in enc.items():
        if torch.is_tensor(v) and v.dim() > 0 and v.shape[0] == n * B:
            for c in range(n):
                outs[c][k] = v[c * B:(c + 1) * B]
        elif isinstance(v, (list, tuple)) and v and all(torch.is_tensor(t) and t.dim() > 0 and t.shape[0] == n * B
                                                         for t in v):
            for c in range(n):
                outs[c][k] = [t[c * B:(c + 1) * B] for t in v]
        else:
            for c in range(n):
                outs[c][k] = v
    return outs


def _record_stream(obj, stream) -> None:
    """Mark every device tensor in obj (dict / list nesting) as used on
    ``stream`` so the caching allocator keeps it until that stream is done."""
    if torch.is_tensor(obj):
        if obj.is_cuda:
            obj.record_stream(stream)
    elif isinstance(obj, dict):
        for v in obj.values():
            _record_stream(v, stream)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            _record_stream(v, stream)


def _overlap_of(S: int, num_overlap: int) -> int:
    """featureAligned_vggt.py:93."""
    return num_overlap if S > num_overlap else S - 1


class ChunkPipeline:
    """Run a whole sequence through ``model`` with chunks spread over the
    ranks of ``group`` (see module docstring).  ``model`` must provide
    ``encode_chunk(images)`` and ``align_chunk(enc, num_overlap, context)``
    (FeatureAlignedVGGT does) and be replicated on every rank."""

    def __init__(self, model, group=None, device=None, gather_dense: bool = False,
                 encode_group: Optional[int] = None, overlap_align: Optional[bool] = None,
                 time_align: bool = False, short_workgroups: Optional[bool] = None,
                 gate_encode: Optional[bool] = None):
        self.model = model
        # one rank: align chunk i on the side stream while the next encode group
        # runs (the ring's planned schedule with the baton kept on the device; the
        # planner picks the ungated form there).  Default since round 5: the W = 1
        # sequence 1,245 -> 1,194 ms (configs[3]), 1,252 -> 1,194 ms (configs[4]),
        # 634 -> 631 ms (configs[2]) against the sequential loop, whose results it
        # matches bitwise (profiles/r10/c3.json, tests/test_gpu_pipeline.py).
        # VGGT_OVERLAP_ALIGN=0: the sequential loop.  time_align: HIP events around
        # every align_chunk on its stream (align_ms()).
        if overlap_align is None:
            overlap_align = os.environ.get("VGGT_OVERLAP_ALIGN", "1") == "1"
        self.overlap_align = overlap_align
        self.time_align = time_align
        # reserve_cus: the encodes run on a stream masked off that many CUs (spread
        # over the XCDs), so the alignment recurrence's kernels never queue behind a
        # full-chip encode launch; VGGT_ALIGN_RESERVE_CUS sets the default (0: off)
        self.reserve_cus = int(os.environ.get("VGGT_ALIGN_RESERVE_CUS", "0"))
        # short_workgroups: the ring's encodes (and, ungated, its alignments) run on
        # dedicated streams configured for short workgroups (vggt_set_stream_config: no
        # persistent GEMM forms, whose one-workgroup-per-CU grids hold every CU for a
        # whole launch).  Ungated that took t_align beside an encode 7.6 -> 5.4 ms per
        # 154x518 chunk; with the gate below it no longer helps (3.6 vs 3.7 ms) and costs
        # the encode 7 %, so it is off by default.  VGGT_RING_SHORT_WG=1.
        if short_workgroups is None:
            short_workgroups = os.environ.get("VGGT_RING_SHORT_WG", "0") == "1"
        self.short_workgroups = short_workgroups
        # gate_encode: in the ring's schedule the encode stream pauses at its yield points
        # (between transformer blocks, before each head) while an alignment runs
        # (runtime.EncodeGate: one signal word, hipStreamWriteValue32 / hipStreamWaitValue32),
        # so the alignment -- the recurrence's critical path -- runs alone after at most one
        # yield interval of sharing.  VGGT_RING_GATE=0 turns it off.
        if gate_encode is None:
            gate_encode = os.environ.get("VGGT_RING_GATE", "1") != "0"
        self.gate_encode = gate_encode
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.device = device
        self.gather_dense = gather_dense
        # encode_group: up to this many consecutive equal-length chunks encoded
        # together as one batch (encode_chunk is context-free; every kernel on it
        # is row- or (batch, head)-local), capped at GROUP_TOKENS token rows per
        # encode.  Small chunks (154x518: 6,592 token rows, fc2 = 140 GEMM tiles
        # on 256 CUs) fill the GPU poorly one at a time: configs[3] 1637 ->
        # 1415-1466 ms per 43 chunks in groups of 3; 518^2 chunks in pairs: the
        # GEMM / attention rounds quantise better (profiles/r4/encode_groups.md).
        # On W > 1 ranks a group is a run of the rank's OWN consecutive chunks
        # (i, i + W, ...).  VGGT_ENCODE_GROUP sets the default.
        if encode_group is None:
            encode_group = int(os.environ.get("VGGT_ENCODE_GROUP", "3"))
        self.encode_group = max(1, encode_group)
        # the ring's planner (dist/schedule.py) may choose, per rank, where the DPT heads
        # run ("with" the encode, "lag" one group behind, at the "end") and whether the
        # rank's encode is gated; these restrict its choices
        self.plan_policies = tuple(os.environ.get("VGGT_RING_POLICIES", "with,lag,end").split(","))
        self.plan_gates = (True, False)
        # alignments moved off their owner ride a second process group (ships) between
        # the same rank pairs as the batons; the model credits them only 1.7-3 % at
        # W = 8, priced at an assumed link speed, and their progress
        # relies on RCCL's p2p kernels co-residing with the persistent encode kernels.
        # Off by default until a measured 8-GPU run shows it pays: VGGT_RING_OFFLOAD=1.
        self.plan_offload = os.environ.get("VGGT_RING_OFFLOAD", "0") == "1"
        # device-memory bound on the ring's plans: the core results a rank holds for a
        # later DPT job ("end" / "lag" policies) stay under this many bytes
        # (dist/schedule.py plan_ring max_held); VGGT_RING_HELD_GB
        self.held_budget = float(os.environ.get("VGGT_RING_HELD_GB", "24")) * (1 << 30)
        self._local = None
        self.prediction = None

    # ------------------------------------------------------------ lifetime
    def close(self) -> None:
        """Release what the pipeline owns on the device: the encode gate's
        signal word.  Its HIP streams are process-wide (runtime.shared_stream),
        reused by every pipeline with the same configuration."""
        gate = self.__dict__.pop("_gate", None)
        if gate is not None:
            gate.close()
        self.__dict__.pop("_enc_streams", None)
        self.__dict__.pop("_align_streams", None)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    # ----------------------------------------------------- frame transfer
    def _fetch(self, images: torch.Tensor, idx):
        """Frames of one chunk on the device.  Host frames go through a pinned
        staging copy on a side stream, so the transfer overlaps the chunk in
        flight instead of stalling the launch thread (a synchronous pageable
        copy left the GPU idle ~10-25 ms per chunk, profiles r3h)."""
        x = images[:, idx]
        dev = torch.device(self.device) if self.device is not None else x.device
        if x.device == dev:
            return (x, None, None)
        if dev.type != "cuda" or x.device.type != "cpu":
            return (x.to(dev), None, None)
        xp = x.pin_memory()
        side = self.__dict__.get("_side")
        if side is None:
            side = self._side = torch.cuda.Stream(dev)
        # allocated on the side stream (the copy's producer): a block allocated on
        # the compute stream could be one whose previous contents queued compute
        # kernels still read, and the side-stream copy is not ordered after them;
        # _ready's record_stream covers the consumer side
        with torch.cuda.stream(side):
            xd = torch.empty(xp.shape, dtype=xp.dtype, device=dev)
            xd.copy_(xp, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(side)
        return (xd, ev, xp)

    @staticmethod
    def _ready(f):
        xd, ev, _ = f
        if ev is not None:
            torch.cuda.current_stream(xd.device).wait_event(ev)
            xd.record_stream(torch.cuda.current_stream(xd.device))
        return xd

    # ---------------------------------------------------------- baton I/O
    def _baton_shapes(self, B: int, S_prev: int, ov_prev: int, P1: int, C: int, mem):
        shapes = {"overlap_tokens": (B, ov_prev + 1, P1, C), "pose_enc": (B, S_prev, 9)}
        if mem is not None:
            shapes["memory_tokens"] = mem
        return shapes

    @property
    def _comm_device(self):
        """Where the collectives' tensors live: the GPU for RCCL; host memory
        for gloo (CPU tests, and the single-GPU multi-process GPU test, where
        every baton is staged through the host)."""
        dev = torch.device(self.device) if self.device is not None else torch.device("cpu")
        if dev.type == "cuda" and dist.is_initialized() and dist.get_backend(self.group) == "gloo":
            return torch.device("cpu")
        return dev

    def _isend(self, ctx: dict, dst: int, keys):
        """Post the baton's tensors to ``dst`` (RCCL: on its own stream, after
        the current stream's queued work); returns (works, tensors) -- the
        tensors must stay alive until the works complete."""
        cd = self._comm_device
        ts = [(ctx[k][-1] if isinstance(ctx[k], list) else ctx[k]).contiguous().to(cd) for k in keys]
        ops = [dist.P2POp(dist.isend, t, dst, group=self.group) for t in ts]
        return dist.batch_isend_irecv(ops), ts

    def _irecv(self, src: int, shapes: Dict[str, tuple], group=None):
        out = {k: torch.empty(shp, device=self._comm_device, dtype=torch.float32) for k, shp in shapes.items()}
        ops = [dist.P2POp(dist.irecv, t, src, group=self.group if group is None else group) for t in out.values()]
        return dist.batch_isend_irecv(ops), out

    def _p2p_warmup(self, baton_pairs=None, ship_pairs=()):
        """Create the ring's point-to-point communicators up front (RCCL builds
        a pair's communicator on its first send/recv, blocking both hosts until
        the peer joins -- inside the timed loop that would stall the enqueue of
        the next encode).  baton_pairs: (src, dst) rank pairs the batons travel
        (default r -> r + 1); ship_pairs: those that carry offloaded
        alignments' inputs, on their own process group (so a ship and a baton
        between the same two ranks are never matched against each other)."""
        if self.world == 1:
            return
        W, r = self.world, self.rank
        if baton_pairs is None:
            baton_pairs = [(q, (q + 1) % W) for q in range(W)]
        key = (tuple(sorted(set(baton_pairs))), tuple(sorted(set(ship_pairs))))
        done = self.__dict__.setdefault("_p2p_done", set())
        if ship_pairs and self.__dict__.get("_ship_group") is None:
            ranks = dist.get_process_group_ranks(self.group) if self.group is not None else list(range(W))
            # local synchronisation: only the ring's own ranks make this call (the ring may
            # run on a subgroup of a larger job, whose other ranks never get here)
            self._ship_group = dist.new_group(ranks=ranks, backend=dist.get_backend(self.group),
                                              use_local_synchronization=True)
        for pairs, grp in ((key[0], self.group), (key[1], self.__dict__.get("_ship_group"))):
            if not pairs or (pairs, id(grp)) in done:
                continue
            ops, keep = [], []
            for src, dst in pairs:  # the same canonical order on every rank
                if src == dst or r not in (src, dst):
                    continue
                t = torch.zeros(1, device=self._comm_device)
                keep.append(t)
                ops.append(dist.P2POp(dist.isend if r == src else dist.irecv, t, dst if r == src else src, group=grp))
            if ops:
                for w in dist.batch_isend_irecv(ops):
                    w.wait()
            done.add((pairs, id(grp)))

    # ---------------------------------------------------------------- run
    @torch.no_grad()
    def run(self, images: torch.Tensor, chunk_width: int, num_overlap: int, token_dims=None,
            memory_shape=None) -> Optional[dict]:
        """images: (B, N, 3, H, W) (any device; each rank moves only its
        chunks).  token_dims = (P+1, C) of the alignment head's tokens;
        memory_shape = (B, n_mem, dec) or None.  Returns the merged predictions
        on every rank (pose_enc (B,N,9), chunk_sim3_alignment_enc (B,n_chunks,8),
        frame_se3_alignment_enc (B,sum(S_i-1),7), and depth if gathered)."""
        B, Nf = images.shape[:2]
        chunks = generate_chunks(Nf, "chunk_overlap", chunk_width, num_overlap)
        keys = ["overlap_tokens", "pose_enc"] + (["memory_tokens"] if memory_shape is not None else [])
        self.align_events = []
        dense: Dict[int, dict] = {}
        if self.world == 1 and not self.overlap_align:
            mine = self._run_local(images, chunks, num_overlap, keys, memory_shape, B)
        elif ((self.reserve_cus > 0 or self.short_workgroups or self.gate_encode) and self.device is not None
              and torch.device(self.device).type == "cuda"):
            enc_stream = self._encode_stream()
            cur = torch.cuda.current_stream(self.device)
            enc_stream.wait_stream(cur)
            with torch.cuda.stream(enc_stream):
                mine, dense = self._run_ring(images, chunks, num_overlap, keys, token_dims, memory_shape, B)
            cur.wait_stream(enc_stream)
            for v in list(mine.values()) + list(dense.values()):
                _record_stream(v, cur)
        else:
            mine, dense = self._run_ring(images, chunks, num_overlap, keys, token_dims, memory_shape, B)
        return self._gather(mine, dense, chunks, num_overlap, B)

    def prepare(self, images: torch.Tensor, chunk_width: int, num_overlap: int) -> None:
        """Compute (and cache) the ring's plans for this sequence shape ahead of
        ``run`` -- the planner's search is a few seconds of host time
        (dist/schedule.py), which the first ``run`` of a configuration would
        otherwise spend before its first launch."""
        if self.world == 1 and not self.overlap_align:
            return
        chunks = generate_chunks(images.shape[1], "chunk_overlap", chunk_width, num_overlap)
        cuda = self.device is not None and torch.device(self.device).type == "cuda"
        self.plans(chunks, images, cuda)

    def _encode_stream(self):
        """The ring's encode stream: a dedicated non-blocking HIP stream, or one
        masked off `reserve_cus` CUs, registered with the library
        (vggt_set_stream_config) so its persistent kernels size their grids to
        the CUs it can use and, with short_workgroups, it gets no persistent
        GEMM forms at all (runtime.shared_stream)."""
        from ..runtime import shared_stream
        return shared_stream(self.device, exclude_cus=self.reserve_cus, short_workgroups=self.short_workgroups)

    def _groups(self, chunks, own: List[int], images) -> List[List[int]]:
        """Encode groups over this rank's own chunks (runs of equal length)."""
        g = _encode_groups([len(chunks[i]) for i in own], images, self.model, self.encode_group)
        return [[own[j] for j in grp] for grp in g]

    def _group_cap(self, chunks, images) -> int:
        """Most chunks one encode may batch (encode_group, GROUP_TOKENS token rows)."""
        B, H, W = images.shape[0], images.shape[-2], images.shape[-1]
        agg = getattr(self.model, "aggregator", None)
        ps = getattr(agg, "patch_size", 14)
        ps = ps[0] if isinstance(ps, (tuple, list)) else int(ps)
        P = (H // ps) * (W // ps) + int(getattr(agg, "patch_start_idx", 5))
        n = max(len(c) for c in chunks)
        return max(1, min(self.encode_group, GROUP_TOKENS // (B * n * P)))

    def _held_chunk_bytes(self, chunks, images) -> int:
        """Device bytes one chunk's core result keeps while it waits for its DPT
        job: the kept aggregator layers (S, P, 2C) fp32, the alignment head's
        prefix rows (S, P + 1, C) fp32 and the frames."""
        B, H, W = images.shape[0], images.shape[-2], images.shape[-1]
        agg = getattr(self.model, "aggregator", None)
        ps = getattr(agg, "patch_size", 14)
        ps = ps[0] if isinstance(ps, (tuple, list)) else int(ps)
        P = (H // ps) * (W // ps) + int(getattr(agg, "patch_start_idx", 5))
        C = int(getattr(self.model, "embed_dim", 1024))
        S = max(len(c) for c in chunks)
        n_layers = len(getattr(self.model, "intermediate_layer_indices", (4, 11, 17, 23)))
        return 4 * B * S * (n_layers * P * 2 * C + (P + 1) * C + 3 * H * W)

    def plans(self, chunks, images, cuda: bool):
        """This ring's per-rank encode plans (dist/schedule.py ``plan_ring``:
        group sizes, where the DPT heads run, gated or not; cached per
        chunking).  VGGT_RING_PLAN=legacy: round 4's schedule (greedy groups of
        the cap, DPT inside each encode, every rank gated) for A/B."""
        from . import schedule as SC
        W = self.world
        lengths = [len(c) for c in chunks]
        cap = self._group_cap(chunks, images)
        defer = hasattr(self.model, "encode_dense") and getattr(self.model, "point_head", None) is None
        policies = tuple(self.plan_policies) if defer else ("with",)
        gates = tuple(self.plan_gates) if (cuda and self.gate_encode) else (False,)
        legacy = os.environ.get("VGGT_RING_PLAN", "auto") == "legacy"
        # alignments may run away from their chunk's owner when the model can ship
        # their inputs (the alignment head's prefix rows: FeatureAlignedVGGT in
        # no-grad inference with VGGT_ALIGN_PREFIX on)
        offload = self.plan_offload and W > 1 and hasattr(self.model, "ship_spec") and \
            self.model.ship_spec(images.shape[0], lengths[0], *images.shape[-2:]) is not None
        max_held = max(cap, int(self.held_budget // max(1, self._held_chunk_bytes(chunks, images))))
        key = (tuple(lengths), W, cap, policies, gates, legacy, offload, max_held)
        cache = self.__dict__.setdefault("_plan_cache", {})
        if key not in cache:
            costs = SC.load_costs()
            if legacy:
                plans = SC.legacy_plans(lengths, W, cap)
                for pl in plans:
                    pl.gated = gates[0]
                pred = SC.simulate(lengths, W, plans, costs)
            else:
                plans, pred = SC.plan_ring(lengths, W, costs, cap, policies, gates, offload=offload,
                                           max_held=max_held)
            cache[key] = (plans, pred)
        self.prediction = cache[key][1]
        plans = cache[key][0]
        ov = self.__dict__.get("align_rank_override")
        if ov is not None:  # tests: a fixed alignment placement instead of the planner's
            import dataclasses
            plans = [dataclasses.replace(pl, align_rank=tuple(ov)) for pl in plans]
        self._last_plans = plans
        return plans

    def _encode(self, images, chunks, g: List[int], frames, dense: bool = True):
        """One encode job over the chunks in g: (per-chunk results, the batched result)."""
        xs = [self._ready(f) for f in frames]
        B = xs[0].shape[0]
        kw = {} if dense else {"dense": False}
        if len(g) == 1:
            enc = self.model.encode_chunk(xs[0], **kw)
            return {g[0]: enc}, enc
        enc = self.model.encode_chunk(torch.cat(xs, 0), **kw)
        return dict(zip(g, _split_batch(enc, B, len(g)))), enc

    @staticmethod
    def _summary(pred: dict, S: int) -> dict:
        out = {"pose_enc": pred["pose_enc"][-1], "chunk_sim3": pred["chunk_sim3_alignment_enc"][:, -1:],
               "frame_se3": pred["frame_se3_alignment_enc"][:, -(S - 1):] if S > 1
               else pred["frame_se3_alignment_enc"][:, :0]}
        if "depth" in pred:
            out["depth"] = pred["depth"][-1]
            out["depth_conf"] = pred["depth_conf"][-1]
        return out

    def _ctx_from(self, ctx_in: dict, B: int, memory_shape) -> dict:
        ctx = {"overlap_tokens": ctx_in["overlap_tokens"], "pose_enc": [ctx_in["pose_enc"]],
               "chunk_sim3_alignment_enc": torch.zeros(B, 0, 8, device=self.device),
               "frame_se3_alignment_enc": torch.zeros(B, 0, 7, device=self.device)}
        if memory_shape is not None:
            ctx["memory_tokens"] = [ctx_in["memory_tokens"]]
        return ctx

    def _run_local(self, images, chunks, num_overlap, keys, memory_shape, B) -> Dict[int, dict]:
        """One rank: every chunk in order, the baton kept in memory; the next
        group's frames prefetched while the current group runs."""
        n = len(chunks)
        groups = self._groups(chunks, list(range(n)), images)
        fetch = lambda g: [self._fetch(images, chunks[i]) for i in g]  # noqa: E731
        nxt = fetch(groups[0]) if groups else None
        mine: Dict[int, dict] = {}
        encs: Dict[int, dict] = {}
        local = None
        gi = 0
        for i in range(n):
            if i not in encs:
                frames, g = nxt, groups[gi]
                gi += 1
                nxt = fetch(groups[gi]) if gi < len(groups) else None
                encs.update(self._encode(images, chunks, g, frames)[0])
            ctx = self._ctx_from(local, B, memory_shape) if i > 0 else None
            ev0 = self._tick()
            pred = self.model.align_chunk(encs.pop(i), num_overlap, ctx)
            if ev0 is not None:
                self.align_events.append((i, ev0, self._tick()))
            if i + 1 < n:
                local = {k: (pred[k][-1] if isinstance(pred[k], list) else pred[k]) for k in keys}
            mine[i] = self._summary(pred, len(chunks[i]))
        return mine

    def _align_stream(self, align_short: bool):
        """The high-priority stream alignments run on (cached)."""
        streams = self.__dict__.setdefault("_align_streams", {})
        side = streams.get(align_short)
        if side is None:
            lo, hi = torch.cuda.Stream.priority_range()
            if align_short:
                # a dedicated high-priority stream, also short-workgroup: beside an encode its
                # GEMMs' tiles go to whichever CUs free up first instead of one persistent
                # workgroup per CU that starts only when its CU does
                from ..runtime import shared_stream
                side = shared_stream(self.device, priority=hi, short_workgroups=True)
            else:
                side = torch.cuda.Stream(self.device, priority=hi)
            streams[align_short] = side
        return side

    def _gate_for(self, main, side, plan) -> object:
        """The encode gate of this rank, or None.  Only when the alignment
        stream outranks the encode stream: a gated wait then never sits in a
        hardware queue ahead of the alignment's end() write (runtime.EncodeGate)."""
        if not (self.gate_encode and plan.gated and main.cuda_stream != 0):
            return None
        from ..runtime import EncodeGate, stream_priority
        if not stream_priority(side) < stream_priority(main):
            return None
        gate = self.__dict__.get("_gate")
        if gate is None:
            gate = self._gate = EncodeGate(self.device)
        return gate

    def _run_ring(self, images, chunks, num_overlap, keys, token_dims, memory_shape, B):
        """Rank r encodes chunks r, r + W, ... (its encode stream runs the
        plan's jobs, dist/schedule.py: groups of its own chunks, the DPT heads
        with the encode or later) and aligns the chunks the plan gives it
        (``align_rank``: its own, minus those shipped to a less loaded rank,
        plus those shipped to it).  Each alignment runs on a high-priority
        side stream that waits (device-side) for the chunk's core encode -- or
        for its shipped inputs -- and for the baton from the rank that aligned
        chunk i - 1, and posts the baton to the rank that aligns chunk i + 1
        (isend) as soon as it is done: the host never blocks on a peer, and the
        compute stream keeps encoding while a baton is in flight.

        The baton's irecv is posted on the side stream BEFORE the side stream
        waits for the chunk's encode: RCCL orders its communication stream
        after the stream current at the call, so the receive can land while
        the encode still runs (posted after the wait it could not start until
        the encode had finished).  Under gloo ``w.wait()`` blocks the host
        instead, which only orders the launches.

        W == 1 (``overlap_align``): the same schedule on one GPU with the baton
        kept on the device -- chunk i aligns on the side stream while the next
        encode job runs on the compute stream.

        Returns (summaries of the chunks aligned here, raw DPT outputs of own
        chunks whose depth was not scaled by their alignment: a DPT head that
        ran after it, or an alignment shipped away -- scaled in ``_gather``)."""
        from .schedule import enqueue_order
        W, r = self.world, self.rank
        n = len(chunks)
        P1, C = token_dims
        cuda = self.device is not None and torch.device(self.device).type == "cuda"
        plan = self.plans(chunks, images, cuda)[r]
        ar = plan.align_rank or tuple(i % W for i in range(n))
        self._p2p_warmup([(ar[i - 1], ar[i]) for i in range(1, n) if ar[i - 1] != ar[i]],
                         [(i % W, ar[i]) for i in range(n) if ar[i] != i % W])
        own = list(range(r, n, W))
        self.enqueue_log = []  # ("job", kind, chunks) / ("ship", i) / ("align", i): the host's issue order (tests)
        side = main = None
        if cuda:
            # the alignment's own GEMMs: persistent when the encode is gated (the
            # alignment then has the GPU to itself after one yield interval), else short
            side = self._align_stream(self.short_workgroups and not (self.gate_encode and plan.gated))
            main = torch.cuda.current_stream(self.device)
        gate = self._gate_for(main, side, plan) if cuda else None
        encs: Dict[int, dict] = {}
        ready: Dict[int, object] = {}
        held: Dict[tuple, dict] = {}  # batched core results waiting for their DPT job
        dense: Dict[int, dict] = {}
        sends = []
        hw = tuple(images.shape[-2:])

        def run_job(j):
            kind, g = plan.jobs[j]
            self.enqueue_log.append(("job", kind, tuple(g)))
            if kind == "dense":
                benc = held.pop(tuple(g))
                self.model.encode_dense(benc)
                dk = {k: benc[k] for k in ("depth", "depth_conf") if k in benc}
                parts = [dk] if len(g) == 1 else _split_batch(dk, benc["images"].shape[0] // len(g), len(g))
                for i, p in zip(g, parts):
                    dense[i] = p
                return
            out, benc = self._encode(images, chunks, list(g), [self._fetch(images, chunks[i]) for i in g],
                                     dense=(kind == "enc"))
            if kind == "core":
                held[tuple(g)] = benc
            ev = None
            if cuda:
                ev = torch.cuda.Event()
                ev.record(main)
            for i in g:
                encs[i] = out[i]
                ready[i] = ev
                if kind == "enc" and ar[i] != r and "depth" in out[i]:
                    dense[i] = {k: out[i][k] for k in ("depth", "depth_conf") if k in out[i]}

        def ship(i):
            """Chunk i's alignment inputs to the rank that aligns it (in chunk order on
            both ends, on the ship group; RCCL: after the core encode on this stream)."""
            self.enqueue_log.append(("ship", i))
            enc = encs.pop(i)
            ready.pop(i, None)
            cd = self._comm_device
            ts = [t.contiguous().to(cd) for t in self.model.ship_payload(enc).values()]
            ops = [dist.P2POp(dist.isend, t, ar[i], group=self._ship_group) for t in ts]
            sends.append((dist.batch_isend_irecv(ops), ts))

        mine: Dict[int, dict] = {}
        gate_ctx = contextlib.nullcontext()
        if gate is not None:
            from ..runtime import gated
            gate_ctx = gated(main, gate)
        with gate_ctx:
            for kind, arg in enqueue_order(plan, own, r):
                if kind == "job":
                    run_job(arg)
                elif kind == "ship":
                    ship(arg[0])
                else:
                    self.enqueue_log.append(("align", arg[0]))
                    self._align_one(arg[0], ar, encs, ready, side, cuda, chunks, num_overlap, keys, B, P1, C,
                                    memory_shape, mine, sends, gate, hw)
        for works, _ in sends:
            for w in works:
                w.wait()
        if cuda:
            main.wait_stream(side)
            for v in list(mine.values()) + list(dense.values()):
                _record_stream(v, main)
        return mine, dense

    def _align_one(self, i, ar, encs, ready, side, cuda, chunks, num_overlap, keys, B, P1, C, memory_shape, mine,
                   sends, gate, hw) -> None:
        W, n, r = self.world, len(chunks), self.rank
        S = len(chunks[i])
        with (torch.cuda.stream(side) if cuda else contextlib.nullcontext()):
            ctx = None
            works = ()
            if i > 0 and ar[i - 1] != r:
                Sp = len(chunks[i - 1])
                works, ctx_in = self._irecv(ar[i - 1], self._baton_shapes(
                    B, Sp, _overlap_of(Sp, num_overlap), P1, C, memory_shape))
            if i % W == r:
                enc = encs.pop(i)
                if cuda:
                    side.wait_event(ready.pop(i))
                    _record_stream(enc, side)
            else:  # shipped here by its owner
                spec = self.model.ship_spec(B, S, *hw)
                sw, got = self._irecv(i % W, spec, group=self._ship_group)
                for w in sw:
                    w.wait()
                enc = self.model.enc_from_ship({k: v.to(self.device) for k, v in got.items()}, B, S, *hw)
            if i > 0:
                if ar[i - 1] != r:
                    for w in works:
                        w.wait()  # RCCL: the side stream waits; gloo: the host does
                    ctx_in = {k: v.to(self.device) for k, v in ctx_in.items()}  # no-op unless host-staged
                else:
                    ctx_in = self._local
                ctx = self._ctx_from(ctx_in, B, memory_shape)
            if gate is not None and hasattr(self.model, "prepare_align"):
                # whatever may synchronise the device (a HIP graph's first capture) happens
                # BEFORE the gate closes: a device-wide wait while it is held would wait for
                # the paused encode, which waits for the gate (runtime.EncodeGate)
                self.model.prepare_align(enc, num_overlap, ctx)
            if gate is not None:
                gate.begin(side)  # the encode stream pauses at its next yield point
            try:
                ev0 = self._tick()
                pred = self.model.align_chunk(enc, num_overlap, ctx)
                if ev0 is not None:
                    self.align_events.append((i, ev0, self._tick()))
            finally:
                if gate is not None:
                    gate.end(side)  # also on an error: a held gate would stall every later encode
            if i + 1 < n:
                if ar[i + 1] != r:
                    sends.append(self._isend(pred, ar[i + 1], keys))
                else:
                    self._local = {k: (pred[k][-1] if isinstance(pred[k], list) else pred[k]) for k in keys}
            mine[i] = self._summary(pred, S)

    def _tick(self):
        """A timing event on the current stream (``time_align`` on a HIP device), else None."""
        if not self.time_align or self.device is None or torch.device(self.device).type != "cuda":
            return None
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(self.device))
        return ev

    def align_ms(self) -> List[float]:
        """Per-chunk alignment time (ms, HIP events on the align stream) of the
        last ``run`` with ``time_align`` set; synchronises."""
        out = []
        for _, a, b in getattr(self, "align_events", []):
            b.synchronize()
            out.append(a.elapsed_time(b))
        return out

    def _gather(self, mine: Dict[int, dict], dense: Dict[int, dict], chunks: List[List[int]], num_overlap: int,
                B: int) -> Optional[dict]:
        """Every chunk's small outputs (pose encodings, chunk Sim(3), frame
        SE(3)) on every rank through ONE fixed-shape ``all_gather_into_tensor``
        (RCCL over xGMI), then the depth maps of chunks whose DPT head ran after
        their alignment (or whose alignment ran on another rank) scaled by their
        chunk Sim(3) on the owner (featureAligned_vggt.py:171), and with
        ``gather_dense`` the depth maps through a second one."""
        n = len(chunks)
        W = self.world
        # _collective_gather (tests): the collective form at W = 1 too, so one GPU runs
        # the RCCL all-gathers on device buffers (tests/test_gpu_pipeline.py)
        if W > 1 or self.__dict__.get("_collective_gather"):
            per_chunk = self._all_gather_chunks(mine, dense, chunks, B)
        else:
            per_chunk = mine
            for i, d in dense.items():
                per_chunk[i].update(self.model.scale_dense(d, per_chunk[i]["chunk_sim3"]))
        ov = num_overlap
        out = {
            "pose_enc": torch.cat([per_chunk[i]["pose_enc"][:, (ov if i > 0 else 0):] for i in range(n)], 1),
            "chunk_sim3_alignment_enc": torch.cat([per_chunk[i]["chunk_sim3"] for i in range(n)], 1),
            "frame_se3_alignment_enc": torch.cat([per_chunk[i]["frame_se3"] for i in range(n)], 1),
        }
        if all("depth" in per_chunk[i] for i in range(n)):
            out["depth"] = torch.cat([per_chunk[i]["depth"][:, (ov if i > 0 else 0):] for i in range(n)], 1)
            out["depth_conf"] = torch.cat([per_chunk[i]["depth_conf"][:, (ov if i > 0 else 0):] for i in range(n)], 1)
        return out

    def _all_gather_chunks(self, mine: Dict[int, dict], dense: Dict[int, dict], chunks: List[List[int]],
                           B: int) -> Dict[int, dict]:
        """Rank q's block of the small gather holds the chunks it aligned
        (align_rank) in chain order, each padded to the longest chunk; the
        dense gather holds the chunks it owns (i mod W), whose depth it has."""
        W, r = self.world, self.rank
        n = len(chunks)
        plan = self._last_plans[r]  # the plans this run executed
        ar = plan.align_rank or tuple(i % W for i in range(n))
        aligned = [[i for i in range(n) if ar[i] == q] for q in range(W)]
        slot_of = {i: (q, j) for q in range(W) for j, i in enumerate(aligned[q])}
        slots = max(1, max(len(a) for a in aligned))
        smax = max(len(c) for c in chunks)
        dev = self._comm_device
        # small outputs, per slot: [pose_enc B*smax*9, chunk_sim3 B*8, frame_se3 B*(smax-1)*7]
        seg = (0, B * smax * 9, B * 8, B * (smax - 1) * 7)
        per = sum(seg)
        buf = torch.zeros(slots, per, device=dev, dtype=torch.float32)
        for j, i in enumerate(aligned[r]):
            S, m = len(chunks[i]), mine[i]
            o = seg[0]
            buf[j, o:o + B * S * 9] = m["pose_enc"].reshape(-1).to(dev)
            o += seg[1]
            buf[j, o:o + B * 8] = m["chunk_sim3"].reshape(-1).to(dev)
            o += seg[2]
            buf[j, o:o + B * (S - 1) * 7] = m["frame_se3"].reshape(-1).to(dev)
        allb = torch.empty(W * slots, per, device=dev, dtype=torch.float32)
        dist.all_gather_into_tensor(allb, buf, group=self.group)
        out_dev = torch.device(self.device) if self.device is not None else dev
        allb = allb.to(out_dev)
        per_chunk: Dict[int, dict] = {}
        for i in range(n):
            q, j = slot_of[i]
            row = allb[q * slots + j]
            S = len(chunks[i])
            o = seg[0]
            per_chunk[i] = {"pose_enc": row[o:o + B * S * 9].view(B, S, 9)}
            o += seg[1]
            per_chunk[i]["chunk_sim3"] = row[o:o + B * 8].view(B, 1, 8)
            o += seg[2]
            per_chunk[i]["frame_se3"] = row[o:o + B * (S - 1) * 7].view(B, S - 1, 7)
        # this rank's own depth maps: scaled by their alignment already, or now (deferred / shipped)
        own = list(range(r, n, W))
        local = {}
        for i in own:
            if i in dense:
                local[i] = self.model.scale_dense(dense[i], per_chunk[i]["chunk_sim3"].to(out_dev))
            elif i in mine and "depth" in mine[i]:
                local[i] = {"depth": mine[i]["depth"], "depth_conf": mine[i]["depth_conf"]}
        # the dense collective only when every chunk has a depth map and it was asked for:
        # one flag per rank (all agree), the DPT map size with it (14*(H//14) x 14*(W//14))
        hwf = torch.zeros(1, 3, device=dev, dtype=torch.float32)
        if self.gather_dense and all(i in local for i in own):
            hwf[0, 0] = 1.0
            if own:
                hwf[0, 1], hwf[0, 2] = float(local[own[0]]["depth"].shape[2]), float(local[own[0]]["depth"].shape[3])
        allf = torch.empty(W, 3, device=dev, dtype=torch.float32)
        dist.all_gather_into_tensor(allf, hwf, group=self.group)
        allf = allf.cpu()
        if bool((allf[:, 0] > 0).all()):
            H, Wd = int(allf[0, 1]), int(allf[0, 2])  # rank 0 owns chunk 0
            pix = H * Wd
            oslots = (n + W - 1) // W
            d = torch.zeros(oslots, 2, B * smax * pix, device=dev, dtype=torch.float32)
            for j, i in enumerate(own):
                S = len(chunks[i])
                d[j, 0, :B * S * pix] = local[i]["depth"].reshape(-1).to(dev)
                d[j, 1, :B * S * pix] = local[i]["depth_conf"].reshape(-1).to(dev)
            alld = torch.empty(W * oslots, 2, B * smax * pix, device=dev, dtype=torch.float32)
            dist.all_gather_into_tensor(alld, d, group=self.group)
            alld = alld.to(out_dev)
            for i in range(n):
                row = alld[(i % W) * oslots + i // W]
                S = len(chunks[i])
                per_chunk[i]["depth"] = row[0, :B * S * pix].view(B, S, H, Wd, 1)
                per_chunk[i]["depth_conf"] = row[1, :B * S * pix].view(B, S, H, Wd)
        return per_chunk
