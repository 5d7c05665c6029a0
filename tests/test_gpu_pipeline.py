"""GPU checks of the chunk pipeline's stream concurrency (the multi-GPU ring's
schedule, dist/pipeline.py ``_run_ring``) on one MI355X.

The ring aligns chunk i on a high-priority side stream while the compute
stream encodes the next group.  With W = 1 and ``overlap_align`` the same code
path runs with the baton kept on the device, so everything the ring does with
streams -- ``wait_event`` on the encode events, ``record_stream`` of the encode
results, per-(device, stream) workspaces and split-K scratch, the camera
head's skinny fp32 linears running on the compute stream at the same time as
the alignment decoder's on the side stream -- is exercised here against the
plain sequential chunk loop (training_metrics.py:616-659)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from aligned_vggt import _native
    _native.lib()
    return torch.device("cuda")


def test_scratch_is_per_stream(cuda):
    """Split-K and training-reduction scratch must never be shared by two
    streams (a device-keyed slab let the side stream's decoder and
    the compute stream's camera head write the same partial sums)."""
    from aligned_vggt import _native as N
    from aligned_vggt.runtime import Workspace
    a = N._split_ws(cuda, 1 << 16)
    b_ = N._train_ws(cuda, 1 << 16)
    wa = Workspace.get(cuda).buf("x", 16, 16)
    s = torch.cuda.Stream(cuda)
    with torch.cuda.stream(s):
        a2 = N._split_ws(cuda, 1 << 16)
        b2 = N._train_ws(cuda, 1 << 16)
        wa2 = Workspace.get(cuda).buf("x", 16, 16)
    assert a.data_ptr() != a2.data_ptr()
    assert b_.data_ptr() != b2.data_ptr()
    assert wa.data_ptr() != wa2.data_ptr()
    assert N._split_ws(cuda, 1 << 16).data_ptr() == a.data_ptr()  # reused in stream order


def _model(cuda, monkeypatch, depth=4):
    from aligned_vggt.backbone.aggregator import Aggregator
    from aligned_vggt.models import featureAligned_vggt as FAmod
    from aligned_vggt.models.featureAligned_vggt import FeatureAlignedVGGT
    from aligned_vggt.utils.synthetic import condition_pose_outputs_, synthetic_init_
    monkeypatch.setattr(FAmod, "Aggregator", lambda **kw: Aggregator(depth=depth, dino_depth=1, **kw))
    m = FeatureAlignedVGGT(enable_point=False, enable_track=False, num_memory_tokens=8)
    m.intermediate_layer_indices = [0, 1, 2, 3]
    synthetic_init_(m, seed=21)
    condition_pose_outputs_(m)
    return m.to(cuda).eval()


@pytest.mark.parametrize("group,reserve,policy", [(1, 0, "with"), (3, 0, "with"), (3, 16, "with"), (2, 0, "lag"),
                                                  (3, 0, "end")])
def test_overlapped_schedule_matches_sequential_loop(cuda, monkeypatch, group, reserve, policy):
    """The side-stream schedule (align on its own stream, concurrent with the
    next encode job; optionally the encodes on a CU-masked stream; the DPT
    heads with each encode, one group behind or after every core -- then the
    depth maps are scaled after their alignment) is bitwise equal to the
    sequential chunk loop."""
    from aligned_vggt.dist.pipeline import ChunkPipeline, apply_sequence_to_model
    from aligned_vggt.utils.data import generate_chunks
    from aligned_vggt.utils.synthetic import synthetic_images
    m = _model(cuda, monkeypatch)
    N_, w, ov, H, W = 40, 8, 2, 56, 70
    imgs = synthetic_images(1, N_, H, W, seed=3).to(cuda)
    monkeypatch.setenv("VGGT_ENCODE_GROUP", str(group))
    ref = apply_sequence_to_model({"images": imgs}, m, [w], [ov], "chunk_overlap", None)
    P1 = 6 + (H // 14) * (W // 14)
    pipe = ChunkPipeline(m, device=cuda, gather_dense=True, encode_group=group, overlap_align=True, time_align=True)
    pipe.reserve_cus = reserve  # > 0: encodes on a stream masked off that many CUs
    pipe.plan_policies = (policy,)
    pipe.plan_gates = (True,)
    for _ in range(2):  # the second run reuses every per-stream buffer
        got = pipe.run(imgs, w, ov, token_dims=(P1, 1024), memory_shape=(1, 8, 512))
        torch.cuda.synchronize()
        for k in ("pose_enc", "chunk_sim3_alignment_enc", "frame_se3_alignment_enc", "depth", "depth_conf"):
            a, b = got[k].cpu(), ref[k].cpu()
            assert a.shape == b.shape, k
            assert torch.equal(a, b), (k, (a - b).abs().max().item())
    t = pipe.align_ms()
    n = len(generate_chunks(N_, "chunk_overlap", w, ov))
    assert len(t) == n and all(x > 0 for x in t), t
    assert pipe.__dict__.get("_gate") is not None  # the alignment stream outranks the encode stream: gated
    kinds = {k for _, k, _ in (e for e in pipe.enqueue_log if e[0] == "job")}
    assert kinds == ({"enc"} if policy == "with" else {"core", "dense"}), kinds
    print("align_chunk ms under concurrent encodes:", [round(x, 3) for x in t])
    pipe.close()


def test_gated_ring_with_align_graph(cuda, monkeypatch):
    """with VGGT_ALIGN_GRAPH=1 the first alignment of each shape
    captures a HIP graph, and capture synchronises the device.  The ring does
    that capture (prepare_align) before it closes the encode gate, so a gated
    encode never waits for a gate the host cannot release; results equal the
    sequential loop's eager path to fp32 round-off."""
    from aligned_vggt.dist.pipeline import ChunkPipeline, apply_sequence_to_model
    from aligned_vggt.models import featureAligned_vggt as FAmod
    from aligned_vggt.utils.synthetic import synthetic_images
    m = _model(cuda, monkeypatch)
    N_, w, ov, H, W = 30, 8, 2, 56, 70  # a shorter tail chunk: two graph shapes
    imgs = synthetic_images(1, N_, H, W, seed=12).to(cuda)
    ref = apply_sequence_to_model({"images": imgs}, m, [w], [ov], "chunk_overlap", None)
    monkeypatch.setattr(FAmod, "_ALIGN_GRAPH", True)
    P1 = 6 + (H // 14) * (W // 14)
    with ChunkPipeline(m, device=cuda, gather_dense=True, encode_group=2, overlap_align=True) as pipe:
        pipe.plan_gates = (True,)
        for _ in range(2):  # first run captures inside the ring, second replays
            got = pipe.run(imgs, w, ov, token_dims=(P1, 1024), memory_shape=(1, 8, 512))
            torch.cuda.synchronize()
        assert pipe.__dict__.get("_gate") is not None
    assert m.__dict__.get("_mi355x_align_graphs"), "no graph was captured"
    for k in ("pose_enc", "chunk_sim3_alignment_enc", "frame_se3_alignment_enc", "depth"):
        a, b = got[k].cpu(), ref[k].cpu()
        e = ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
        assert e < 1e-5, (k, e)


def test_pipeline_streams_are_shared(cuda):
    """pipelines must not leak HIP streams or the library's 16
    stream-configuration slots: their dedicated streams are process-wide per
    configuration (runtime.shared_stream), so 20 short-workgroup pipelines in
    a row use one encode and one alignment stream; the alignment stream
    outranks the encode stream (the gate's condition)."""
    from aligned_vggt.dist.pipeline import ChunkPipeline
    from aligned_vggt.runtime import stream_priority
    seen = set()
    for _ in range(20):
        pipe = ChunkPipeline(None, device=cuda, short_workgroups=True, gate_encode=False)
        s = pipe._encode_stream()
        side = pipe._align_stream(True)
        assert stream_priority(side) < stream_priority(s)
        seen.add((s.cuda_stream, side.cuda_stream))
        pipe.close()
    assert len(seen) == 1, seen


def test_pipeline_close_then_new_pipeline_reuses_shared_streams(cuda, monkeypatch):
    """The r9b fault: on the fdd8166 tree ``close()`` destroyed
    the pipeline's HIP streams while the caching allocator still held blocks
    handed out on them, and the next pipeline's run crashed (segfault in this
    file's overlapped-schedule test).  Streams are process-wide since 3eb7faf;
    this is the exact sequence: run, close, a second pipeline on the same
    shared streams, run again -- both bitwise the sequential loop."""
    from aligned_vggt.dist.pipeline import ChunkPipeline, apply_sequence_to_model
    from aligned_vggt.utils.synthetic import synthetic_images
    m = _model(cuda, monkeypatch)
    N_, w, ov, H, W = 20, 8, 2, 56, 70
    imgs = synthetic_images(1, N_, H, W, seed=5).to(cuda)
    ref = apply_sequence_to_model({"images": imgs}, m, [w], [ov], "chunk_overlap", None)
    P1 = 6 + (H // 14) * (W // 14)
    streams = []
    for _ in range(2):
        pipe = ChunkPipeline(m, device=cuda, gather_dense=True, encode_group=2, overlap_align=True)
        pipe.plan_gates = (True,)
        got = pipe.run(imgs, w, ov, token_dims=(P1, 1024), memory_shape=(1, 8, 512))
        streams.append(pipe._encode_stream().cuda_stream)
        pipe.close()
        del pipe
        torch.cuda.synchronize()
        for k in ("pose_enc", "chunk_sim3_alignment_enc", "frame_se3_alignment_enc", "depth"):
            assert torch.equal(got[k].cpu(), ref[k].cpu()), k
        del got
    assert streams[0] == streams[1]


def test_collective_gather_over_rccl_world1(cuda, monkeypatch):
    """the end-of-sequence gathers -- the small per-chunk slab,
    the dense-map flags and the dense depth maps (gather_dense) -- through
    ``all_gather_into_tensor`` on DEVICE buffers of an ``nccl`` (RCCL) process
    group, world size 1 on the one GPU of the test box.  Results equal the
    sequential loop bitwise (the gather only moves bytes)."""
    import socket

    import torch.distributed as dist
    from aligned_vggt.dist.pipeline import ChunkPipeline, apply_sequence_to_model
    from aligned_vggt.utils.synthetic import synthetic_images
    assert not dist.is_initialized()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=cuda if cuda.index is not None else torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        m = _model(cuda, monkeypatch)
        N_, w, ov, H, W = 20, 8, 2, 56, 70
        imgs = synthetic_images(1, N_, H, W, seed=8).to(cuda)
        ref = apply_sequence_to_model({"images": imgs}, m, [w], [ov], "chunk_overlap", None)
        P1 = 6 + (H // 14) * (W // 14)
        with ChunkPipeline(m, device=cuda, gather_dense=True, encode_group=2, overlap_align=True) as pipe:
            assert pipe.world == 1 and pipe._comm_device.type == "cuda"
            pipe._collective_gather = True
            calls = []
            real = dist.all_gather_into_tensor

            def spy(out, inp, group=None, **kw):
                calls.append((tuple(out.shape), out.device.type, inp.device.type))
                return real(out, inp, group=group, **kw)

            monkeypatch.setattr(dist, "all_gather_into_tensor", spy)
            got = pipe.run(imgs, w, ov, token_dims=(P1, 1024), memory_shape=(1, 8, 512))
            torch.cuda.synchronize()
        assert len(calls) == 3 and all(d == "cuda" and i == "cuda" for _, d, i in calls), calls
        for k in ("pose_enc", "chunk_sim3_alignment_enc", "frame_se3_alignment_enc", "depth", "depth_conf"):
            assert torch.equal(got[k].cpu(), ref[k].cpu()), k
    finally:
        dist.destroy_process_group()


def test_baton_p2p_batch_over_rccl_self():
    """VERDICT r5 missing #3: the baton's ``batch_isend_irecv`` of P2POps on an
    ``nccl`` (RCCL) group with DEVICE buffers, world size 1 -- the rank sends
    the baton's tensors to itself, sends and receives in ONE batch (RCCL pairs
    them in one group call), on the default group and on a second group made
    like the pipeline's ship group (``use_local_synchronization=True``).  The
    ring's two-device case stays for the driver's 8-GPU run."""
    import socket

    import torch.distributed as dist
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    assert not dist.is_initialized()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    try:
        ship = dist.new_group(ranks=[0], backend="nccl", use_local_synchronization=True)
        g = torch.Generator(device="cuda").manual_seed(0)
        P1 = 6 + 11 * 37
        baton = {"overlap_tokens": torch.randn(1, 5, P1, 1024, device=dev, generator=g),
                 "pose_enc": torch.randn(1, 16, 9, device=dev, generator=g),
                 "memory_tokens": torch.randn(1, 8, 512, device=dev, generator=g)}
        for grp in (None, ship):
            out = {k: torch.empty_like(v) for k, v in baton.items()}
            ops = [dist.P2POp(dist.isend, t, 0, group=grp) for t in baton.values()]
            ops += [dist.P2POp(dist.irecv, t, 0, group=grp) for t in out.values()]
            for w in dist.batch_isend_irecv(ops):
                w.wait()
            torch.cuda.synchronize()
            for k in baton:
                assert torch.equal(out[k], baton[k]), k
    finally:
        dist.destroy_process_group()
