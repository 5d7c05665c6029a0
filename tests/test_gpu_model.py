"""GPU parity of the full per-chunk FeatureAlignedVGGT forward (aggregator +
alignment head + camera head + DPT depth/point heads + Sim(3) composition) and
its multi-chunk ``context`` recurrence against the CPU oracle, through the
HIP C ABI."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import vggt_oracle as O  # noqa: E402


def _rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture(scope="module")
def models():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from aligned_vggt.models.featureAligned_vggt import FeatureAlignedVGGT
    from aligned_vggt.utils.synthetic import condition_pose_outputs_, synthetic_init_
    m = FeatureAlignedVGGT(enable_point=True, enable_track=False, num_memory_tokens=8)
    synthetic_init_(m, seed=11)
    condition_pose_outputs_(m)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    return m.cuda().eval(), sd


def test_state_dict_names_cover_reference_tree(models):
    m, sd = models
    for k in ("aggregator.camera_token", "aggregator.patch_embed.blocks.23.mlp.fc2.weight",
              "aggregator.global_blocks.23.attn.k_norm.bias", "camera_head.poseLN_modulation.1.weight",
              "camera_head.trunk.3.ls2.gamma", "depth_head.scratch.refinenet1.resConfUnit1.conv2.weight",
              "depth_head.resize_layers.3.weight", "depth_head.scratch.output_conv2.2.bias",
              "alignment_head.temporal_blocks.3.attn.k_norm.weight", "alignment_head.gated_update.gate_mlp.2.bias",
              "alignment_head.memory_token", "alignment_head.frame_proj.weight", "alignment_head.alpha",
              "point_head.projects.0.weight"):
        assert k in sd, k


@pytest.mark.parametrize("S,ov,H,W", [(3, 1, 56, 56), (4, 2, 42, 70)])
def test_feature_aligned_two_chunks(models, S, ov, H, W):
    m, sd = models
    from aligned_vggt.utils.synthetic import synthetic_images
    imgs = synthetic_images(1, 2 * S - ov, H, W, seed=5)
    chunks = O.generate_chunks(imgs.shape[1], S, ov)
    ref_ctx = ref32 = None
    got_ctx = None
    for ids in chunks:
        x = imgs[:, ids]
        ref_ctx = O.feature_aligned_forward(sd, x, ov, ref_ctx, enable_point=True, bf16=True)
        ref32 = O.feature_aligned_forward(sd, x, ov, ref32, enable_point=True, bf16=False)
        got_ctx = m(x.cuda(), ov, got_ctx)
    torch.cuda.synchronize()

    def errs(g, r):
        return {
            "chunk_sim3": _rel(g["chunk_sim3_alignment_enc"], r["chunk_sim3_alignment_enc"]),
            "frame_se3": _rel(g["frame_se3_alignment_enc"], r["frame_se3_alignment_enc"]),
            "pose_enc": max(_rel(a, b) for a, b in zip(g["pose_enc"], r["pose_enc"])),
            "depth": max(_rel(a, b) for a, b in zip(g["depth"], r["depth"])),
            "depth_conf": max(_rel(a, b) for a, b in zip(g["depth_conf"], r["depth_conf"])),
            "points": max(_rel(a, b) for a, b in zip(g["world_points"], r["world_points"])),
            "overlap_tokens": _rel(g["overlap_tokens"], r["overlap_tokens"]),
            "memory": max(_rel(a, b) for a, b in zip(g["memory_tokens"], r["memory_tokens"])),
        }
    r, g = ref_ctx, got_ctx
    assert len(g["pose_enc"]) == len(chunks)
    assert g["chunk_sim3_alignment_enc"].shape == r["chunk_sim3_alignment_enc"].shape
    e_hip = errs(g, r)            # HIP vs bf16-mixed reference emulation
    e_hip32 = errs(g, ref32)      # HIP vs the fp32 reference numerics
    e_ref = errs(r, ref32)        # the reference's own bf16-mixed deviation from fp32
    print("hip vs bf16 emulation", e_hip)
    print("hip vs fp32", e_hip32)
    print("ref bf16 vs fp32", e_ref)
    # Per-output bars vs the bf16-mixed emulation, about 2x the values measured on
    # MI355X (round 4: chunk_sim3 6.3e-4 / 6.1e-4, frame_se3 9.1e-4 / 9.4e-4, depth
    # 4.2e-4 / 2.9e-4, depth_conf 1.1e-5, overlap tokens 7.6e-3, memory 3.0e-3 /
    # 3.5e-3, points 1.3e-2 / 1.9e-2, pose_enc 1.6e-2 / 3.7e-2 for (3, 1) / (4, 2)),
    # the chunk Sim(3) at the north star's 1e-3.  Points and poses pass through
    # random-init camera / decoder weights that amplify token-level rounding (and,
    # at overlap 2, the Markley eigen-average of geometry.py:4-37), so they are
    # ALSO held to their distance from the fp32 numerics: within 2x (poses) /
    # 1.5x (points) of the reference's own bf16-vs-fp32 spread.
    bars = {"chunk_sim3": 1e-3, "frame_se3": 1e-3, "depth": 1.5e-3, "depth_conf": 5e-5, "overlap_tokens": 1.2e-2,
            "memory": 6e-3, "points": 3e-2, "pose_enc": 5e-2 if ov > 1 else 3e-2}
    for k, v in e_hip.items():
        assert v < bars[k], (k, v, bars[k], e_hip)
    assert e_hip32["pose_enc"] < 2.0 * e_ref["pose_enc"], (e_hip32, e_ref)
    assert e_hip32["points"] < 1.5 * e_ref["points"], (e_hip32, e_ref)


def test_heads_fp32_tier_tight(models):
    """Camera + depth heads consume the same (oracle-produced) aggregator
    tokens: both run fp32, so agreement is tight."""
    m, sd = models
    from aligned_vggt.utils.synthetic import synthetic_images
    imgs = synthetic_images(1, 3, 56, 70, seed=9)
    toks, psi = O.aggregator(sd, imgs, bf16=True)
    cam_ref = O.camera_head(sd, toks)[-1]
    d_ref, c_ref = O.dpt_head(sd, "depth_head.", toks, imgs, psi, "exp")
    tg = [t.cuda() for t in toks]
    cam = m.camera_head(tg)[-1]
    d, c = m.depth_head(tg, images=imgs.cuda(), patch_start_idx=psi)
    assert _rel(cam, cam_ref) < 1e-4
    assert _rel(d, d_ref) < 1e-4 and _rel(c, c_ref) < 1e-4


def test_dpt_presplit_bitwise(models):
    """The pre-split DPT path (each producer writes the split halves its consumer
    gathers) is bitwise equal to the register-staged split form; the fused
    output stage agrees to fp32 round-off."""
    m, sd = models
    from aligned_vggt.backbone import dpt_head as D
    from aligned_vggt.utils.synthetic import synthetic_images
    imgs = synthetic_images(1, 2, 56, 70, seed=4)
    toks, psi = O.aggregator(sd, imgs, bf16=True)
    tg = [t.cuda() for t in toks]
    prev = D.CONV_PRECISION, D.FUSE_UPSAMPLE_CONV
    try:
        outs = {}
        D.FUSE_UPSAMPLE_CONV = False
        for prec in ("bf16x3", "bf16x3pre"):
            D.CONV_PRECISION = prec
            outs[prec] = m.depth_head(tg, images=imgs.cuda(), patch_start_idx=psi)
        # the fused resize + conv output stage (vggt_conv2d_upsample_bf16x3): same
        # products, its interpolation compiled in another kernel -> fp32 round-off
        D.FUSE_UPSAMPLE_CONV = True
        outs["fused"] = m.depth_head(tg, images=imgs.cuda(), patch_start_idx=psi)
    finally:
        D.CONV_PRECISION, D.FUSE_UPSAMPLE_CONV = prev
    assert torch.equal(outs["bf16x3"][0], outs["bf16x3pre"][0])
    assert torch.equal(outs["bf16x3"][1], outs["bf16x3pre"][1])
    assert _rel(outs["fused"][0], outs["bf16x3pre"][0]) < 1e-6 and _rel(outs["fused"][1], outs["bf16x3pre"][1]) < 1e-6


def test_dpt_frame_groups_match(models, monkeypatch):
    """A chunk whose widest DPT map would pass the convolutions' 32-bit offsets
    runs in groups of frames: with the bound lowered so 3 frames
    split 2 + 1 (and B = 2 chunks split across the batch boundary), the outputs
    equal the one-launch form."""
    m, sd = models
    from aligned_vggt.backbone import dpt_head as D
    from aligned_vggt.utils.synthetic import synthetic_images
    imgs = synthetic_images(2, 3, 56, 70, seed=14)
    toks, psi = O.aggregator(sd, imgs, bf16=True)
    tg = [t.cuda() for t in toks]
    scale = torch.tensor([1.5, 0.75], device="cuda")
    full = m.depth_head(tg, images=imgs.cuda(), patch_start_idx=psi, _scale=scale)
    monkeypatch.setattr(D, "MAP_BYTES_LIMIT", 2 * 56 * 70 * 128 * 2 + 1)
    grouped = m.depth_head(tg, images=imgs.cuda(), patch_start_idx=psi, _scale=scale)
    for a, b in zip(grouped, full):
        assert a.shape == b.shape
        assert _rel(a, b) < 1e-6
    # and a single chunk (B = 1) past the bound
    one = m.depth_head([t[:1] for t in tg], images=imgs[:1].cuda(), patch_start_idx=psi, _scale=scale[:1])
    for a, b in zip(one, full):
        assert _rel(a, b[:1]) < 1e-6


def test_alignment_head_bf16_tier(models):
    m, sd = models
    from aligned_vggt.utils.synthetic import synthetic_images
    imgs = synthetic_images(1, 4, 42, 56, seed=3)
    toks, _ = O.aggregator(sd, imgs, bf16=True)
    ref = O.alignment_head(sd, toks[-1], (42, 56), 2, None, None, bf16=True)
    got = m.alignment_head(toks[-1].cuda(), (42, 56), 2)
    for name, a, b in zip(("chunk_sim3", "frame_se3", "memory", "overlap"), got, ref):
        assert _rel(a, b) < 2e-2, (name, _rel(a, b))
    ref2 = O.alignment_head(sd, toks[-1], (42, 56), 2, ref[3], ref[2], bf16=True)
    got2 = m.alignment_head(toks[-1].cuda(), (42, 56), 2, overlap_tokens=ref[3].cuda(), memory_tokens=ref[2].cuda())
    for name, a, b in zip(("chunk_sim3", "frame_se3", "memory", "overlap"), got2, ref2):
        assert _rel(a, b) < 2e-2, (name, _rel(a, b))


def test_feature_aligned_given_oracle_tokens(models, monkeypatch):
    """Feed the oracle's aggregator tokens into the HIP model: isolates the
    alignment head + heads + Sim(3) composition (per-component report)."""
    m, sd = models
    from aligned_vggt.utils.synthetic import synthetic_images
    S, ov, H, W = 4, 2, 42, 70
    imgs = synthetic_images(1, 2 * S - ov, H, W, seed=5)
    chunks = O.generate_chunks(imgs.shape[1], S, ov)
    ref_ctx = got_ctx = None
    for ids in chunks:
        x = imgs[:, ids]
        toks, psi = O.aggregator(sd, x, bf16=True)
        monkeypatch.setattr(m.aggregator, "forward", lambda images, keep_layers=None, t=toks: ([a.cuda() for a in t], 5))
        ref_ctx = O.feature_aligned_forward(sd, x, ov, ref_ctx, enable_point=True, bf16=True)
        got_ctx = m(x.cuda(), ov, got_ctx)
    for ci, (a, b) in enumerate(zip(got_ctx["pose_enc"], ref_ctx["pose_enc"])):
        a = a.cpu()
        print("chunk", ci, "T", _rel(a[..., :3], b[..., :3]), "quat", _rel(a[..., 3:7], b[..., 3:7]),
              "fov", _rel(a[..., 7:], b[..., 7:]))
        print("  got", a[0, :, :7])
        print("  ref", b[0, :, :7])
    print("sim3", _rel(got_ctx["chunk_sim3_alignment_enc"], ref_ctx["chunk_sim3_alignment_enc"]))
    for a, b in zip(got_ctx["pose_enc"], ref_ctx["pose_enc"]):
        assert _rel(a[..., 7:], b[..., 7:]) < 1e-5
        assert _rel(a[..., 3:7], b[..., 3:7]) < 2e-3
        assert _rel(a[..., :3], b[..., :3]) < 5e-3
    assert _rel(got_ctx["chunk_sim3_alignment_enc"], ref_ctx["chunk_sim3_alignment_enc"]) < 1e-3
    for a, b in zip(got_ctx["depth"], ref_ctx["depth"]):
        assert _rel(a, b) < 1e-3


def test_align_graph_survives_other_shapes(models):
    """A captured alignment-recurrence graph (featureAligned_vggt._AlignGraph)
    replayed after more graphs than torch's 32-stream pool holds were captured
    for larger patch grids, and after an eager run on yet another grid, must
    still give the eager recurrence's result: every table and scratch slab the
    graph reads has to outlive those (a one-entry RoPE-table cache and
    stream-keyed scratch shared with later captures did not)."""
    m, _ = models
    from aligned_vggt.models.featureAligned_vggt import _align_core
    head = m.alignment_head
    gen = torch.Generator().manual_seed(3)

    def core_in(H, W, S=4):
        P = head.patch_start_idx + (H // 14) * (W // 14)
        toks = (torch.randn(1, S, P, 2 * 1024, generator=gen) * 0.5).cuda()
        prep = head.prepare_infer(toks, (H, W))
        return (prep[:S * (P + 1)].view(1, S * (P + 1), -1), (1, S, P), (H, W), 2, None, None, None, None, False)

    a = core_in(42, 70)
    ref = [t.clone() for t in _align_core(head, *a) if t is not None]
    first = [t for t in m._align_graph(a) if t is not None]
    for k in range(6, 6 + 34):
        m._align_graph(core_in(42, 14 * k))
    _align_core(head, *core_in(28, 28))
    again = [t for t in m._align_graph(a) if t is not None]
    torch.cuda.synchronize()
    for r, f, g in zip(ref, first, again):
        assert _rel(f, r) < 1e-6, _rel(f, r)
        assert _rel(g, r) < 1e-6, _rel(g, r)


def _synthetic_w2c(S, seed=7):
    """Smooth synthetic trajectory (yaw random walk, ~1 unit forward per frame), w2c (1,S,3,4)."""
    g = torch.Generator().manual_seed(seed)
    yaw = torch.cumsum(torch.randn(S, generator=g) * 0.0087, 0)
    c2w = torch.eye(4).repeat(S, 1, 1)
    c2w[:, 0, 0], c2w[:, 0, 2], c2w[:, 2, 0], c2w[:, 2, 2] = yaw.cos(), yaw.sin(), -yaw.sin(), yaw.cos()
    c2w[:, :3, 3] = torch.cumsum(torch.stack([yaw.sin(), torch.zeros(S), yaw.cos()], -1), 0)
    return torch.linalg.inv(c2w)[:, :3, :][None]


def test_sequence_ate_rpe_parity(models):
    """Full-sequence evaluation (training_metrics.py:157-260 pose path): the
    HIP model through apply_sequence_to_model (3 overlapping chunks, GT scale
    alignment 'scale_from_poses') vs the oracle chunk loop; ATE / RPE of both
    against the same synthetic GT trajectory must agree."""
    m, sd = models
    from aligned_vggt.dist.pipeline import apply_sequence_to_model
    from aligned_vggt.eval import AbsoluteTrajectoryError, RelativePoseError, poses_c2w_from_predictions
    from aligned_vggt.utils import alignment as A
    from aligned_vggt.utils.synthetic import synthetic_images
    S, w, ov, H, W = 7, 4, 2, 42, 56
    imgs = synthetic_images(1, S, H, W, seed=12)
    extr = _synthetic_w2c(S)
    batch = {"images": imgs.cuda(), "extrinsics": extr.cuda()}
    got = apply_sequence_to_model(batch, m, [w], [ov], "chunk_overlap", "scale_from_poses")

    def oracle_seq(bf16):
        ctx = None
        for ids in O.generate_chunks(S, w, ov):
            ctx = O.feature_aligned_forward(sd, imgs[:, ids], ov, ctx, enable_point=True, bf16=bf16)
        pe = torch.cat([p[:, (ov if i else 0):] for i, p in enumerate(ctx["pose_enc"])], 1)
        pred = {"pose_enc": pe}
        A.scale_alignment_from_poses(pred, {"extrinsics": extr})
        return pred["pose_enc"]

    def metrics(pose_enc):
        p, g = poses_c2w_from_predictions(pose_enc.cpu(), extr, (H, W))
        ate, rpe = AbsoluteTrajectoryError(), RelativePoseError()
        ate.update(p[0], g[0])
        rpe.update(p[0], g[0])
        return {**ate.compute(), **rpe.compute()}

    assert got["pose_enc"].shape == (1, S, 9)
    pe_ref, pe_32 = oracle_seq(True), oracle_seq(False)
    pe_hip = got["pose_enc"].cpu()
    # the merged, GT-scale-aligned trajectory itself: translation / quaternion / FoV parts
    for sl, name in ((slice(0, 3), "t"), (slice(3, 7), "q"), (slice(7, 9), "fov")):
        e_hip, e_32 = _rel(pe_hip[..., sl], pe_ref[..., sl]), _rel(pe_32[..., sl], pe_ref[..., sl])
        print(f"pose_enc[{name}] rel vs bf16 oracle: hip {e_hip:.3e}  fp32 oracle {e_32:.3e}")
        assert e_hip < max(2e-2, 3 * e_32), (name, e_hip, e_32)
    m_hip, m_ref, m_32 = metrics(pe_hip), metrics(pe_ref), metrics(pe_32)
    print("hip", m_hip, "\nref bf16", m_ref, "\nref fp32", m_32)
    # ATE / RPE of a random-weight trajectory (RPE-rot ~90 deg) amplify the
    # pose differences above: the oracle's own metrics move by several % between
    # boxes (CPU thread count -> fp32 summation order), so the metric bar is 10%
    # (the metric code itself is pinned by golden fixtures, test_eval_alignment.py)
    for k in m_ref:
        spread = abs(m_32[k] - m_ref[k])
        assert abs(m_hip[k] - m_ref[k]) <= max(1e-1 * abs(m_ref[k]), 1.5 * spread) + 1e-6, (k, m_hip, m_ref, m_32)


def test_feature_aligned_batch2(models):
    """B = 2 (two independent sequences in one call): every stage keeps the
    batch elements apart (global attention per batch element, per-batch Sim(3)
    composition); each element must equal its own B = 1 run."""
    m, sd = models
    from aligned_vggt.utils.synthetic import synthetic_images
    S, ov, H, W = 3, 1, 42, 56
    a = synthetic_images(1, 2 * S - ov, H, W, seed=21)
    b = synthetic_images(1, 2 * S - ov, H, W, seed=22)
    both = torch.cat([a, b], 0)
    chunks = O.generate_chunks(both.shape[1], S, ov)
    ctx2 = ctxa = ctxb = None
    for ids in chunks:
        ctx2 = m(both[:, ids].cuda(), ov, ctx2)
        ctxa = m(a[:, ids].cuda(), ov, ctxa)
        ctxb = m(b[:, ids].cuda(), ov, ctxb)
    torch.cuda.synchronize()
    for key in ("chunk_sim3_alignment_enc", "frame_se3_alignment_enc"):
        assert _rel(ctx2[key][:1], ctxa[key]) < 1e-5 and _rel(ctx2[key][1:], ctxb[key]) < 1e-5, key
    for key in ("pose_enc", "depth"):
        for x2, xa, xb in zip(ctx2[key], ctxa[key], ctxb[key]):
            assert _rel(x2[:1], xa) < 1e-5 and _rel(x2[1:], xb) < 1e-5, key


@pytest.mark.parametrize("H,W,N,w,ov", [(42, 56, 14, 4, 1), (70, 56, 14, 4, 1), (518, 518, 28, 16, 4)])
def test_pipeline_grouped_encode_matches(models, H, W, N, w, ov):
    """ChunkPipeline's grouped encode (consecutive equal-length chunks through
    the aggregator / camera / depth heads as one batch) against one chunk at a
    time, incl. a shorter tail chunk that stays ungrouped: every kernel on the
    encode path is row- or (batch, head)-local, so the merged poses, Sim(3) /
    SE(3) encodings and depths must agree to fp32 round-off.  At 518^2 two
    16-frame chunks form one encode and the DPT head runs per chunk (its
    32-bit offset guard)."""
    m, _ = models
    from aligned_vggt.dist.pipeline import ChunkPipeline
    from aligned_vggt.utils.synthetic import synthetic_images
    imgs = synthetic_images(1, N, H, W, seed=21).cuda()
    P1 = 6 + (H // 14) * (W // 14)
    outs = {}
    for g in (1, 2, 3):
        outs[g] = ChunkPipeline(m, device=torch.device("cuda"), gather_dense=True, encode_group=g).run(
            imgs, w, ov, token_dims=(P1, 1024), memory_shape=(1, 8, 512))
    # host-resident frames: grouped chunks arrive through the pinned side-stream prefetch
    outs["host"] = ChunkPipeline(m, device=torch.device("cuda"), gather_dense=True, encode_group=3).run(
        imgs.cpu(), w, ov, token_dims=(P1, 1024), memory_shape=(1, 8, 512))
    for g in (2, 3, "host"):
        for k in ("pose_enc", "chunk_sim3_alignment_enc", "frame_se3_alignment_enc", "depth"):
            e = _rel(outs[g][k], outs[1][k])
            assert outs[g][k].shape == outs[1][k].shape, k
            assert e < 1e-5, (g, k, e)


# measured (round 4): 2.6e-6 for the split-bf16 convolutions, 4.6e-7 on exact fp32
@pytest.mark.parametrize("conv,reorder,tol", [("bf16x3pre", True, 1e-5), ("bf16x3pre", False, 1e-5),
                                              ("bf16x3", True, 1e-5), ("fp32", True, 2e-6)])
def test_dpt_matches_transformers_depth_anything(golden, monkeypatch, conv, reorder, tol):
    """HIP DPTHead (pos_embed off) vs the in-container transformers
    Depth-Anything neck + head run with the same weights (tests/golden/dpt_hf.npz,
    an independent third-party DPT: reassemble, layer*_rn, four fusion blocks with
    the in-place-ReLU residual units, align_corners=True resizes at rectangular
    sizes, output convs).  The depth channel's pre-activation is log(depth)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import numpy as np
    from aligned_vggt.backbone import dpt_head as D
    monkeypatch.setattr(D, "CONV_PRECISION", conv)
    monkeypatch.setattr(D, "REORDER_OUT_CONV", reorder)
    g = golden("dpt_hf")
    sd = {k[3:]: torch.from_numpy(np.ascontiguousarray(v)) for k, v in g.items() if k.startswith("sd.")}
    head = D.DPTHead(dim_in=256, features=64, out_channels=(32, 32, 64, 64), output_dim=2, activation="exp",
                     pos_embed=False, intermediate_layer_idx=range(4))
    head.load_state_dict(sd, strict=True)
    head = head.cuda()
    ph, pw = int(g["ph"]), int(g["pw"])
    tok = torch.from_numpy(g["tokens"])
    F_, hw, C = tok.shape
    toks = torch.cat([torch.full((F_, 5, C), 7.0), tok], 1).reshape(1, F_, 5 + hw, C).cuda()
    imgs = torch.zeros(1, F_, 3, ph * 14, pw * 14, device="cuda")
    depth, conf = head([toks] * 4, images=imgs, patch_start_idx=5)
    torch.cuda.synchronize()
    pre = torch.log(depth[0, ..., 0]).cpu()
    ref = torch.from_numpy(g["head_pre"][:, 0])
    e = _rel(pre, ref)
    print(f"DPT ({conv}, reorder={reorder}) vs transformers Depth-Anything: rel-L2 {e:.3e}")
    assert pre.shape == ref.shape and e < tol, e
