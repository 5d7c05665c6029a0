"""Oracle parity at the production shapes (reduced depth), where the code
paths that only switch on at size run composed:

  * the headline chunk, 1 x 16 x 518^2 (BASELINE configs[1]): 21,984 token
    rows -> 8-wave global attention, persistent GEMMs with the fused q/k-norm +
    RoPE and GELU epilogues, the fused residual-add + next-LayerNorm row pass;
  * the VKitti-shaped 154 x 518 sequence chunk (configs[3]/[4]: 16 frames,
    overlap 4, 6,592 token rows) through apply_sequence_to_model with a shorter
    tail chunk (featureAligned_vggt.py:93, data.py:188-190), memory on.

The CPU oracle runs the same reduced depth (~20-60 s on the box's cores)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import vggt_oracle as O  # noqa: E402


def _rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture(scope="module")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    return torch.device("cuda")


def test_aggregator_headline_chunk_reduced_depth(cuda):
    """Aggregator(depth=2, dino_depth=1) on one 16 x 518^2 chunk vs the oracle's
    bf16-mixed emulation (same tolerance as the small-shape tests)."""
    from aligned_vggt.backbone.aggregator import Aggregator
    from aligned_vggt.utils.synthetic import synthetic_images, synthetic_init_
    agg = Aggregator(depth=2, dino_depth=1)
    synthetic_init_(agg, seed=7)
    sd = {"aggregator." + k: v for k, v in agg.state_dict().items()}
    img = synthetic_images(1, 16, 518, 518, seed=1234)
    agg = agg.to(cuda)
    outs, psi = agg(img.to(cuda), keep_layers=(0, 1))
    torch.cuda.synchronize()
    outs = [o.cpu() for o in outs]
    with torch.no_grad():
        ref, psi_ref = O.aggregator(sd, img, bf16=True, keep=(0, 1), depth=2, dino_depth=1)
    assert psi == psi_ref == 5
    for o, r in zip(outs, ref):
        assert o.shape == r.shape == (1, 16, 1374, 2048)
        assert torch.isfinite(o).all()
        e = _rel(o, r)
        print("headline chunk layer rel-L2 vs bf16 oracle", e)
        assert e < 4e-3, e  # measured 1.7e-3 (round 3); 2x that, rounded up


def test_aggregator_headline_chunk_full_depth(cuda):
    """the headline config end to end -- the full HIP
    Aggregator (DINOv2 x 24, 24 frame + 24 global blocks, 21,984-token global
    attention) on one 16 x 518^2 chunk -- against the CPU oracle run at the
    same depth and size in both tiers (tests/golden/configs1_full.npz, a
    strided subsample of layers 4/11/17/23, made by
    tests/golden/gen_configs1_full.py; featureAligned_vggt.py:78-82).  bf16
    error compounding through 24 global-attention layers at nk = 21,984 (the
    offset-free softmax's range guard, P rounded to bf16, fp32 row sums over
    21,984 keys) is what this measures.  Bars per kept layer: the HIP output
    no further from the fp32 oracle, and from the bf16 oracle, than 1.25x the
    oracle's own bf16-vs-fp32 spread."""
    import numpy as np
    from aligned_vggt.backbone.aggregator import Aggregator
    from aligned_vggt.utils.synthetic import synthetic_images, synthetic_init_
    ref = np.load(os.path.join(os.path.dirname(__file__), "golden", "configs1_full.npz"))
    keep = tuple(int(x) for x in ref["keep"])
    frames = [int(x) for x in ref["frames"]]
    ts, cs = int(ref["token_stride"]), int(ref["channel_stride"])
    agg = Aggregator()
    synthetic_init_(agg, seed=int(ref["weight_seed"]))
    img = synthetic_images(1, 16, 518, 518, seed=int(ref["image_seed"]))
    agg = agg.to(cuda)
    with torch.no_grad():
        outs, psi = agg(img.to(cuda), keep_layers=keep)
    torch.cuda.synchronize()
    assert psi == 5 and len(outs) == len(keep)
    got = torch.stack([o[0, frames, ::ts, ::cs].float().cpu() for o in outs])
    del outs
    rb, rf = torch.from_numpy(ref["bf16"]), torch.from_numpy(ref["fp32"])
    assert got.shape == rb.shape, (got.shape, rb.shape)
    assert torch.isfinite(got).all()
    for li, layer in enumerate(keep):
        e_b, e_f, sp = _rel(got[li], rb[li]), _rel(got[li], rf[li]), _rel(rb[li], rf[li])
        print(f"configs[1] full depth, layer {layer}: hip vs bf16 oracle {e_b:.3e}, hip vs fp32 oracle {e_f:.3e}, "
              f"oracle bf16 vs fp32 {sp:.3e} (full tensor {float(ref['spread_full'][li]):.3e})")
        assert e_f <= 1.25 * sp, (layer, e_f, sp)
        assert e_b <= 1.25 * sp, (layer, e_b, sp)


def test_vkitti_sequence_with_tail_reduced_depth(cuda, monkeypatch):
    """36 frames of 154 x 518, chunk 16 / overlap 4 -> chunks [0-15], [12-27] and
    a 12-frame tail [24-35]: HIP model through apply_sequence_to_model (grouped
    encode of the two equal chunks, the tail alone) vs the oracle chunk loop."""
    from aligned_vggt.backbone.aggregator import Aggregator
    from aligned_vggt.dist.pipeline import apply_sequence_to_model
    from aligned_vggt.models.featureAligned_vggt import FeatureAlignedVGGT
    from aligned_vggt.utils.synthetic import condition_pose_outputs_, synthetic_images, synthetic_init_
    N, w, ov, H, W = 36, 16, 4, 154, 518
    chunks = O.generate_chunks(N, w, ov)
    assert [len(c) for c in chunks] == [16, 16, 12]
    from aligned_vggt.models import featureAligned_vggt as FAmod
    monkeypatch.setattr(FAmod, "Aggregator", lambda **kw: Aggregator(depth=4, dino_depth=1, **kw))
    m = FeatureAlignedVGGT(enable_point=False, enable_track=False, num_memory_tokens=8)
    m.intermediate_layer_indices = [0, 1, 2, 3]
    synthetic_init_(m, seed=13)
    condition_pose_outputs_(m)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(cuda).eval()
    imgs = synthetic_images(1, N, H, W, seed=31)
    got = apply_sequence_to_model({"images": imgs.to(cuda)}, m, [w], [ov], "chunk_overlap", None)
    torch.cuda.synchronize()
    agg_kw = {"keep": (0, 1, 2, 3), "depth": 4, "dino_depth": 1}

    def oracle(bf16):
        ctx = None
        with torch.no_grad():
            for ids in chunks:
                ctx = O.feature_aligned_forward(sd, imgs[:, ids], ov, ctx, bf16=bf16, agg_kwargs=agg_kw)
        return ctx

    ref, ref32 = oracle(True), oracle(False)
    pe_ref = torch.cat([p[:, (ov if i else 0):] for i, p in enumerate(ref["pose_enc"])], 1)
    pe_32 = torch.cat([p[:, (ov if i else 0):] for i, p in enumerate(ref32["pose_enc"])], 1)
    d_ref = torch.cat([d[:, (ov if i else 0):] for i, d in enumerate(ref["depth"])], 1)
    e = {"chunk_sim3": _rel(got["chunk_sim3_alignment_enc"], ref["chunk_sim3_alignment_enc"]),
         "frame_se3": _rel(got["frame_se3_alignment_enc"], ref["frame_se3_alignment_enc"]),
         "pose_T": _rel(got["pose_enc"][..., :3], pe_ref[..., :3]),
         "pose_fov": _rel(got["pose_enc"][..., 7:], pe_ref[..., 7:]),
         "depth": _rel(got["depth"], d_ref)}
    d_32 = torch.cat([d[:, (ov if i else 0):] for i, d in enumerate(ref32["depth"])], 1)
    e_ref = {"chunk_sim3": _rel(ref32["chunk_sim3_alignment_enc"], ref["chunk_sim3_alignment_enc"]),
             "frame_se3": _rel(ref32["frame_se3_alignment_enc"], ref["frame_se3_alignment_enc"]),
             "pose_T": _rel(pe_32[..., :3], pe_ref[..., :3]), "pose_fov": _rel(pe_32[..., 7:], pe_ref[..., 7:]),
             "depth": _rel(d_32, d_ref)}
    print("154x518 sequence: hip vs bf16 oracle", e, "oracle fp32 vs bf16", e_ref)
    assert got["pose_enc"].shape == (1, N, 9) and got["depth"].shape[:2] == (1, N)
    assert got["chunk_sim3_alignment_enc"].shape == (1, 3, 8)
    # north star on the Sim(3) chunk alignment; per-output bars about 2x the values
    # measured on MI355X (round 4: chunk_sim3 4.8e-4, frame_se3 8.0e-4, depth 1.4e-4,
    # pose T 5.6e-2, FoV 4.4e-2).  The poses pass through the random-init camera head,
    # which amplifies bf16 token rounding (the oracle's own bf16-vs-fp32 spread here:
    # T 5.6e-2, FoV 3.2e-2), so they are ALSO held within twice that spread.
    bars = {"chunk_sim3": 1e-3, "frame_se3": 1e-3, "depth": 5e-4, "pose_T": 1e-1, "pose_fov": 8e-2}
    for k, bar in bars.items():
        assert e[k] < bar, (k, e, bar)
    for k in ("pose_T", "pose_fov"):
        assert e[k] < 2.0 * e_ref[k], (k, e, e_ref)


def _configs2():
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_configs2", os.path.join(os.path.dirname(__file__), "golden",
                                                                               "gen_configs2.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _quat_rel(a, b):
    """rel-L2 of unit quaternions up to sign (q and -q are one rotation)."""
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    s = torch.sign((a * b).sum(-1, keepdim=True))
    s[s == 0] = 1
    return ((a * s - b).norm() / b.norm()).item()


def _report(name, e, spread):
    print(f"{name}: hip vs bf16 oracle " + ", ".join(f"{k} {v:.2e}" for k, v in e.items()))
    print(f"{name}: oracle fp32 vs bf16 " + ", ".join(f"{k} {v:.2e}" for k, v in spread.items()))


def test_alignment_head_at_configs2_size(cuda):
    """the AlignmentHead alone at configs[2]'s frame size --
    P + 1 = 1,375 tokens per frame (518^2), 16 frames: d=128 frame attention
    with nk = 1,375 tile tails, the temporal cross-attention over 1,375 raw-view
    groups of 16 queries (22,000 rows) -- on seeded tokens, a first chunk and a
    continuation chunk (overlap tokens + memory), vs the oracle's bf16-mixed
    emulation (tests/golden/configs2_head.npz, tests/golden/gen_configs2.py)."""
    import numpy as np
    G = _configs2()
    ref = np.load(os.path.join(os.path.dirname(__file__), "golden", "configs2_head.npz"))
    h = G.head_model().to(cuda).eval()
    tok0, tok1 = G.head_inputs()
    hw, ov, st = (G.HEAD["H"], G.HEAD["W"]), G.HEAD["ov"], G.TOK_STRIDE
    with torch.no_grad():
        cs0, fs0, m0, o0 = h(tok0.to(cuda), hw, ov)
        cs1, fs1, m1, o1 = h(tok1.to(cuda), hw, ov, overlap_tokens=o0, memory_tokens=m0)
    torch.cuda.synchronize()
    got = {"cs0": cs0, "fs0": fs0, "mem0": m0, "ov0": o0[:, :, ::st], "cs1": cs1, "fs1": fs1, "mem1": m1,
           "ov1": o1[:, :, ::st]}
    t = lambda k: torch.from_numpy(ref[k])  # noqa: E731
    e = {k: _rel(v, t("bf16_" + k)) for k, v in got.items()}
    spread = {k: _rel(t("fp32_" + k), t("bf16_" + k)) for k in got}
    _report("AlignmentHead 16 x 1375", e, spread)
    assert o0.shape == (1, ov + 1, 1375, 1024) and cs1.shape == (1, 1, 8) and fs1.shape == (1, 15, 7)
    for k in ("cs0", "cs1"):  # the north star on the chunk Sim(3)
        assert e[k] < 1e-3, (k, e)
    # about 2x the values measured on MI355X (round 5: fs 8.3e-4 / 6.6e-4, memory 2.8e-3 / 2.6e-3, the
    # post-head overlap tokens 4.0e-5 / 5.5e-5 -- the oracle's own bf16-vs-fp32 spread is 2.9e-3 there)
    bars = {"fs0": 1e-3, "fs1": 1e-3, "mem0": 6e-3, "mem1": 6e-3, "ov0": 1.5e-4, "ov1": 1.5e-4}
    for k, bar in bars.items():
        assert e[k] < bar, (k, e[k], bar)


def test_configs2_sequence_518_reduced_depth(cuda):
    """BASELINE configs[2]'s shape -- 16-frame 518^2 chunks,
    overlap 4, alignment head + Sim(3) decode, memory 8 -- at reduced
    aggregator depth (4 + DINOv2 1, kept layers 0-3), 28 frames = two chunks
    (one grouped encode of both, the DPT head per chunk), through
    apply_sequence_to_model, against the oracle chunk loop in the bf16-mixed
    tier; every error printed beside the oracle's own bf16-vs-fp32 spread
    (tests/golden/configs2_seq.npz, tests/golden/gen_configs2.py)."""
    import numpy as np
    from aligned_vggt.dist.pipeline import apply_sequence_to_model
    G = _configs2()
    ref = np.load(os.path.join(os.path.dirname(__file__), "golden", "configs2_seq.npz"))
    m = G.seq_model().to(cuda).eval()
    imgs = G.seq_images().to(cuda)
    P = G.SEQ
    got = apply_sequence_to_model({"images": imgs}, m, [P["w"]], [P["ov"]], "chunk_overlap", None)
    torch.cuda.synchronize()
    ds, ts = G.DEPTH_STRIDE, G.TOK_STRIDE
    pe = got["pose_enc"]
    g = {"chunk_sim3": got["chunk_sim3_alignment_enc"], "frame_se3": got["frame_se3_alignment_enc"],
         "pose_T": pe[..., :3], "pose_quat": pe[..., 3:7], "pose_fov": pe[..., 7:],
         "depth": got["depth"][:, :, ::ds, ::ds], "depth_conf": got["depth_conf"][:, :, ::ds, ::ds],
         "memory": torch.stack([x.to(cuda) for x in got["memory_tokens"]]),
         "overlap": got["overlap_tokens"][:, :, ::ts]}

    def r(tier):
        t = lambda k: torch.from_numpy(ref[f"{tier}_{k}"])  # noqa: E731
        pr = t("pose_enc")
        return {"chunk_sim3": t("chunk_sim3"), "frame_se3": t("frame_se3"), "pose_T": pr[..., :3],
                "pose_quat": pr[..., 3:7], "pose_fov": pr[..., 7:], "depth": t("depth"),
                "depth_conf": t("depth_conf"), "memory": t("memory"), "overlap": t("overlap")}

    rb, rf = r("bf16"), r("fp32")
    assert got["pose_enc"].shape == (1, P["N"], 9) and g["chunk_sim3"].shape == (1, 2, 8)
    e = {k: (_quat_rel if k == "pose_quat" else _rel)(g[k], rb[k]) for k in g}
    spread = {k: (_quat_rel if k == "pose_quat" else _rel)(rf[k], rb[k]) for k in g}
    _report("configs[2] 2 x 16 x 518^2", e, spread)
    assert e["chunk_sim3"] < 1e-3, e  # north star
    # 2x the values measured on MI355X (round 5: frame_se3 8.3e-4, depth 1.4e-4, conf 3.1e-6, memory
    # 2.8e-3, overlap 3.1e-3, pose T 8.9e-2 / quat 1.5e-2 / FoV 9.6e-3).  The poses go through the
    # random-init camera head, whose translations amplify the bf16 tier's token error (the camera
    # head itself matches the oracle to 1e-4 on identical tokens, test_gpu_model.py
    # test_heads_fp32_tier_tight; the oracle's own bf16-vs-fp32 pose spread here: T 7.8e-2, quat
    # 1.2e-2, FoV 1.1e-2), so the poses are ALSO held within 1.5x of that spread
    bars = {"frame_se3": 1e-3, "depth": 3e-4, "depth_conf": 1e-5, "memory": 6e-3, "overlap": 7e-3,
            "pose_T": 0.18, "pose_quat": 3e-2, "pose_fov": 2e-2}
    for k, bar in bars.items():
        assert e[k] < bar, (k, e[k], bar)
    for k in ("pose_T", "pose_quat", "pose_fov"):
        assert e[k] < 1.5 * spread[k], (k, e[k], spread[k])


def _synthetic_w2c(S, seed=7):
    """GT trajectory of SURVEY.md §8d: yaw random walk (sigma 0.5 deg / frame),
    1 unit forward per frame, seed 7; w2c (1, S, 3, 4) (OpenCV, README.md:127)."""
    g = torch.Generator().manual_seed(seed)
    yaw = torch.cumsum(torch.randn(S, generator=g) * 0.0087, 0)
    c2w = torch.eye(4).repeat(S, 1, 1)
    c2w[:, 0, 0], c2w[:, 0, 2], c2w[:, 2, 0], c2w[:, 2, 2] = yaw.cos(), yaw.sin(), -yaw.sin(), yaw.cos()
    c2w[:, :3, 3] = torch.cumsum(torch.stack([yaw.sin(), torch.zeros(S), yaw.cos()], -1), 0)
    return torch.linalg.inv(c2w)[:, :3, :][None]


def test_vkitti_sequence_ate_rpe_parity(cuda, monkeypatch):
    """the metric's "ATE/RPE parity vs ref" at the
    configs[3]/[4] chunk shape -- 38 frames of 154 x 518, chunk 16 / overlap 4
    -> chunks [0-15], [12-27] and a 14-frame tail [24-37]; memory 8, reduced
    aggregator depth (4 + DINOv2 1) -- through apply_sequence_to_model with the
    'scale_from_poses' GT alignment (training_metrics.py:239-262,
    alignment.py:206-242), against the oracle chunk loop in both tiers.  The
    camera head's translation is conditioned (4 x 0.25 along the optical axis)
    so its relative error is well-posed.  ATE RMSE (trajectory_metrics.py:28-77)
    and RPE trans / rot (:154-223) of the HIP trajectory against the synthetic
    GT must match the bf16 oracle's."""
    from aligned_vggt.backbone.aggregator import Aggregator
    from aligned_vggt.dist.pipeline import apply_sequence_to_model
    from aligned_vggt.eval import AbsoluteTrajectoryError, RelativePoseError, poses_c2w_from_predictions
    from aligned_vggt.models import featureAligned_vggt as FAmod
    from aligned_vggt.models.featureAligned_vggt import FeatureAlignedVGGT
    from aligned_vggt.utils import alignment as A
    from aligned_vggt.utils.synthetic import condition_pose_outputs_, synthetic_images, synthetic_init_
    N, w, ov, H, W = 38, 16, 4, 154, 518
    chunks = O.generate_chunks(N, w, ov)
    assert [len(c) for c in chunks] == [16, 16, 14]  # a shorter tail chunk (data.py:188-190)
    monkeypatch.setattr(FAmod, "Aggregator", lambda **kw: Aggregator(depth=4, dino_depth=1, **kw))
    m = FeatureAlignedVGGT(enable_point=False, enable_track=False, num_memory_tokens=8)
    m.intermediate_layer_indices = [0, 1, 2, 3]
    synthetic_init_(m, seed=17)
    condition_pose_outputs_(m, translation=0.25)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(cuda).eval()
    imgs = synthetic_images(1, N, H, W, seed=41)
    extr = _synthetic_w2c(N)
    got = apply_sequence_to_model({"images": imgs.to(cuda), "extrinsics": extr.to(cuda)}, m, [w], [ov],
                                  "chunk_overlap", "scale_from_poses")
    torch.cuda.synchronize()
    agg_kw = {"keep": (0, 1, 2, 3), "depth": 4, "dino_depth": 1}

    def oracle(bf16):
        ctx = None
        with torch.no_grad():
            for ids in chunks:
                ctx = O.feature_aligned_forward(sd, imgs[:, ids], ov, ctx, bf16=bf16, agg_kwargs=agg_kw)
        pe = torch.cat([p[:, (ov if i else 0):] for i, p in enumerate(ctx["pose_enc"])], 1)
        pred = {"pose_enc": pe}
        A.scale_alignment_from_poses(pred, {"extrinsics": extr})
        return ctx, pred["pose_enc"]

    (ctx_b, pe_b), (ctx_f, pe_f) = oracle(True), oracle(False)
    pe = got["pose_enc"].cpu()
    assert pe.shape == (1, N, 9)

    def parts(p, ctx):
        return {"chunk_sim3": ctx["chunk_sim3_alignment_enc"] if ctx is not None else None,
                "pose_T": p[..., :3], "pose_quat": p[..., 3:7], "pose_fov": p[..., 7:]}

    e = {"chunk_sim3": _rel(got["chunk_sim3_alignment_enc"], ctx_b["chunk_sim3_alignment_enc"]),
         "frame_se3": _rel(got["frame_se3_alignment_enc"], ctx_b["frame_se3_alignment_enc"]),
         "pose_T": _rel(pe[..., :3], pe_b[..., :3]), "pose_quat": _quat_rel(pe[..., 3:7], pe_b[..., 3:7]),
         "pose_fov": _rel(pe[..., 7:], pe_b[..., 7:])}
    spread = {"chunk_sim3": _rel(ctx_f["chunk_sim3_alignment_enc"], ctx_b["chunk_sim3_alignment_enc"]),
              "frame_se3": _rel(ctx_f["frame_se3_alignment_enc"], ctx_b["frame_se3_alignment_enc"]),
              "pose_T": _rel(pe_f[..., :3], pe_b[..., :3]), "pose_quat": _quat_rel(pe_f[..., 3:7], pe_b[..., 3:7]),
              "pose_fov": _rel(pe_f[..., 7:], pe_b[..., 7:])}
    _report("154x518 ATE/RPE sequence", e, spread)

    def metrics(pose_enc):
        p, g = poses_c2w_from_predictions(pose_enc.cpu(), extr, (H, W))
        ate, rpe = AbsoluteTrajectoryError(), RelativePoseError()
        ate.update(p[0], g[0])
        rpe.update(p[0], g[0])
        return {k: float(v) for k, v in {**ate.compute(), **rpe.compute()}.items()}

    m_hip, m_b, m_f = metrics(pe), metrics(pe_b), metrics(pe_f)
    print("ATE/RPE hip", m_hip, "\nATE/RPE oracle bf16", m_b, "\nATE/RPE oracle fp32", m_f)
    assert e["chunk_sim3"] < 1e-3 and e["frame_se3"] < 1e-3, e  # the north star's 1e-3
    # Poses and the metrics built on them: about 2x the values measured on MI355X
    # (round 6: pose T 6.6e-2 / quat 1.0e-2 / FoV 1.1e-2 against the oracle's own
    # bf16-vs-fp32 spread of 2.6e-2 / 1.3e-2 / 1.0e-2; ATE 0.57 %, RPE trans 5.7 %,
    # RPE rot 0.08 % from the bf16 oracle's).  The translations are the ill-conditioned
    # quantity: the camera head reads one small-norm camera token per frame whose bf16
    # error is ~2x the layer's, and amplifies it 2-4x even with |T| ~ 1
    # (tests/test_pose_conditioning.py measures that floor on the oracle alone);
    # RPE-trans, the frame-to-frame translation, inherits the most of it.
    for k, bar in {"pose_T": 0.13, "pose_quat": 2.1e-2, "pose_fov": 2.2e-2}.items():
        assert e[k] < bar, (k, e[k], bar)
    for k in ("pose_quat", "pose_fov"):
        assert e[k] < 1.5 * spread[k], (k, e[k], spread[k])
    bars = {"ate_rmse": 1.2e-2, "rpe_trans_rmse": 0.115, "rpe_rot_rmse": 2e-3}
    for k in m_b:
        d_hip, d_sp = abs(m_hip[k] - m_b[k]), abs(m_f[k] - m_b[k])
        rel = d_hip / max(abs(m_b[k]), 1e-12)
        print(f"{k}: hip {m_hip[k]:.6g} oracle bf16 {m_b[k]:.6g} fp32 {m_f[k]:.6g} | hip-vs-bf16 rel {rel:.2e}, "
              f"|hip-bf16| / |fp32-bf16| = {d_hip / max(d_sp, 1e-30):.2f}")
        assert rel < bars[k], (k, rel, bars[k], m_hip, m_b)
