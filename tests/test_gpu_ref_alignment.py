"""The HIP alignment path against fixtures of the reference's OWN modules
(tests/golden/ref_*.npz: alignment_head.py:224-540, cross_attention.py:47-131
and the featureAligned_vggt.py:84-225 composition, run on the test-only vggt
shim; see tests/test_ref_alignment_golden.py for the oracle's pin).

Tolerances (north star: Sim(3) within 1e-3 rel):
  * bf16 tier (trunk) vs the reference under emulated bf16-mixed autocast:
    chunk Sim(3) < 1e-3; frame SE(3) / memory / overlap tokens < 3e-3
    (measured on MI355X: 3e-4 - 9e-4; the reference's own bf16-vs-fp32 spread
    on these cases is ~7e-4 - 9e-4); composed poses / depths / points < 5e-3
    (measured <= 1.7e-3 after four chained chunks), quaternions 1e-5, FoV 1e-6;
  * fp32 tier (decoder, cross-attention block in fp32) vs the fp32 reference:
    1e-5 rel.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle.fixture_weights import (ALIGN_CASES, FA_RUNS, FIX_HW, FIX_SEED, fa_feed, fa_gt_poses,  # noqa: E402
                                    fa_images, fix_tokens_per_frame, fixture_tensor, load_fixture_weights_)
from oracle import vggt_oracle as O  # noqa: E402


def t(a):
    return torch.from_numpy(np.asarray(a))


def _rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.fixture(scope="module")
def heads():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from aligned_vggt.heads.alignment_head import AlignmentHead
    out = {}
    for tag, nm in (("m8", 8), ("m0", 0)):
        torch.manual_seed(0)
        h = AlignmentHead(in_dim=2048, patch_size=14, num_memory_tokens=nm, temporal_attention=True)
        out[tag] = load_fixture_weights_(h, FIX_SEED, prefix="alignment_head.").cuda().eval()
    return out


def test_alignment_head_vs_reference(heads, golden):
    g = golden("ref_alignment_head")
    P = fix_tokens_per_frame()
    for case, head, B, S, nov, prev in ALIGN_CASES:
        tok = fixture_tensor(f"ah.{case}.tokens", (B, S, P, 2048), FIX_SEED).cuda()
        ov = t(g[f"{prev}_bf16_new_ov"]).cuda() if prev else None
        mem = t(g[f"{prev}_bf16_memory"]).cuda() if prev and head == "m8" else None
        cs, fs, m, nov_t = heads[head](tok, FIX_HW, nov, overlap_tokens=ov, memory_tokens=mem)
        torch.cuda.synchronize()
        e = {"chunk_sim3": _rel(cs, g[f"{case}_bf16_chunk_sim3"]), "frame_se3": _rel(fs, g[f"{case}_bf16_frame_se3"]),
             "new_ov": _rel(nov_t, g[f"{case}_bf16_new_ov"])}
        e32 = {"chunk_sim3": _rel(cs, g[f"{case}_f32_chunk_sim3"]), "frame_se3": _rel(fs, g[f"{case}_f32_frame_se3"])}
        if head == "m8":
            e["memory"] = _rel(m, g[f"{case}_bf16_memory"])
        else:
            assert m is None
        print(case, "vs bf16 ref", e, "vs fp32 ref", e32)
        assert tuple(nov_t.shape) == g[f"{case}_bf16_new_ov"].shape
        assert e["chunk_sim3"] < 1e-3 and e["frame_se3"] < 1e-3, (case, e)  # the north star's 1e-3
        assert max(e.values()) < 3e-3, (case, e)


def test_decode_alignments_vs_reference(heads, golden):
    """_decode_alignments (fp32 tier: the reference disables autocast there)."""
    g = golden("ref_alignment_head")
    h = heads["m8"]
    mem = None
    for i, first in ((1, True), (2, False)):
        ft = fixture_tensor(f"dec.tokens{i}", (2, 4, 1024), FIX_SEED).cuda()
        cs, fs, m = h._decode_alignments(ft, 2, first, memory_tokens=mem)
        torch.cuda.synchronize()
        for name, v in (("chunk_sim3", cs), ("frame_se3", fs), ("memory", m)):
            assert _rel(v, g[f"dec{i}_{name}"]) < 1e-5, (i, name, _rel(v, g[f"dec{i}_{name}"]))
        mem = t(g[f"dec{i}_memory"]).cuda()


def test_cross_attention_block_vs_reference(golden):
    """The two roles of CrossAttentionBlock: decoder block on the fp32 tier
    (forward_f32) and temporal block on the bf16 tier (forward_rows_bf16, the
    raw-view row grouping: 36 groups of 3 queries vs 2 keys)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from aligned_vggt import _native as N
    from aligned_vggt.layers.cross_attention import CrossAttentionBlock
    from aligned_vggt.layers.rope import RotaryPositionEmbedding
    from aligned_vggt.runtime import Workspace, round_up
    g = golden("ref_cross_attention")
    dev = torch.device("cuda")
    rope = RotaryPositionEmbedding(frequency=100)
    # decoder role, fp32
    blk = CrossAttentionBlock(dim=512, num_heads=8, init_values=0.01, qk_norm=True, rope=rope)
    blk = load_fixture_weights_(blk, FIX_SEED, prefix="cab_dec.").to(dev).eval()
    x = fixture_tensor("cab_dec.x", (2, 1, 512), FIX_SEED).to(dev)
    y = fixture_tensor("cab_dec.y", (2, 11, 512), FIX_SEED).to(dev)
    pq, pk = t(g["dec_pos_q"]), t(g["dec_pos_k"])
    tabs = rope.tables(64, int(max(pq.max(), pk.max())), dev)
    out = blk.forward_f32(x, y, pq.to(torch.int32).to(dev), pk.to(torch.int32).to(dev), tabs)
    torch.cuda.synchronize()
    assert _rel(out, g["dec_f32"]) < 1e-5, _rel(out, g["dec_f32"])
    # temporal role, bf16 tier, rows streamed in place
    blk = CrossAttentionBlock(dim=1024, num_heads=8, init_values=0.01, qk_norm=True, rope=rope)
    blk = load_fixture_weights_(blk, FIX_SEED, prefix="cab_tmp.").to(dev).eval()
    G, S, T = 36, 3, 2
    xr = torch.zeros(round_up(G * S, 256), 1024, device=dev)
    xr[:G * S] = fixture_tensor("cab_tmp.x", (G, S, 1024), FIX_SEED).reshape(G * S, 1024).to(dev)
    yr = torch.zeros(round_up(G * T, 256), 1024, device=dev)
    yr[:G * T] = fixture_tensor("cab_tmp.y", (G, T, 1024), FIX_SEED).reshape(G * T, 1024).to(dev)
    pq, pk = t(g["tmp_pos_q"]), t(g["tmp_pos_k"])
    c, s = rope.tables(128, int(max(pq.max(), pk.max())), dev)
    rq = (pq.to(torch.int32).to(dev), c, s)
    rk = (pk.to(torch.int32).to(dev), c, s)
    blk.forward_rows_bf16(xr, G * S, yr, G * T, G, S, T, rq, rk, Workspace.get(dev))
    torch.cuda.synchronize()
    got = xr[:G * S].view(G, S, 1024)
    e, e32 = _rel(got, g["tmp_bf16"]), _rel(got, g["tmp_f32"])
    print("temporal block vs bf16 ref", e, "vs fp32 ref", e32)
    assert e < 2e-4, (e, e32)  # measured 2.6e-5


@pytest.fixture(scope="module")
def model():
    """FeatureAlignedVGGT with the fixture alignment head; the encoders are
    never run (align_chunk is fed the stub encoder outputs), so they are left
    unmaterialised-then-empty to keep the test fast."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from aligned_vggt.models.featureAligned_vggt import FeatureAlignedVGGT
    with torch.device("meta"):
        m = FeatureAlignedVGGT(enable_track=False, enable_point=True, num_memory_tokens=8)
    m = m.to_empty(device="cuda")
    load_fixture_weights_(m.alignment_head, FIX_SEED, prefix="alignment_head.")
    return m.eval()


def _quat_err(a, b):
    qa, qb = a[..., 3:7].double(), b[..., 3:7].double()
    return float((1.0 - (qa * qb).sum(-1).abs()).abs().max())


@pytest.mark.parametrize("run", [r[0] for r in FA_RUNS])
def test_feature_aligned_composition_vs_reference(model, golden, run):
    """align_chunk (alignment head + Sim(3)/SE(3) composition + Markley mean +
    context lists) over whole chunk sequences, fed the same stub encoder
    outputs as the reference run."""
    g = golden("ref_feature_aligned")
    (_, N, w, ov, use_gt), = [r for r in FA_RUNS if r[0] == run]
    chunks = O.generate_chunks(N, w, ov)
    imgs = fa_images(run, N).cuda()
    ctx = None
    for i, ids in enumerate(chunks):
        f = fa_feed(run, i, len(ids))
        enc = {"images": imgs[:, ids], "tokens": [x.cuda() for x in f["tokens"]], "patch_start_idx": 5,
               "cam_pose_enc": f["pose_enc"].cuda(), "depth": f["depth"].cuda(), "depth_conf": f["depth_conf"].cuda(),
               "points": f["points"].cuda(), "points_conf": f["points_conf"].cuda()}
        gt = fa_gt_poses(run, i, len(ids)).cuda() if use_gt else None
        ctx = model.align_chunk(enc, ov, ctx, gt_poses=gt)
    torch.cuda.synchronize()
    p = f"{run}_bf16_"
    assert len(ctx["pose_enc"]) == int(g[p + "nchunks"])
    e = {"chunk_sim3": _rel(ctx["chunk_sim3_alignment_enc"], g[p + "chunk_sim3"]),
         "frame_se3": _rel(ctx["frame_se3_alignment_enc"], g[p + "frame_se3"]),
         "overlap": _rel(ctx["overlap_tokens"], g[p + "overlap_tokens"])}
    for i in range(len(chunks)):
        pe, ref = ctx["pose_enc"][i].cpu(), t(g[p + f"pose_enc{i}"])
        e[f"T{i}"] = _rel(pe[..., :3], ref[..., :3])
        e[f"q{i}"] = _quat_err(pe, ref)
        e[f"fov{i}"] = _rel(pe[..., 7:], ref[..., 7:])
        e[f"mem{i}"] = _rel(ctx["memory_tokens"][i], g[p + f"memory{i}"])
        e[f"depth{i}"] = _rel(ctx["depth"][i][:, :, ::7, ::7], g[p + f"depth{i}"])
        e[f"pts{i}"] = _rel(ctx["world_points"][i][:, :, ::7, ::7], g[p + f"points{i}"])
        assert torch.equal(ctx["depth_conf"][i][:, :, ::7, ::7].cpu(), t(g[p + f"depth_conf{i}"]))
    print(run, {k: f"{v:.2e}" for k, v in e.items()})
    assert e["chunk_sim3"] < 1e-3, e
    for k, v in e.items():
        if k.startswith("fov"):
            assert v < 1e-6, (k, e)
        elif k.startswith("q"):
            assert v < 1e-5, (k, e)
        elif k.startswith(("T", "pts")):
            # composed translations / points: 2x the measured (<= 1.7e-3 after four chained chunks;
            # the budget is test_pose_error_budget: head error x chain, composition 1e-7)
            assert v < 3.5e-3, (k, e)
        elif k.startswith("depth"):
            assert v < 1e-3, (k, e)  # = the chunk scale's error (measured <= 5e-4)
        else:
            assert v < 3e-3, (k, e)


def _pose_errs(pe, ref):
    """(translation rel-L2, quaternion 1-|<q,r>| max, FoV rel-L2) of pose encodings (B,S,9)."""
    pe, ref = torch.as_tensor(pe).double(), torch.as_tensor(ref).double()
    return _rel(pe[..., :3], ref[..., :3]), _quat_err(pe, ref), _rel(pe[..., 7:], ref[..., 7:])


@pytest.mark.parametrize("run", [r[0] for r in FA_RUNS])
def test_pose_error_budget(model, golden, run):
    """where the composed-pose error at identical encoder
    outputs comes from.  The reference's composition (featureAligned_vggt.py:
    96-143, data.py:33-52, geometry.py:4-37 -- the oracle's compose_poses, which
    reproduces the reference's own fp32 AND bf16 fixtures at <= 1e-5 given the
    reference head's outputs) is fed the HIP head's outputs and, one input at a
    time, the reference's:

      * composition: oracle(HIP head outputs, HIP context) vs the HIP pose --
        the composition itself, fp32 on both sides: <= 1e-5;
      * attribution: oracle(one input from the HIP run, the rest from the
        reference) vs the reference pose -- chunk Sim(3), frame SE(3), the
        previous chunk's poses (context, through the Markley mean);
      * depth: depth x chunk scale, so its error is the scale's exactly.

    The bars on T / depth below are 2x the measured values; the printed gains
    (pose error / input error) show how the bf16-tier head error (<= 1e-3)
    becomes a larger relative error of the composed translations."""
    g = golden("ref_feature_aligned")
    (_, N, w, ov, use_gt), = [r for r in FA_RUNS if r[0] == run]
    chunks = O.generate_chunks(N, w, ov)
    imgs = fa_images(run, N).cuda()
    H, W = imgs.shape[-2:]
    ctx = None
    feeds = []
    for i, ids in enumerate(chunks):
        f = fa_feed(run, i, len(ids))
        feeds.append(f)
        enc = {"images": imgs[:, ids], "tokens": [x.cuda() for x in f["tokens"]], "patch_start_idx": 5,
               "cam_pose_enc": f["pose_enc"].cuda(), "depth": f["depth"].cuda(), "depth_conf": f["depth_conf"].cuda(),
               "points": f["points"].cuda(), "points_conf": f["points_conf"].cuda()}
        gt = fa_gt_poses(run, i, len(ids)).cuda() if use_gt else None
        ctx = model.align_chunk(enc, ov, ctx, gt_poses=gt)
    torch.cuda.synchronize()
    p = f"{run}_bf16_"
    sizes = [len(c) - 1 for c in chunks]
    # fp32 throughout, as the reference composes (featureAligned_vggt.py:104: autocast off)
    cs_h = ctx["chunk_sim3_alignment_enc"].cpu().float()
    fs_h = list(torch.split(ctx["frame_se3_alignment_enc"].cpu().float(), sizes, dim=1))
    cs_r = t(g[p + "chunk_sim3"]).float()
    fs_r = list(torch.split(t(g[p + "frame_se3"]).float(), sizes, dim=1))
    pe_h = [x.cpu().float() for x in ctx["pose_enc"]]
    pe_r = [t(g[p + f"pose_enc{i}"]).float() for i in range(len(chunks))]

    def compose(i, cs, fs, prev):
        S = len(chunks[i])
        o = ov if S > ov else S - 1
        gt0 = fa_gt_poses(run, i, S)[:, 0].float() if (use_gt and i > 0) else None
        return O.compose_poses(cs[:, i:i + 1], fs, feeds[i]["pose_enc"].float(), prev if i > 0 else None, gt0, o,
                               (H, W))[0]

    rows = []
    worst = {"comp": 0.0, "comp_ref": 0.0}
    for i in range(len(chunks)):
        prev_h = pe_h[i - 1] if i else None
        prev_r = pe_r[i - 1] if i else None
        comp = _pose_errs(compose(i, cs_h, fs_h[i], prev_h), pe_h[i])
        comp_ref = _pose_errs(compose(i, cs_r, fs_r[i], prev_r), pe_r[i])
        worst["comp"] = max(worst["comp"], comp[0], comp[1], comp[2])
        worst["comp_ref"] = max(worst["comp_ref"], comp_ref[0], comp_ref[1], comp_ref[2])
        e_cs = _rel(cs_h[:, i], cs_r[:, i])
        e_fs = _rel(fs_h[i], fs_r[i]) if sizes[i] else 0.0
        e_scale = float(((cs_h[:, i, 7] - cs_r[:, i, 7]).abs() / cs_r[:, i, 7].abs()).max())
        row = {"chunk": i, "in_chunk_sim3": e_cs, "in_frame_se3": e_fs, "in_scale": e_scale,
               "T_total": _pose_errs(pe_h[i], pe_r[i])[0],
               "T_from_chunk_sim3": _pose_errs(compose(i, cs_h, fs_r[i], prev_r), pe_r[i])[0],
               "T_from_frame_se3": _pose_errs(compose(i, cs_r, fs_h[i], prev_r), pe_r[i])[0],
               "T_from_context": _pose_errs(compose(i, cs_r, fs_r[i], prev_h), pe_r[i])[0] if i else 0.0,
               "depth": _rel(ctx["depth"][i][:, :, ::7, ::7], g[p + f"depth{i}"])}
        rows.append(row)
        print(run, {k: (f"{v:.2e}" if isinstance(v, float) else v) for k, v in row.items()})
    print(run, "composition error (HIP vs oracle on HIP inputs)", f"{worst['comp']:.2e}",
          "| oracle vs reference on reference inputs", f"{worst['comp_ref']:.2e}")
    assert worst["comp"] < 1e-5, worst
    assert worst["comp_ref"] < 1e-5, worst
    for r in rows:
        # depth = depth_raw x scale: its error IS the scale's (fp32 round-off aside)
        assert abs(r["depth"] - r["in_scale"]) < 1e-5 + 1e-3 * r["in_scale"], r
        # every input's share is bounded by the total it composes to (no hidden term)
        assert max(r["T_from_chunk_sim3"], r["T_from_frame_se3"], r["T_from_context"]) < 2.5 * r["T_total"] + 1e-5, r
    # measured on MI355X (round 5): a first chunk (no context) composes to T 4.2e-4 .. 5.0e-4 -- within the
    # north star's 1e-3 -- and the error grows along the chain only through the context (the previous
    # chunk's poses via the Markley mean): 1.3e-3 .. 1.6e-3 after four chunks; bars 2x measured
    assert rows[0]["T_total"] < 1e-3, rows[0]
    assert all(r["T_total"] < 3.5e-3 for r in rows), rows
    if use_gt:
        assert all(r["T_from_context"] == 0.0 for r in rows)  # chunk_gt: the GT pose replaces the context
