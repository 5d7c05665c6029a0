"""Pin the CPU oracle against fixtures produced by the reference's own code
(tests/golden/gen_golden.py).  CPU only."""
import numpy as np
import torch

from oracle import vggt_oracle as O


def t(a):
    return torch.from_numpy(np.asarray(a))


def test_rope1d_matches_reference(golden):
    g = golden("rope1d")
    for i in range(3):
        y = O.rope1d(t(g[f"x{i}"]), t(g[f"pos{i}"]))
        np.testing.assert_allclose(y.numpy(), g[f"y{i}"], rtol=0, atol=1e-6)


def test_gated_update_matches_reference(golden):
    assert int(golden("gated_update_nparams")["d512_n8"]) == 8922113
    for tag in ("d64", "d32"):
        g = golden("gated_update_" + tag)
        sd = {k[2:]: t(v) for k, v in g.items() if k.startswith("p.")}
        out = O.gated_update(sd, "", t(g["memory"]), t(g["update"]))
        np.testing.assert_allclose(out.numpy(), g["out"], rtol=0, atol=2e-6)


def test_generate_chunks_matches_reference(golden):
    rows = golden("generate_chunks")["rows"]
    cases = {}
    for n, w, ov, ci, f in rows:
        cases.setdefault((n, w, ov), {}).setdefault(ci, []).append(f)
    assert len(cases) > 100
    for (n, w, ov), chunks in cases.items():
        ref = [chunks[i] for i in range(len(chunks))]
        assert O.generate_chunks(int(n), int(w), int(ov)) == ref, (n, w, ov)
    # the BASELINE counts quoted in SURVEY.md §8(a) a14
    assert len(O.generate_chunks(64, 16, 4)) == 5
    c = O.generate_chunks(512, 16, 4)
    assert len(c) == 43 and len(c[-1]) == 8


def test_average_pose_encodings_matches_reference(golden):
    g = golden("average_pose_encodings")
    out = O.average_pose_encodings(t(g["enc"])).numpy()
    ref = g["out"]
    np.testing.assert_allclose(out[..., :3], ref[..., :3], atol=1e-6)
    # eigenvector sign is arbitrary: compare up to sign
    dots = np.abs((out[..., 3:] * ref[..., 3:]).sum(-1))
    np.testing.assert_allclose(dots, 1.0, atol=1e-5)


def test_small_fns_match_reference(golden):
    g = golden("small_fns")
    np.testing.assert_array_equal(O.merge_results(t(g["a"]), t(g["b"]), 0).numpy(), g["merged0"])
    np.testing.assert_array_equal(O.merge_results(t(g["a"]), t(g["b"]), 2).numpy(), g["merged2"])
    np.testing.assert_array_equal(O.slice_expand_and_flatten(t(g["tok"]), 2, 4).numpy(), g["sef"])


def test_dinov2_stage_matches_transformers(golden):
    g = golden("dinov2_hf")
    sd = {k[3:]: t(v) for k, v in g.items() if k.startswith("sd.")}
    for tag in ("sq", "rect"):
        out = O.dinov2(sd, "", t(g["img_" + tag]), bf16=False, depth=2, num_heads=4)
        np.testing.assert_allclose(out.numpy(), g["patch_" + tag], rtol=1e-4, atol=1e-4)


def _dpt_tokens(g, nspecial=5):
    """The fixture's patch tokens as a (1, F, nspecial + h*w, C) aggregator layer
    (special-token rows arbitrary: the DPT head reads from patch_start_idx)."""
    tok = t(g["tokens"])
    F_, hw, C = tok.shape
    spec = torch.full((F_, nspecial, C), 7.0)
    return torch.cat([spec, tok], 1).reshape(1, F_, nspecial + hw, C)


def test_dpt_stages_match_transformers_depth_anything(golden):
    """The oracle's DPT decoder vs the in-container transformers Depth-Anything
    neck + head with the same weights (tests/golden/gen_golden.py gen_dpt_hf):
    reassemble (incl. ConvTranspose 4x / 2x and the stride-2 conv), layer*_rn,
    every fusion block (in-place-ReLU residual units, align_corners=True
    resize, rectangular 3x4 -> 5x7 sizes) and the pre-activation head output."""
    g = golden("dpt_hf")
    sd = {k[3:]: t(v) for k, v in g.items() if k.startswith("sd.")}
    ph, pw = int(g["ph"]), int(g["pw"])
    toks = _dpt_tokens(g)
    imgs = torch.zeros(1, toks.shape[1], 3, ph * 14, pw * 14)
    st = {}
    with torch.no_grad():
        O.dpt_head(sd, "", [toks] * 4, imgs, 5, "exp", pos_embed=False, stages=st)
    for k in [f"reassemble{i}" for i in range(4)] + [f"rn{i}" for i in range(4)] + [f"fused{j}" for j in range(4)]:
        # measured 2e-7 .. 6e-7 rel-L2 per stage (max abs 6.6e-7): fp32 summation order only
        np.testing.assert_allclose(st[k].numpy(), g[k], rtol=1e-5, atol=2e-6, err_msg=k)
    np.testing.assert_allclose(st["head_pre"][:, :1].numpy(), g["head_pre"], rtol=1e-5, atol=2e-6)
    np.testing.assert_allclose(torch.sigmoid(st["head_pre"][:, 0]).numpy(), g["out_sigmoid"], rtol=1e-5, atol=1e-6)


def test_pose_roundtrip_known_answer():
    g = torch.Generator().manual_seed(0)
    q = torch.nn.functional.normalize(torch.randn(2, 5, 4, generator=g), dim=-1)
    R = O.quat_to_mat(q)
    np.testing.assert_allclose((R @ R.transpose(-1, -2)).numpy(), np.eye(3)[None, None].repeat(2, 0).repeat(5, 1),
                               atol=1e-5)
    q2 = O.mat_to_quat(R)
    dots = (q * q2).sum(-1).abs()
    np.testing.assert_allclose(dots.numpy(), 1.0, atol=1e-5)
    T = torch.eye(4).repeat(10, 1, 1)
    T[:, :3, :3] = R.reshape(10, 3, 3)
    T[:, :3, 3] = torch.randn(10, 3, generator=g)
    np.testing.assert_allclose((O.closed_form_inverse_se3(T) @ T).numpy(), np.eye(4)[None].repeat(10, 0), atol=1e-5)
    enc = torch.cat([torch.randn(2, 5, 3, generator=g), q], dim=-1)
    np.testing.assert_allclose(O.extri_to_pose_encoding(O.pose_encoding_to_extri(enc))[..., :3].numpy(),
                               enc[..., :3].numpy(), atol=1e-6)


def test_irls_sim3_oracle_matches_reference(golden):
    from oracle import alignment_oracle as AO
    g = golden("irls_sim3")
    r, t, s = AO.irls_sim3_umeyama(*(torch.from_numpy(g[k]) for k in ("src", "dst", "conf_src", "conf_dst")))
    np.testing.assert_allclose(r.numpy(), g["r"], atol=1e-5)
    np.testing.assert_allclose(t.numpy(), g["t"], atol=1e-5)
    np.testing.assert_allclose(float(s), g["s"], rtol=1e-5)
    gb = golden("irls_sim3_batch")
    for b in range(3):
        r, t, s = AO.irls_sim3_umeyama(*(torch.from_numpy(gb[f"{k}{b}"]) for k in ("src", "dst", "cs", "cd")))
        np.testing.assert_allclose(r.numpy(), gb[f"r{b}"], atol=1e-5)
        np.testing.assert_allclose(t.numpy(), gb[f"t{b}"], atol=1e-4)
        np.testing.assert_allclose(float(s), gb[f"s{b}"], rtol=1e-5)


def test_sim3_point_map_oracle_matches_reference(golden):
    from oracle import alignment_oracle as AO
    g = golden("alignment_utils")
    out = AO.apply_sim3_alignment_on_point_maps(torch.from_numpy(g["pm"]), torch.from_numpy(g["T"]),
                                                torch.from_numpy(g["sc"]))
    np.testing.assert_allclose(out.numpy(), g["pm_out"], rtol=1e-6, atol=1e-6)
