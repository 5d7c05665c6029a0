"""Pin the oracle's alignment path against the reference's OWN modules
(alignment_head.py:224-540, cross_attention.py:47-131, the
featureAligned_vggt.py:84-225 composition), run by tests/golden/gen_golden.py on
the test-only vggt shim in fp32 and under an emulated bf16-mixed autocast.
Weights / inputs are regenerated from oracle.fixture_weights.  CPU only."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import vggt_oracle as O
from oracle.fixture_weights import (ALIGN_CASES, FA_RUNS, FIX_HW, FIX_SEED, fa_feed, fa_gt_poses, fa_images,
                                    fixture_state_dict, fixture_tensor, fix_tokens_per_frame)

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _keys():
    with open(os.path.join(GOLDEN, "ref_alignment_keys.json")) as f:
        return json.load(f)


def head_state_dict(head: str = "m8"):
    """Oracle state dict (alignment_head.* names) with the fixture values."""
    return fixture_state_dict([("alignment_head." + k, tuple(s)) for k, s in _keys()[head]], FIX_SEED)


def t(a):
    return torch.from_numpy(np.asarray(a))


def _rel(a, b):
    a, b = torch.as_tensor(a).double(), torch.as_tensor(b).double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


# fp32 fixtures: the same arithmetic up to summation order; bf16-mixed: the
# emulated autocast rounds at the same points as the oracle's bf16 tier, so
# only rare one-ulp bf16 flips (fp32 summation order decides a rounding) remain
# (measured: 1e-7 level on both tiers)
TOL = {"f32": 2e-6, "bf16": 1e-5}


@pytest.mark.parametrize("prec", ["f32", "bf16"])
def test_cross_attention_block_matches_reference(golden, prec):
    g = golden("ref_cross_attention")
    for tag, xs, ys in (("dec", (2, 1, 512), (2, 11, 512)), ("tmp", (36, 3, 1024), (36, 2, 1024))):
        dim = xs[-1]
        names = [("norm1.weight", (dim,)), ("norm1.bias", (dim,)), ("norm2.weight", (dim,)), ("norm2.bias", (dim,)),
                 ("norm3.weight", (dim,)), ("norm3.bias", (dim,)), ("ls1.gamma", (dim,)), ("ls2.gamma", (dim,)),
                 ("mlp.fc1.weight", (4 * dim, dim)), ("mlp.fc1.bias", (4 * dim,)),
                 ("mlp.fc2.weight", (dim, 4 * dim)), ("mlp.fc2.bias", (dim,)),
                 ("attn.q_norm.weight", (dim // 8,)), ("attn.q_norm.bias", (dim // 8,)),
                 ("attn.k_norm.weight", (dim // 8,)), ("attn.k_norm.bias", (dim // 8,))]
        for n in ("q", "k", "v", "proj"):
            names += [(f"attn.{n}.weight", (dim, dim)), (f"attn.{n}.bias", (dim,))]
        sd = {k[len(f"cab_{tag}."):]: v for k, v in fixture_state_dict([(f"cab_{tag}." + n, s) for n, s in names],
                                                                        FIX_SEED).items()}
        x = fixture_tensor(f"cab_{tag}.x", xs, FIX_SEED)
        y = fixture_tensor(f"cab_{tag}.y", ys, FIX_SEED)
        pq, pk = t(g[f"{tag}_pos_q"]), t(g[f"{tag}_pos_k"])
        pos = (pq.view(1, -1).expand(xs[0], -1), pk.view(1, -1).expand(xs[0], -1))
        out = O.cross_attention_block(sd, "", x, y, 8, pos, prec == "bf16")
        assert _rel(out, g[f"{tag}_{prec}"]) < TOL[prec], (tag, prec, _rel(out, g[f"{tag}_{prec}"]))


@pytest.mark.parametrize("prec", ["f32", "bf16"])
def test_alignment_head_matches_reference(golden, prec):
    g = golden("ref_alignment_head")
    sds = {"m8": head_state_dict("m8"), "m0": head_state_dict("m0")}
    P = fix_tokens_per_frame()
    for case, head, B, S, nov, prev in ALIGN_CASES:
        tok = fixture_tensor(f"ah.{case}.tokens", (B, S, P, 2048), FIX_SEED)
        ov = t(g[f"{prev}_{prec}_new_ov"]) if prev else None
        mem = t(g[f"{prev}_{prec}_memory"]) if prev and head == "m8" else None
        cs, fs, m, nov_t = O.alignment_head(sds[head], tok, FIX_HW, nov, ov, mem,
                                            num_memory_tokens=8 if head == "m8" else 0, bf16=prec == "bf16")
        errs = {"chunk_sim3": _rel(cs, g[f"{case}_{prec}_chunk_sim3"]),
                "frame_se3": _rel(fs, g[f"{case}_{prec}_frame_se3"]),
                "new_ov": _rel(nov_t, g[f"{case}_{prec}_new_ov"])}
        if head == "m8":
            errs["memory"] = _rel(m, g[f"{case}_{prec}_memory"])
        else:
            assert m is None and f"{case}_{prec}_memory" not in g
        assert nov_t.shape == g[f"{case}_{prec}_new_ov"].shape
        assert max(errs.values()) < TOL[prec], (case, prec, errs)


def test_decode_alignments_matches_reference(golden):
    g = golden("ref_alignment_head")
    sd = head_state_dict("m8")
    mem = None
    for i in (1, 2):
        ft = fixture_tensor(f"dec.tokens{i}", (2, 4, 1024), FIX_SEED)
        cs, fs, mem = O.decode_alignments(sd, "alignment_head.", ft, 8, mem)
        for name, v in (("chunk_sim3", cs), ("frame_se3", fs), ("memory", mem)):
            assert _rel(v, g[f"dec{i}_{name}"]) < 2e-6, (i, name)
        mem = t(g[f"dec{i}_memory"])


def _quat_rot_err(a, b):
    """Pose encodings [T, quat xyzw, FoV]: quaternions compared up to sign
    (the Markley eigenvector sign is arbitrary)."""
    qa, qb = a[..., 3:7], b[..., 3:7]
    return float((1.0 - (qa * qb).sum(-1).abs()).abs().max())


def run_oracle_composition(run, N, w, ov, use_gt, prec, sd):
    ctx = None
    chunks = O.generate_chunks(N, w, ov)
    imgs = fa_images(run, N)
    for i, ids in enumerate(chunks):
        f = fa_feed(run, i, len(ids))
        enc = {"tokens": f["tokens"], "patch_start_idx": 5, "cam_pose_enc": f["pose_enc"], "depth": f["depth"],
               "depth_conf": f["depth_conf"], "points": f["points"], "points_conf": f["points_conf"]}
        gt = fa_gt_poses(run, i, len(ids)) if use_gt else None
        ctx = O.feature_aligned_compose(sd, enc, imgs[:, ids], ov, ctx, gt, num_memory_tokens=8, bf16=prec == "bf16")
    return ctx, len(chunks)


@pytest.mark.parametrize("prec", ["f32", "bf16"])
@pytest.mark.parametrize("run", [r[0] for r in FA_RUNS])
def test_feature_aligned_composition_matches_reference(golden, prec, run):
    g = golden("ref_feature_aligned")
    (_, N, w, ov, use_gt), = [r for r in FA_RUNS if r[0] == run]
    ctx, n = run_oracle_composition(run, N, w, ov, use_gt, prec, head_state_dict("m8"))
    p = f"{run}_{prec}_"
    assert int(g[p + "nchunks"]) == n
    tol = TOL[prec]
    assert _rel(ctx["chunk_sim3_alignment_enc"], g[p + "chunk_sim3"]) < tol
    assert _rel(ctx["frame_se3_alignment_enc"], g[p + "frame_se3"]) < tol
    assert _rel(ctx["overlap_tokens"], g[p + "overlap_tokens"]) < tol
    for i in range(n):
        pe, ref = ctx["pose_enc"][i], t(g[p + f"pose_enc{i}"])
        assert _rel(pe[..., :3], ref[..., :3]) < 10 * tol, (i, _rel(pe[..., :3], ref[..., :3]))
        assert _quat_rot_err(pe, ref) < 10 * tol, i
        assert _rel(pe[..., 7:], ref[..., 7:]) < tol
        assert _rel(ctx["memory_tokens"][i], g[p + f"memory{i}"]) < tol
        for k, key in (("depth", "depth"), ("depth_conf", "depth_conf"), ("world_points", "points"),
                       ("world_points_conf", "points_conf")):
            assert _rel(ctx[k][i][:, :, ::7, ::7], g[p + f"{key}{i}"]) < 10 * tol, (i, k)


def test_reference_tree_names_match_oracle_decoder_keys():
    """Every parameter the oracle reads exists in the reference tree with the
    shape the oracle expects (a missing / renamed key raises KeyError above);
    the memory-free head lacks exactly the memory mechanic's parameters."""
    k8 = {k for k, _ in _keys()["m8"]}
    k0 = {k for k, _ in _keys()["m0"]}
    assert k0 < k8
    extra = {k.split(".")[0] for k in k8 - k0}
    assert extra == {"memory_token", "frame_proj", "alpha", "gated_update"}, extra


@pytest.mark.parametrize("prec", ["f32", "bf16"])
def test_training_gradients_match_reference(golden, prec):
    """Autograd through the oracle's alignment head over two chunks (memory
    recurrence, detached overlap tokens) reproduces the parameter gradients of
    the reference's own AlignmentHead in train mode (tests/golden/ref_train_grads.npz)."""
    from oracle.fixture_weights import TRAIN_CASE, grad_errors, train_inputs, train_loss
    g = golden("ref_train_grads")
    sd = {k: v.clone().requires_grad_(True) for k, v in head_state_dict("m8").items()}
    tok1, tok2 = train_inputs()
    ov = TRAIN_CASE["ov"]
    bf = prec == "bf16"
    r1 = O.alignment_head(sd, tok1, FIX_HW, ov, None, None, bf16=bf)
    r2 = O.alignment_head(sd, tok2, FIX_HW, ov, r1[3], r1[2], bf16=bf)
    loss = train_loss(r1, r2)
    loss.backward()
    assert abs(float(loss) / float(g[prec + "_loss"]) - 1) < 1e-5
    errs = grad_errors(g, prec, {k[len("alignment_head."):]: v.grad if v.grad is not None else torch.zeros_like(v)
                                  for k, v in sd.items()})
    worst = sorted(errs.items(), key=lambda kv: -kv[1])[:5]
    print(prec, "oracle vs reference gradients, worst:", worst)
    assert len(errs) > 100
    # fp32: summation order only (measured 1.4e-6); bf16-mixed: one-ulp bf16 flips between the
    # two emulations feed the small k / k_norm bias gradients (measured 7.4e-3)
    assert max(errs.values()) < (1e-4 if prec == "f32" else 1.5e-2), worst
