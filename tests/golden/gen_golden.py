"""Generate golden fixtures from the reference's own code (run in the build
container only; /root/reference does not exist on the GPU box).

What it runs:
  * ``aligned_vggt.layers.rope.RotaryPositionEmbedding`` and
    ``aligned_vggt.layers.gated_update.GatedUpdate`` imported directly from
    /root/reference (both import standalone);
  * pure-torch/numpy functions pulled out of modules whose module-level
    ``vggt`` imports fail, by parsing the file with ``ast`` and executing only
    those ``def``s (no stand-in for the missing ``vggt`` package is written);
  * ``transformers`` Dinov2WithRegistersModel and the Depth-Anything DPT neck /
    head (third-party, in-container) as independent pins of the DINOv2 stage
    and of the DPT decoder arithmetic.

Outputs are data only (inputs + expected outputs) in ``tests/golden/*.npz``.
Usage:  python tests/golden/gen_golden.py [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import ast
import os
import random
import sys
from typing import Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))


def extract(ref: str, relpath: str, names):
    """Exec only the named top-level functions of a reference file."""
    src = open(os.path.join(ref, relpath)).read()
    tree = ast.parse(src)
    keep = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in names]
    missing = set(names) - {n.name for n in keep}
    assert not missing, missing
    mod = ast.Module(body=keep, type_ignores=[])
    g = {"torch": torch, "np": np, "F": F, "Optional": Optional, "Tuple": Tuple, "random": random,
         "__name__": "golden_extract"}
    exec(compile(mod, relpath, "exec"), g)
    return {n: g[n] for n in names}


def extract_methods(ref: str, relpath: str, cls: str, names):
    """Exec the named methods of a reference class as free functions taking
    an explicit ``self`` (the class's own base, e.g. torchmetrics.Metric, is
    not needed by these bodies: they only read/write plain attributes)."""
    src = open(os.path.join(ref, relpath)).read()
    tree = ast.parse(src)
    (c,) = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == cls]
    keep = [n for n in c.body if isinstance(n, ast.FunctionDef) and n.name in names]
    assert {n.name for n in keep} == set(names)
    mod = ast.Module(body=keep, type_ignores=[])
    g = {"torch": torch, "np": np, "Tuple": Tuple, "__name__": "golden_extract"}
    exec(compile(mod, relpath, "exec"), g)
    return {n: g[n] for n in names}


def save(name, **arrays):
    out = {}
    for k, v in arrays.items():
        if isinstance(v, torch.Tensor):
            v = v.detach().cpu().numpy()
        out[k] = np.asarray(v)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print("wrote", name, {k: v.shape for k, v in out.items()})


def gen_rope(ref):
    sys.path.insert(0, ref)
    from aligned_vggt.layers.rope import RotaryPositionEmbedding  # reference module
    g = torch.Generator().manual_seed(11)
    rope = RotaryPositionEmbedding(frequency=100.0)
    cases = {}
    for ci, (B, H, N, D, maxp) in enumerate([(3, 2, 5, 16, 9), (2, 8, 16, 128, 20), (4, 8, 24, 64, 40)]):
        x = torch.randn(B, H, N, D, generator=g)
        pos = torch.randint(0, maxp, (B, N), generator=g)
        y = rope(x, pos)
        cases[f"x{ci}"] = x
        cases[f"pos{ci}"] = pos
        cases[f"y{ci}"] = y
    save("rope1d", **cases)


def gen_gated_update(ref):
    sys.path.insert(0, ref)
    from aligned_vggt.layers.gated_update import GatedUpdate  # reference module
    torch.manual_seed(5)
    save("gated_update_nparams", d512_n8=np.array(sum(p.numel() for p in GatedUpdate(512, 8).parameters())))
    for D, N, tag in [(64, 8, "d64"), (32, 4, "d32")]:
        m = GatedUpdate(D, N).eval()
        mem = F.normalize(torch.randn(2, N, D), dim=-1)
        upd = torch.randn(2, 1, D) * 3.0
        with torch.no_grad():
            out = m(mem, upd)
        sd = {"p." + k: v for k, v in m.state_dict().items()}
        save("gated_update_" + tag, memory=mem, update=upd, out=out,
             nparams=np.array(sum(p.numel() for p in m.parameters())), **sd)


def gen_chunks(ref):
    fn = extract(ref, "aligned_vggt/utils/data.py", ["generate_chunks"])["generate_chunks"]
    rows = []
    for n in [1, 4, 5, 8, 14, 16, 17, 20, 33, 64, 100, 512]:
        for w in [2, 5, 8, 16, 75]:
            for ov in [0, 1, 2, 4, 30]:
                if ov >= w:
                    continue
                for ci, c in enumerate(fn(n, "chunk_overlap", w, ov)):
                    for f in c:
                        rows.append((n, w, ov, ci, f))
    save("generate_chunks", rows=np.array(rows, dtype=np.int64))


def gen_geometry(ref):
    fns = extract(ref, "aligned_vggt/utils/geometry.py", ["averagePoseEncodings"])
    g = torch.Generator().manual_seed(3)
    enc = torch.randn(6, 4, 7, generator=g, dtype=torch.float64).float()
    enc[..., 3:7] = F.normalize(enc[..., 3:7] * 0.1 + torch.tensor([0, 0, 0, 1.0]), dim=-1)
    out = fns["averagePoseEncodings"](enc)
    save("average_pose_encodings", enc=enc, out=out)


def gen_alignment(ref):
    fns = extract(ref, "aligned_vggt/utils/alignment.py",
                  ["umeyama", "scale_lse_solver", "apply_sim3_alignment_on_point_maps", "apply_sim3_alignment_on_c2w"])
    rng = np.random.default_rng(9)
    x = rng.normal(size=(3, 50))
    ang = 0.4
    R = np.array([[np.cos(ang), -np.sin(ang), 0], [np.sin(ang), np.cos(ang), 0], [0, 0, 1.0]])
    y = 1.7 * R @ x + np.array([[0.3], [-1.0], [2.0]]) + rng.normal(size=(3, 50)) * 1e-3
    r, t, c = fns["umeyama"](x, y)
    s = fns["scale_lse_solver"](x.reshape(-1), y.reshape(-1))
    pm = torch.randn(2, 3, 4, 5, 3, dtype=torch.float32)
    T = torch.eye(4).repeat(2, 1, 1)
    T[:, :3, :3] = torch.tensor(R, dtype=torch.float32)
    T[:, :3, 3] = torch.tensor([0.5, -0.2, 1.0])
    sc = torch.tensor([1.5, 0.7])
    pm_out = fns["apply_sim3_alignment_on_point_maps"](pm, T, sc)
    poses = torch.eye(4).repeat(2, 3, 1, 1)
    poses[..., :3, 3] = torch.randn(2, 3, 3)
    c2w_out = fns["apply_sim3_alignment_on_c2w"](poses.clone(), T, sc)
    save("alignment_utils", x=x, y=y, r=r, t=t, c=np.array(c), s=np.array(s), pm=pm, T=T, sc=sc, pm_out=pm_out,
         poses=poses, c2w_out=c2w_out)


def gen_irls(ref):
    fns = extract(ref, "aligned_vggt/models/pointAligned_wrapped_vggt.py",
                  ["weighted_umeyama_sim3", "irls_sim3_umeyama"])
    g = torch.Generator().manual_seed(21)
    src = torch.randn(2, 6, 8, 3, generator=g)
    ang = 0.3
    R = torch.tensor([[1, 0, 0], [0, np.cos(ang), -np.sin(ang)], [0, np.sin(ang), np.cos(ang)]], dtype=torch.float32)
    dst = 0.8 * src @ R.T + torch.tensor([1.0, 2.0, -0.5])
    dst = dst + 0.01 * torch.randn(dst.shape, generator=g)
    dst[0, 0, :5] += 3.0  # outliers for the Huber weights
    cs = 1 + torch.rand(2, 6, 8, generator=g) * 5
    cd = 1 + torch.rand(2, 6, 8, generator=g) * 5
    r, t, s = fns["irls_sim3_umeyama"](src, dst, cs, cd)
    save("irls_sim3", src=src, dst=dst, conf_src=cs, conf_dst=cd, r=r, t=t, s=np.array(float(s)))


def gen_irls_batch(ref):
    """Three independent problems with 5% gross outliers and ragged confidences
    (the batched GPU kernel solves them in one call)."""
    fns = extract(ref, "aligned_vggt/models/pointAligned_wrapped_vggt.py",
                  ["weighted_umeyama_sim3", "irls_sim3_umeyama"])
    g = torch.Generator().manual_seed(33)
    out = {}
    for b in range(3):
        src = torch.randn(3, 24, 32, 3, generator=g) * 4 + torch.tensor([0.0, 0.0, 10.0])
        ang = 0.2 + 0.3 * b
        ax = F.normalize(torch.randn(3, generator=g), dim=0)
        K = torch.tensor([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
        R = torch.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K
        dst = (0.5 + 0.4 * b) * src @ R.T + torch.randn(3, generator=g)
        dst = dst + 0.02 * torch.randn(dst.shape, generator=g)
        out_mask = torch.rand(src.shape[:-1], generator=g) < 0.05
        dst[out_mask] += torch.randn(int(out_mask.sum()), 3, generator=g) * 5
        cs = 1 + torch.rand(src.shape[:-1], generator=g) * 4
        cd = 1 + torch.rand(src.shape[:-1], generator=g) * 4
        cs[0, :4] = 1.0  # a low-confidence band below the median threshold
        r, t, s = fns["irls_sim3_umeyama"](src, dst, cs, cd)
        out.update({f"src{b}": src, f"dst{b}": dst, f"cs{b}": cs, f"cd{b}": cd, f"r{b}": r, f"t{b}": t,
                    f"s{b}": np.array(float(s))})
    save("irls_sim3_batch", **out)


def gen_trajectory_metrics(ref):
    """ATE / RPE (eval/trajectory_metrics.py:28-77, :154-223): the update /
    compute bodies run on plain attribute holders."""
    from types import SimpleNamespace
    ate = extract_methods(ref, "eval/trajectory_metrics.py", "AbsoluteTrajectoryError", ["update", "compute"])
    rpe = extract_methods(ref, "eval/trajectory_metrics.py", "RelativePoseError", ["update", "compute"])
    g = torch.Generator().manual_seed(7)
    N = 40
    yaw = torch.cumsum(torch.randn(N, generator=g) * np.deg2rad(2.0), 0)
    gt = torch.eye(4).repeat(N, 1, 1)
    gt[:, 0, 0] = torch.cos(yaw)
    gt[:, 0, 2] = torch.sin(yaw)
    gt[:, 2, 0] = -torch.sin(yaw)
    gt[:, 2, 2] = torch.cos(yaw)
    gt[:, :3, 3] = torch.cumsum(torch.stack([torch.sin(yaw), torch.zeros(N), torch.cos(yaw)], -1), 0)
    pred = gt.clone()
    dyaw = torch.randn(N, generator=g) * 0.02
    c, s_ = torch.cos(dyaw), torch.sin(dyaw)
    Rz = torch.eye(4).repeat(N, 1, 1)
    Rz[:, 0, 0], Rz[:, 0, 1], Rz[:, 1, 0], Rz[:, 1, 1] = c, -s_, s_, c
    pred = pred @ Rz
    pred[:, :3, 3] += torch.randn(N, 3, generator=g) * 0.05
    out = {"gt": gt, "pred": pred}
    for det in (False, True):
        st = SimpleNamespace(errors=torch.tensor([], dtype=torch.float32),
                             per_dim_errors=torch.tensor([], dtype=torch.float32), detailed=det)
        ate["update"](st, pred[:25], gt[:25])
        ate["update"](st, pred[25:], gt[25:])
        r = ate["compute"](st)
        for k, v in r.items():
            out[f"ate_{int(det)}_{k}"] = np.array(v)
    for delta in (1, 3):
        st = SimpleNamespace(trans_errors=torch.tensor([], dtype=torch.float32),
                             rot_errors=torch.tensor([], dtype=torch.float32), detailed=True, delta=delta)
        rpe["update"](st, pred, gt)
        rpe["update"](st, pred[:2], gt[:2])  # N <= delta for delta 3: ignored
        for k, v in rpe["compute"](st).items():
            out[f"rpe_{delta}_{k}"] = np.array(v)
    save("trajectory_metrics", **out)


def gen_scale_alignment(ref):
    """GT-based output alignment (aligned_vggt/utils/alignment.py:131-323)."""
    fns = extract(ref, "aligned_vggt/utils/alignment.py",
                  ["scale_lse_solver", "per_frame_scale_alignment_from_poses", "per_chunk_scale_alignment_from_poses",
                   "scale_alignment_from_poses", "scale_align_from_depths"])
    g = torch.Generator().manual_seed(17)
    B, S, H, W = 2, 6, 5, 7

    def preds():
        gg = torch.Generator().manual_seed(18)
        return {"pose_enc": torch.randn(B, S, 9, generator=gg), "depth": torch.rand(B, S, H, W, 1, generator=gg) + 0.5,
                "depth_conf": torch.rand(B, S, H, W, generator=gg) + 1,
                "world_points": torch.randn(B, S, H, W, 3, generator=gg)}
    extr = torch.randn(B, S, 3, 4, generator=g)
    depths = torch.rand(B, S, H, W, generator=g) * 3 + 0.2
    mask = torch.rand(B, S, H, W, generator=g) > 0.2
    out = {"extr": extr, "depths": depths, "mask": mask}
    p0 = preds()
    out.update({"in_" + k: v for k, v in p0.items()})
    for name, call in (("scale_poses", lambda p: fns["scale_alignment_from_poses"](p, {"extrinsics": extr})),
                       ("scale_poses_w3", lambda p: fns["scale_alignment_from_poses"](p, {"extrinsics": extr}, 3)),
                       ("frame_scale", lambda p: fns["per_frame_scale_alignment_from_poses"](p, {"extrinsics": extr})),
                       ("depth_scale", lambda p: fns["scale_align_from_depths"](
                           p, {"depths": depths[..., None], "point_masks": mask}))):
        p = preds()
        call(p)
        for k in ("pose_enc", "depth", "world_points"):
            out[f"{name}_{k}"] = p[k]
        sc = p["alignment_scales"]
        out[f"{name}_scales"] = np.array([np.asarray(v, dtype=np.float64) for v in sc], dtype=np.float64)
    # per chunk: lists of chunks
    pc = preds()
    chunked = {k: [v[:, :3].clone(), v[:, 3:].clone()] for k, v in pc.items()}
    fns["per_chunk_scale_alignment_from_poses"](chunked, {"extrinsics": [extr[:, :3], extr[:, 3:]]})
    for k in ("pose_enc", "depth", "world_points"):
        out[f"chunk_scale_{k}"] = torch.cat(chunked[k], 1)
    out["chunk_scale_scales"] = torch.stack(chunked["alignment_scales_per_chunk"])
    save("scale_alignment", **out)


def gen_small_fns(ref):
    mr = extract(ref, "aligned_vggt/models/featureAligned_vggt.py", ["merge_results"])["merge_results"]
    se = extract(ref, "aligned_vggt/heads/alignment_head.py", ["slice_expand_and_flatten"])["slice_expand_and_flatten"]
    a = torch.arange(2 * 3 * 7, dtype=torch.float32).view(2, 3, 7)
    b = -torch.arange(2 * 4 * 7, dtype=torch.float32).view(2, 4, 7)
    tok = torch.randn(1, 2, 3, 5)
    save("small_fns", a=a, b=b, merged0=mr(a, b, 0, 1), merged2=mr(a, b, 2, 1), tok=tok, sef=se(tok, 2, 4))


def gen_dinov2():
    """Independent third-party pin of the DINOv2 stage (ext)."""
    from transformers import Dinov2WithRegistersConfig, Dinov2WithRegistersModel
    cfg = Dinov2WithRegistersConfig(hidden_size=64, num_hidden_layers=2, num_attention_heads=4, intermediate_size=256,
                                    image_size=56, patch_size=14, num_register_tokens=4, layerscale_value=1.0,
                                    layer_norm_eps=1e-6, hidden_act="gelu", qkv_bias=True)
    torch.manual_seed(2)
    m = Dinov2WithRegistersModel(cfg).eval()
    with torch.no_grad():
        for prm in m.parameters():
            prm.copy_(torch.randn_like(prm) * 0.05)
        for blk in m.encoder.layer:
            blk.layer_scale1.lambda1.fill_(1.0)
            blk.layer_scale2.lambda1.fill_(1.0)
    # Map to VGGT/DINOv2 (aggregator.patch_embed.*) names.
    hf = m.state_dict()
    sd = {
        "cls_token": hf["embeddings.cls_token"],
        "pos_embed": hf["embeddings.position_embeddings"],
        "register_tokens": hf["embeddings.register_tokens"],
        "patch_embed.proj.weight": hf["embeddings.patch_embeddings.projection.weight"],
        "patch_embed.proj.bias": hf["embeddings.patch_embeddings.projection.bias"],
        "norm.weight": hf["layernorm.weight"],
        "norm.bias": hf["layernorm.bias"],
    }
    for i in range(cfg.num_hidden_layers):
        h = f"encoder.layer.{i}."
        o = f"blocks.{i}."
        sd[o + "norm1.weight"] = hf[h + "norm1.weight"]
        sd[o + "norm1.bias"] = hf[h + "norm1.bias"]
        sd[o + "attn.qkv.weight"] = torch.cat([hf[h + f"attention.attention.{n}.weight"] for n in ("query", "key", "value")])
        sd[o + "attn.qkv.bias"] = torch.cat([hf[h + f"attention.attention.{n}.bias"] for n in ("query", "key", "value")])
        sd[o + "attn.proj.weight"] = hf[h + "attention.output.dense.weight"]
        sd[o + "attn.proj.bias"] = hf[h + "attention.output.dense.bias"]
        sd[o + "ls1.gamma"] = hf[h + "layer_scale1.lambda1"]
        sd[o + "norm2.weight"] = hf[h + "norm2.weight"]
        sd[o + "norm2.bias"] = hf[h + "norm2.bias"]
        sd[o + "mlp.fc1.weight"] = hf[h + "mlp.fc1.weight"]
        sd[o + "mlp.fc1.bias"] = hf[h + "mlp.fc1.bias"]
        sd[o + "mlp.fc2.weight"] = hf[h + "mlp.fc2.weight"]
        sd[o + "mlp.fc2.bias"] = hf[h + "mlp.fc2.bias"]
        sd[o + "ls2.gamma"] = hf[h + "layer_scale2.lambda1"]
    g = torch.Generator().manual_seed(4)
    outs = {}
    for tag, (H, W) in {"sq": (56, 56), "rect": (28, 56)}.items():
        img = torch.randn(2, 3, H, W, generator=g)
        with torch.no_grad():
            last = m(pixel_values=img).last_hidden_state  # already final-layernormed
        outs[f"img_{tag}"] = img
        outs[f"patch_{tag}"] = last[:, 1 + cfg.num_register_tokens:]
    save("dinov2_hf", **outs, **{"sd." + k: v for k, v in sd.items()})


def gen_dpt_hf():
    """Independent third-party pin of the DPT decoder arithmetic (ext VGGT
    ``heads/dpt_head.py``, called at featureAligned_vggt.py:166 / :183): the
    in-container ``transformers`` Depth-Anything neck + depth head, a DPT of
    the same lineage -- reassemble (1x1 projection; ConvTranspose 4x / 2x,
    identity, 3x3 stride-2 conv), the 3x3 ``layer*_rn`` convs, FeatureFusion
    (pre-activation residual units, bilinear ``align_corners=True`` resize,
    1x1 projection) and the output convs with the resize to full resolution.
    Two VGGT deviations are configured, not patched: the residual units'
    ReLU is in place (VGGT's ``nn.ReLU(inplace=True)``, so the skip adds
    relu(x)), and the pre-activation head output is taken from ``conv3`` by a
    forward hook.  Not covered here: DPT's positional embedding (VGGT-only),
    the output activations.  Weights are stored under the VGGT DPTHead names."""
    import torch.nn as nn
    from transformers import DepthAnythingConfig
    from transformers.models.depth_anything.modeling_depth_anything import (DepthAnythingDepthEstimationHead,
                                                                            DepthAnythingNeck)
    cin, oc, feat = 256, [32, 32, 64, 64], 64  # cin: the HIP row LayerNorm takes C % 256 == 0
    cfg = DepthAnythingConfig(reassemble_hidden_size=cin, neck_hidden_sizes=oc, reassemble_factors=[4, 2, 1, 0.5],
                              fusion_hidden_size=feat, head_hidden_size=32, head_in_index=-1, patch_size=14,
                              depth_estimation_type="metric", max_depth=1)
    torch.manual_seed(6)
    neck, head = DepthAnythingNeck(cfg).eval(), DepthAnythingDepthEstimationHead(cfg).eval()
    with torch.no_grad():
        for mod in (neck, head):
            for name, prm in mod.named_parameters():
                fan_in = prm[0].numel() if prm.dim() > 1 else 1
                prm.copy_(torch.randn_like(prm) * (0.5 / fan_in ** 0.5 if prm.dim() > 1 else 0.05))
    for fl in neck.fusion_stage.layers:
        for rl in (fl.residual_layer1, fl.residual_layer2):
            rl.activation1 = nn.ReLU(inplace=True)
    hf = {**{"neck." + k: v for k, v in neck.state_dict().items()}, **{"head." + k: v for k, v in head.state_dict().items()}}
    sd = {"norm.weight": torch.ones(cin), "norm.bias": torch.zeros(cin)}
    for i in range(4):
        for t in ("weight", "bias"):
            sd[f"projects.{i}.{t}"] = hf[f"neck.reassemble_stage.layers.{i}.projection.{t}"]
            if i != 2:
                sd[f"resize_layers.{i}.{t}"] = hf[f"neck.reassemble_stage.layers.{i}.resize.{t}"]
        sd[f"scratch.layer{i + 1}_rn.weight"] = hf[f"neck.convs.{i}.weight"]
    for j in range(4):  # the fusion stage runs the deepest level first: layer j = refinenet(4 - j)
        d, s = f"neck.fusion_stage.layers.{j}.", f"scratch.refinenet{4 - j}."
        for t in ("weight", "bias"):
            sd[s + f"out_conv.{t}"] = hf[d + f"projection.{t}"]
            for u in (1, 2):
                for c in (1, 2):
                    if j == 0 and u == 1:
                        continue  # refinenet4 has no residual unit 1 (has_residual=False)
                    sd[s + f"resConfUnit{u}.conv{c}.{t}"] = hf[d + f"residual_layer{u}.convolution{c}.{t}"]
    g = torch.Generator().manual_seed(3)
    for t in ("weight", "bias"):
        sd[f"scratch.output_conv1.{t}"] = hf[f"head.conv1.{t}"]
        sd[f"scratch.output_conv2.0.{t}"] = hf[f"head.conv2.{t}"]
        extra = torch.randn((1,) + hf[f"head.conv3.{t}"].shape[1:], generator=g) * 0.05  # conf channel (unpinned)
        sd[f"scratch.output_conv2.2.{t}"] = torch.cat([hf[f"head.conv3.{t}"], extra], 0)
    F_, ph, pw = 2, 5, 7
    tokens = torch.randn(F_, ph * pw, cin, generator=g)
    x = F.layer_norm(tokens, (cin,), eps=1e-5)
    hs = [torch.cat([torch.zeros(F_, 1, cin), x], 1) for _ in range(4)]  # index 0 = the (dropped) cls slot
    cap = {}
    hooks = [neck.reassemble_stage.layers[i].register_forward_hook(
        lambda m, a, o, i=i: cap.__setitem__(f"reassemble{i}", o.clone())) for i in range(4)]
    hooks += [neck.convs[i].register_forward_hook(
        lambda m, a, o, i=i: cap.__setitem__(f"rn{i}", o.clone())) for i in range(4)]
    hooks += [neck.fusion_stage.layers[j].register_forward_hook(
        lambda m, a, o, j=j: cap.__setitem__(f"fused{j}", o.clone())) for j in range(4)]
    hooks.append(head.conv3.register_forward_hook(lambda m, a, o: cap.__setitem__("head_pre", o.clone())))
    with torch.no_grad():
        feats = neck(hs, ph, pw)
        out = head(feats, ph, pw)
    for h in hooks:
        h.remove()
    save("dpt_hf", tokens=tokens, ph=ph, pw=pw, out_sigmoid=out, **cap, **{"sd." + k: v for k, v in sd.items()})


# ----------------------------------------------------------------------------
# the reference-authored alignment path, run on the test-only vggt shim
# (weights / inputs from oracle.fixture_weights, not stored)
# ----------------------------------------------------------------------------
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
from oracle.fixture_weights import ALIGN_CASES, FA_RUNS, FIX_HW, FIX_SEED  # noqa: E402
from oracle.fixture_weights import fa_feed, fa_gt_poses  # noqa: E402


def _ref_alignment_modules(ref):
    for p in (ROOT, ref):
        if p not in sys.path:
            sys.path.insert(0, p)
    import vggt_shim
    vggt_shim.install()
    from aligned_vggt.heads.alignment_head import AlignmentHead  # reference module
    from aligned_vggt.layers.cross_attention import CrossAttentionBlock  # reference module
    from aligned_vggt.layers.rope import RotaryPositionEmbedding  # reference module
    from aligned_vggt.models.featureAligned_vggt import FeatureAlignedVGGT  # reference module
    return vggt_shim, AlignmentHead, CrossAttentionBlock, RotaryPositionEmbedding, FeatureAlignedVGGT


def gen_ref_cross_attention(ref):
    """CrossAttentionBlock (cross_attention.py:80-131) in its two roles: a
    decoder block (512 wide, 1 query vs S frames + 8 memory tokens) and a
    temporal block (1024 wide, B*P groups of S queries vs T overlap keys)."""
    shim, _, CAB, Rope, _ = _ref_alignment_modules(ref)
    from oracle.fixture_weights import fixture_tensor, load_fixture_weights_
    out = {}
    S, T = 3, 2
    seq = torch.arange(S)
    cases = {
        "dec": (512, (2, 1, 512), (2, 11, 512), torch.zeros(1, dtype=torch.long),
                torch.cat([torch.arange(3), torch.arange(8) + 6])),
        "tmp": (1024, (36, S, 1024), (36, T, 1024), seq + (S - (T - 1)), torch.cat([seq[:1], seq[-(T - 1):]])),
    }
    for tag, (dim, xs, ys, pq, pk) in cases.items():
        torch.manual_seed(0)
        blk = CAB(dim=dim, num_heads=8, mlp_ratio=4.0, qkv_bias=True, proj_bias=True, ffn_bias=True, init_values=0.01,
                  qk_norm=True, rope=Rope(frequency=100)).eval()
        load_fixture_weights_(blk, FIX_SEED, prefix=f"cab_{tag}.")
        x = fixture_tensor(f"cab_{tag}.x", xs, FIX_SEED)
        y = fixture_tensor(f"cab_{tag}.y", ys, FIX_SEED)
        pos = (pq.view(1, -1).expand(xs[0], -1), pk.view(1, -1).expand(xs[0], -1))
        for prec in ("f32", "bf16"):
            with torch.no_grad(), shim.bf16_mixed(prec == "bf16"):
                o = blk(x, y, pos=pos)
            out[f"{tag}_{prec}"] = o.float()
        out[f"{tag}_pos_q"], out[f"{tag}_pos_k"] = pq, pk
    save("ref_cross_attention", **out)


def gen_ref_alignment_head(ref):
    """AlignmentHead.forward (alignment_head.py:224-345, eval) for first and
    continuation chunks (T = ov + 1 overlap tokens), with and without memory,
    B in {1, 2}, a shorter tail chunk; fp32 and emulated bf16-mixed.  Plus
    _decode_alignments (:427-540) alone and the reference tree's parameter
    names / shapes."""
    import json
    shim, AH, _, _, _ = _ref_alignment_modules(ref)
    from oracle.fixture_weights import fixture_tensor, load_fixture_weights_
    H, W = FIX_HW
    P = 5 + (H // 14) * (W // 14)
    heads = {}
    for tag, nm in (("m8", 8), ("m0", 0)):
        torch.manual_seed(0)
        heads[tag] = load_fixture_weights_(AH(in_dim=2048, patch_size=14, num_memory_tokens=nm,
                                              temporal_attention=True).eval(), FIX_SEED, prefix="alignment_head.")
    out = {}
    for prec in ("f32", "bf16"):
        for case, head, B, S, nov, prev in ALIGN_CASES:
            tok = fixture_tensor(f"ah.{case}.tokens", (B, S, P, 2048), FIX_SEED)
            ov = out[f"{prev}_{prec}_new_ov"] if prev else None
            mem = out.get(f"{prev}_{prec}_memory") if prev else None
            with torch.no_grad(), shim.bf16_mixed(prec == "bf16"):
                cs, fs, m, nov_t = heads[head](tok, (H, W), nov, overlap_tokens=ov, memory_tokens=mem)
            out[f"{case}_{prec}_chunk_sim3"] = cs.float()
            out[f"{case}_{prec}_frame_se3"] = fs.float()
            if m is not None:
                out[f"{case}_{prec}_memory"] = m.float()
            out[f"{case}_{prec}_new_ov"] = nov_t.float()
    # _decode_alignments alone (fp32: autocast is off there in the reference)
    h = heads["m8"]
    ft = fixture_tensor("dec.tokens1", (2, 4, 1024), FIX_SEED)
    with torch.no_grad():
        d1 = h._decode_alignments(ft, 2, True, memory_tokens=None)
        ft2 = fixture_tensor("dec.tokens2", (2, 4, 1024), FIX_SEED)
        d2 = h._decode_alignments(ft2, 2, False, memory_tokens=d1[2])
    for i, d in ((1, d1), (2, d2)):
        for name, v in zip(("chunk_sim3", "frame_se3", "memory"), d):
            out[f"dec{i}_{name}"] = v.float()
    save("ref_alignment_head", **out)
    keys = {tag: [[k, list(v.shape)] for k, v in hd.state_dict().items()] for tag, hd in heads.items()}
    with open(os.path.join(HERE, "ref_alignment_keys.json"), "w") as f:
        json.dump(keys, f)
    print("wrote ref_alignment_keys.json", {k: len(v) for k, v in keys.items()})


def gen_ref_train_grads(ref):
    """Training gradients of the reference's own AlignmentHead
    (alignment_head.py:224-540 in train mode: torch.utils.checkpoint around every
    block, the overlap tokens detached at :260, the memory recurrence keeping its
    gradient at :482-484, GatedUpdate's detached gate input, gated_update.py:69)
    over two chunks, for the fixed loss of oracle.fixture_weights.train_loss --
    a linear functional of both chunks' Sim(3) / SE(3) outputs, chunk 2's memory
    and new overlap tokens.  Frame dropout off (drop_prob_nonoverlap = 0; its mask
    is tested separately).  fp32 and emulated bf16-mixed (forward AND backward
    inside the emulation).
    Stored per parameter: the full gradient when small, else the gradient at
    fixed sampled indices plus its norm (oracle.fixture_weights.grad_sample)."""
    shim, AH, _, _, _ = _ref_alignment_modules(ref)
    import aligned_vggt.heads.alignment_head as ahmod  # the reference module
    from oracle.fixture_weights import TRAIN_CASE, grad_sample, load_fixture_weights_, train_inputs, train_loss
    S, ov = TRAIN_CASE["S"], TRAIN_CASE["ov"]
    H, W = FIX_HW
    out = {}
    # torch.utils.checkpoint (alignment_head.py:361, :385, :498, :527) recomputes each
    # block in backward outside the autocast emulation's TorchFunctionMode, so its
    # recompute would not match the forward; a direct call has identical gradients
    # (non-reentrant checkpointing only trades memory for recompute)
    real_ckpt = ahmod.checkpoint
    ahmod.checkpoint = lambda fn, *a, use_reentrant=None, **k: fn(*a, **k)
    for prec in ("f32", "bf16"):
        torch.manual_seed(0)
        head = load_fixture_weights_(AH(in_dim=2048, patch_size=14, num_memory_tokens=8, temporal_attention=True),
                                     FIX_SEED, prefix="alignment_head.").train()
        head.drop_prob_nonoverlap = 0.0
        tok1, tok2 = train_inputs()
        with shim.bf16_mixed(prec == "bf16"):
            o1 = head(tok1, (H, W), ov)
            o2 = head(tok2, (H, W), ov, overlap_tokens=o1[3], memory_tokens=o1[2])
            loss = train_loss(o1, o2)
            loss.backward()
        out[f"{prec}_loss"] = loss.detach().float()
        for name, p in head.named_parameters():
            if p.grad is None:
                continue
            for k, v in grad_sample(name, p.grad.float()).items():
                out[f"{prec}.{name}.{k}"] = v
    ahmod.checkpoint = real_ckpt
    save("ref_train_grads", **out)


def gen_ref_feature_aligned(ref):
    """FeatureAlignedVGGT.forward composition (featureAligned_vggt.py:73-225) over
    whole chunk sequences: the reference's alignment head + Sim(3)/SE(3)
    composition + Markley mean + context bookkeeping, with stub encoders
    returning fixed outputs.  Dense maps are stored at every 7th pixel."""
    import json
    shim, _, _, _, FA = _ref_alignment_modules(ref)
    from oracle import vggt_oracle as O
    from oracle.fixture_weights import fixture_tensor, load_fixture_weights_
    H, W = FIX_HW
    torch.manual_seed(0)
    fa = FA(img_size=518, patch_size=14, embed_dim=1024, enable_camera=True, enable_point=True, enable_depth=True,
            enable_track=False, num_memory_tokens=8).eval()
    load_fixture_weights_(fa.alignment_head, FIX_SEED, prefix="alignment_head.")
    out = {}
    for prec in ("f32", "bf16"):
        for run, N, w, ov, use_gt in FA_RUNS:
            imgs = fixture_tensor(f"fa.{run}.images", (1, N, 3, H, W), FIX_SEED, "uniform")
            ctx = None
            chunks = O.generate_chunks(N, w, ov)
            for i, ids in enumerate(chunks):
                feed = fa_feed(run, i, len(ids))
                shim._Feed.tokens = feed["tokens"]
                for k in ("pose_enc", "depth", "depth_conf", "points", "points_conf"):
                    setattr(shim._Feed, k, feed[k])
                gt = fa_gt_poses(run, i, len(ids)) if use_gt else None
                with torch.no_grad(), shim.bf16_mixed(prec == "bf16"):
                    ctx = fa(imgs[:, ids], ov, ctx, gt_poses=gt)
            p = f"{run}_{prec}_"
            for i in range(len(chunks)):
                out[p + f"pose_enc{i}"] = ctx["pose_enc"][i]
                out[p + f"memory{i}"] = ctx["memory_tokens"][i]
                out[p + f"depth{i}"] = ctx["depth"][i][:, :, ::7, ::7]
                out[p + f"depth_conf{i}"] = ctx["depth_conf"][i][:, :, ::7, ::7]
                out[p + f"points{i}"] = ctx["world_points"][i][:, :, ::7, ::7]
                out[p + f"points_conf{i}"] = ctx["world_points_conf"][i][:, :, ::7, ::7]
            out[p + "chunk_sim3"] = ctx["chunk_sim3_alignment_enc"]
            out[p + "frame_se3"] = ctx["frame_se3_alignment_enc"]
            out[p + "overlap_tokens"] = ctx["overlap_tokens"]
            out[p + "nchunks"] = np.array(len(chunks))
    save("ref_feature_aligned", **out)
    # set_config (featureAligned_vggt.py:34-46) rebuilds the alignment head
    from types import SimpleNamespace
    cfg = SimpleNamespace(enable_camera=True, enable_point=False, enable_depth=True, enable_track=False,
                          num_memory_tokens=0, patch_size=14, temporal_attention=True)
    fa.set_config(cfg)
    info = {"cfg": vars(cfg), "keys": [[k, list(v.shape)] for k, v in fa.state_dict().items()],
            "heads_none": [n for n in ("camera_head", "point_head", "depth_head", "track_head")
                           if getattr(fa, n) is None], "enable_memory": fa.enable_memory}
    with open(os.path.join(HERE, "ref_set_config.json"), "w") as f:
        json.dump(info, f)
    print("wrote ref_set_config.json", len(info["keys"]), info["heads_none"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default=None, help="comma-separated generator names (e.g. irls_batch,trajectory_metrics)")
    a = ap.parse_args()
    if a.only:
        for n in a.only.split(","):
            globals()["gen_" + n](a.ref) if n not in ("dinov2", "dpt_hf") else globals()["gen_" + n]()
        return
    gen_rope(a.ref)
    gen_gated_update(a.ref)
    gen_chunks(a.ref)
    gen_geometry(a.ref)
    gen_alignment(a.ref)
    gen_irls(a.ref)
    gen_irls_batch(a.ref)
    gen_trajectory_metrics(a.ref)
    gen_scale_alignment(a.ref)
    gen_small_fns(a.ref)
    gen_dinov2()
    gen_dpt_hf()
    gen_ref_cross_attention(a.ref)
    gen_ref_alignment_head(a.ref)
    gen_ref_feature_aligned(a.ref)


if __name__ == "__main__":
    main()
