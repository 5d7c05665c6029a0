"""CPU oracle for the point-aligned VGGT path (BASELINE config 1) and its
robust Sim(3) alignment.

TEST INFRASTRUCTURE ONLY: imported by ``tests/`` (and nothing in the product)
as the checker of the HIP kernels ``vggt_irls_sim3`` / ``vggt_sim3_points`` and
of ``aligned_vggt.models.pointAligned_wrapped_vggt.VGGT``.

Restates aligned_vggt/models/pointAligned_wrapped_vggt.py:14-305 and
aligned_vggt/utils/alignment.py:491-594 in fp32 torch on the CPU.  The
IRLS / weighted Umeyama restatement is pinned by tests/golden/irls_sim3*.npz
(outputs of the reference's own functions); the backbone parts reuse
``vggt_oracle`` (parity unpinned except the DINOv2 stage, see there).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from . import vggt_oracle as O

Tensor = torch.Tensor


def weighted_umeyama_sim3(src: Tensor, dst: Tensor, weights: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    """pointAligned_wrapped_vggt.py:159-219."""
    assert src.ndim == 2 and src.shape[1] == 3 and dst.shape == src.shape
    M = src.shape[0]
    w = weights.view(M, 1)
    W = weights.sum()
    if W < 1e-6:
        raise ValueError("Total weight too small for meaningful estimation")
    mu_x = (w * src).sum(dim=0) / W
    mu_y = (w * dst).sum(dim=0) / W
    xc, yc = src - mu_x, dst - mu_y
    Sigma = ((w * yc).T @ xc) / W
    U, Sv, Vh = torch.linalg.svd(Sigma, full_matrices=True)
    V = Vh.T
    d = torch.sign(torch.det(U @ V.T)).item()
    D = torch.diag(torch.tensor([1.0, 1.0, d], dtype=src.dtype))
    r = U @ D @ V.T
    var_x = (weights * (xc ** 2).sum(dim=1)).sum() / W
    s = (Sv * D).sum() / var_x  # (sic) Sv broadcast against the 3x3 diag, pointAligned :214
    t = mu_y - s * (r @ mu_x)
    return r, t, s


def irls_sim3_umeyama(src: Tensor, dst: Tensor, conf_src: Tensor, conf_dst: Tensor,
                      conf_threshold_factor: float = 0.5, delta: float = 0.1, max_iters: int = 20,
                      tol: float = 1e-9) -> Tuple[Tensor, Tensor, Tensor]:
    """pointAligned_wrapped_vggt.py:221-305."""
    assert src.shape[0] == dst.shape[0]
    src, dst = src.reshape(-1, 3), dst.reshape(-1, 3)
    comb = torch.sqrt(conf_src.reshape(-1) * conf_dst.reshape(-1))
    mask = comb >= conf_threshold_factor * torch.median(comb)
    src, dst, comb = src[mask], dst[mask], comb[mask]
    R, t, s = weighted_umeyama_sim3(src, dst, comb.clone())
    lR, lt, ls = R.clone(), t.clone(), s.clone()
    for _ in range(max_iters):
        res = torch.linalg.norm(s * (src @ R.T) + t - dst, dim=1)
        rw = torch.where(res <= delta, torch.ones_like(res), delta / res.clamp_min(1e-12))
        R, t, s = weighted_umeyama_sim3(src, dst, comb * rw)
        dR, dt, ds = torch.norm(R - lR), torch.norm(t - lt), torch.abs(s - ls)
        lR, lt, ls = R.clone(), t.clone(), s.clone()
        if dR < tol and dt < tol and ds < tol:
            break
    return R, t, s


def apply_sim3_alignment_on_point_maps(pm: Tensor, T: Tensor, sc: Tensor) -> Tensor:
    """alignment.py:491-526."""
    B, S, H, W, _ = pm.shape
    p = pm * sc.view(B, 1, 1, 1, 1)
    p = torch.cat([p, torch.ones_like(p[..., :1])], -1).view(B, -1, 4)
    out = torch.matmul(T.unsqueeze(1).expand(-1, S * H * W, -1, -1), p.unsqueeze(-1)).squeeze(-1)
    return out.view(B, S, H, W, 4)[..., :3]


def apply_sim3_alignment_on_w2c(extr: Tensor, T: Tensor, sc: Tensor) -> Tensor:
    """alignment.py:528-594."""
    B, S = extr.shape[:2]
    poses = torch.stack([O.closed_form_inverse_se3(extr[b]) for b in range(B)])
    poses[:, :, :3, 3] = poses[:, :, :3, 3] * sc.view(B, 1, 1)
    poses = torch.matmul(T.unsqueeze(1).expand(-1, S, -1, -1), poses)
    return torch.stack([O.closed_form_inverse_se3(poses[b]) for b in range(B)])


def point_aligned_forward(sd: dict, images: Tensor, num_overlap: int, context: Optional[dict] = None,
                          enable_camera=True, enable_point=True, enable_depth=True, bf16: bool = False,
                          training: bool = False, agg_kwargs: Optional[dict] = None) -> dict:
    """pointAligned_wrapped_vggt.py:34-156 (aggregator under autocast, heads
    and alignment in fp32)."""
    B, S, _, H, W = images.shape
    pred = {}
    toks, psi = O.aggregator(sd, images, bf16=bf16, **(agg_kwargs or {}))
    T = sc = None
    if enable_point:
        pts, pconf = O.dpt_head(sd, "point_head.", toks, images, psi, "inv_log")
        if context is not None:
            cpm = context["world_points"][-1][:, -num_overlap:]
            cpc = context["world_points_conf"][-1][:, -num_overlap:]
            Ts, ss = [], []
            for b in range(B):
                r, t, s = irls_sim3_umeyama(pts[b, :num_overlap], cpm[b], pconf[b, :num_overlap], cpc[b])
                pose = F.pad(r, (0, 1, 0, 1))
                pose[:3, 3] = t
                pose[3, 3] = 1.0
                Ts.append(pose)
                ss.append(s)
            T = torch.stack(Ts)
            sc = torch.stack([s.reshape(()) for s in ss]).to(pts)
        else:
            T = torch.eye(4, dtype=images.dtype).view(1, 4, 4).expand(B, -1, -1)
            sc = torch.ones(B, dtype=pts.dtype)
        pts_f = apply_sim3_alignment_on_point_maps(pts, T, sc)
        if context is None:
            pred["world_points"], pred["world_points_conf"] = [pts_f], [pconf]
        else:
            context.setdefault("world_points", []).append(pts_f)
            pred["world_points"] = context["world_points"]
            context.setdefault("world_points_conf", []).append(pconf)
            pred["world_points_conf"] = context["world_points_conf"]
    if enable_camera:
        penc = O.camera_head(sd, toks)[-1]
        if enable_point:
            extr, intr = O.pose_encoding_to_extri_intri(penc, (H, W))
            aligned = apply_sim3_alignment_on_w2c(extr, T, sc)
            penc = O.extri_intri_to_pose_encoding(aligned, intr, (H, W))
        if context is None:
            pred["pose_enc"] = [penc]
        else:
            context.setdefault("pose_enc", []).append(penc)
            pred["pose_enc"] = context["pose_enc"]
    if enable_depth:
        depth, dconf = O.dpt_head(sd, "depth_head.", toks, images, psi, "exp")
        if enable_point:
            depth = depth * sc.view(B, 1, 1, 1, 1)
        if context is None:
            pred["depth"], pred["depth_conf"] = [depth], [dconf]
        else:
            context.setdefault("depth", []).append(depth)
            pred["depth"] = context["depth"]
            context.setdefault("depth_conf", []).append(dconf)
            pred["depth_conf"] = context["depth_conf"]
    if not training:
        if context is None:
            pred["images"] = [images]
        else:
            context.setdefault("images", []).append(images)
            pred["images"] = context["images"]
    return pred
