"""Sim(3) / scale alignment utilities (aligned_vggt/utils/alignment.py).

Two kinds of callers:
  * the point-aligned model (pointAligned_wrapped_vggt.py) applies Sim(3)
    transforms to dense point maps / poses every chunk -- the dense part runs
    in the HIP kernel ``vggt_sim3_points`` (device tensors only);
  * GT-based evaluation post-processing (``alignAndConvertOutputs``,
    data.py:108-153): closed-form Umeyama / Horn and the L1/LSE scale
    alignments -- host-side numpy/torch exactly as the reference (small,
    once per sequence), pinned by tests/golden/{alignment_utils,
    scale_alignment}.npz.
"""
from __future__ import annotations

import numpy as np
import torch

from .geometry import closed_form_inverse_se3
from .pose_enc import extri_intri_to_pose_encoding, pose_encoding_to_extri_intri


def umeyama(x: np.ndarray, y: np.ndarray) -> tuple:
    """alignment.py:6-59: Sim(m) least squares x -> y (3xn each); returns r, t, c."""
    if x.shape != y.shape:
        raise AssertionError("x shape not equal to y shape")
    m, n = x.shape
    mean_x = x.mean(axis=1)
    mean_y = y.mean(axis=1)
    sigma_x = 1.0 / n * (np.linalg.norm(x - mean_x[:, None]) ** 2)
    cov_xy = (y - mean_y[:, None]) @ (x - mean_x[:, None]).T / n
    u, d, v = np.linalg.svd(cov_xy)
    s = np.eye(m)
    if np.linalg.det(u) * np.linalg.det(v) < 0.0:
        s[m - 1, m - 1] = -1
    r = u.dot(s).dot(v)
    c = 1 / sigma_x * np.trace(np.diag(d).dot(s))
    t = mean_y - c * r.dot(mean_x)
    return r, t, c


def methodOfHorn(model: np.ndarray, data: np.ndarray, align_scale: bool = True) -> tuple:
    """alignment.py:61-111 (Horn closed form, evaluate_ate_scale convention)."""
    if model.shape != data.shape:
        raise AssertionError("model shape not equal to data shape")
    mz = model - model.mean(1, keepdims=True)
    dz = data - data.mean(1, keepdims=True)
    Wm = mz @ dz.T
    U, d, Vh = np.linalg.svd(Wm.T)
    S = np.identity(3)
    if np.linalg.det(U) * np.linalg.det(Vh) < 0:
        S[2, 2] = -1
    rot = U @ S @ Vh
    if align_scale:
        rotmodel = rot @ mz
        s = float((dz * rotmodel).sum() / (mz ** 2).sum())
    else:
        s = 1.0
    trans = data.mean(1) - s * rot @ model.mean(1)
    return rot, trans, np.asarray(s)


def scale_lse_solver(x: np.ndarray, y: np.ndarray) -> float:
    """alignment.py:113-129."""
    if x.shape != y.shape:
        raise AssertionError("x shape not equal to y shape")
    return np.abs(np.sum(x * y) / np.sum(x ** 2))


def per_frame_scale_alignment_from_poses(predictions: dict, batch: dict) -> None:
    """alignment.py:131-165 (note: ``alignment_scales`` keeps the last batch
    element's per-frame list, as the reference does)."""
    B, S = batch["extrinsics"].shape[:2]
    gt_positions = batch["extrinsics"][..., :3, 3].detach().cpu().numpy()
    pred_positions = predictions["pose_enc"][..., :3].detach().cpu().numpy()
    frame_scales = []
    for b in range(B):
        frame_scales = []
        for s in range(S):
            frame_scale = 1.0 if s == 0 else scale_lse_solver(pred_positions[b, s], gt_positions[b, s])
            predictions["pose_enc"][b, s, :3] *= frame_scale
            frame_scales.append(frame_scale)
            if "depth" in predictions:
                predictions["depth"][b, s] *= frame_scale
            if "world_points" in predictions:
                predictions["world_points"][b, s] *= frame_scale
    predictions["alignment_scales"] = frame_scales


def per_chunk_scale_alignment_from_poses(predictions: dict, batch: dict) -> None:
    """alignment.py:167-204 (chunked lists)."""
    C = len(batch["extrinsics"])
    B = batch["extrinsics"][0].shape[0]
    chunk_scales = []
    for c in range(C):
        gt = batch["extrinsics"][c][..., :3, 3].detach().cpu().numpy()
        pred = predictions["pose_enc"][c][..., :3].detach().cpu().numpy()
        scales = []
        for b in range(B):
            sc = scale_lse_solver(pred[b], gt[b])
            predictions["pose_enc"][c][b, :, :3] *= sc
            scales.append(sc)
            if b == B - 1:
                chunk_scales.append(torch.tensor(scales))
            if "depth" in predictions:
                predictions["depth"][c][b, ...] *= sc
            if "world_points" in predictions:
                predictions["world_points"][c][b, ...] *= sc
    predictions["alignment_scales_per_chunk"] = chunk_scales


def scale_alignment_from_poses(predictions: dict, batch: dict, seq_width: int = -1) -> None:
    """alignment.py:206-242."""
    B = batch["extrinsics"].shape[0]
    if seq_width == -1:
        seq_width = batch["extrinsics"].shape[1]
    gt = batch["extrinsics"][:, :seq_width, :3, 3].detach().cpu().numpy()
    pred = predictions["pose_enc"][:, :seq_width, :3].detach().cpu().numpy()
    scales = []
    for b in range(B):
        sc = scale_lse_solver(pred[b], gt[b])
        predictions["pose_enc"][b, :, :3] *= sc
        scales.append(sc)
        if "depth" in predictions:
            predictions["depth"][b, ...] *= sc
        if "world_points" in predictions:
            predictions["world_points"][b, ...] *= sc
    predictions["alignment_scales"] = scales


@torch.no_grad()
def scale_align_from_depths(predictions: dict, batch: dict) -> None:
    """alignment.py:244-323: per-batch weighted-median (L1-optimal) depth scale."""
    d_pred, conf, d_gt, mask = predictions["depth"], predictions["depth_conf"], batch["depths"], batch["point_masks"]
    B, S, H, W, _ = d_pred.shape
    N = S * H * W
    x = d_pred.reshape(B, N).float()
    y = d_gt.reshape(B, N).float()
    m = mask.reshape(B, N).float()
    w_conf = conf.reshape(B, N).float()
    sum_valid = m.sum(dim=-1, keepdim=True).clamp_min(1.0)
    mean_depth = (y * m).sum(dim=-1, keepdim=True) / sum_valid
    y_clamped = torch.max(y, 0.1 * mean_depth)
    w = m * w_conf * (1.0 / y_clamped.clamp_min(1e-6))
    sign = torch.sign(x)
    sign = torch.where(sign == 0, torch.ones_like(sign), sign)
    x_pos, y_pos = x * sign, y * sign
    r = y_pos / x_pos.clamp_min(1e-6)
    w_eff = w * x_pos
    r_sorted, idx = torch.sort(r, dim=-1)
    cumsum = torch.gather(w_eff, -1, idx).cumsum(-1)
    idx_med = torch.searchsorted(cumsum, 0.5 * cumsum[:, -1:], side="left").clamp(max=N - 1)
    scales = torch.gather(r_sorted, -1, idx_med).squeeze(-1)
    scales[scales <= 0] *= -1
    predictions["depth"] *= scales[:, None, None, None, None]
    if "world_points" in predictions:
        predictions["world_points"] *= scales[:, None, None, None, None]
    if "pose_enc" in predictions:
        predictions["pose_enc"][..., :3] *= scales[:, None, None]
    predictions["alignment_scales"] = [scales[b].item() for b in range(B)]


def apply_sim3_alignment_on_point_maps(point_maps: torch.Tensor, alignment_transforms: torch.Tensor,
                                       alignment_scales: torch.Tensor) -> torch.Tensor:
    """alignment.py:491-526 -> (B,S,H,W,3): T[:3,:3] (s p) + T[:3,3].  Device
    tensors go through the HIP kernel; host tensors (evaluation on offloaded
    outputs) through the same arithmetic in torch."""
    if point_maps.dim() == 4:
        point_maps, alignment_transforms, alignment_scales = (point_maps[None], alignment_transforms[None],
                                                              alignment_scales.reshape(1))
    assert point_maps.shape[0] == alignment_transforms.shape[0] == alignment_scales.shape[0], \
        "Inputs must have matching batch dimension"
    B = point_maps.shape[0]
    T = alignment_transforms.float()
    sc = torch.as_tensor(alignment_scales, dtype=torch.float32, device=point_maps.device).reshape(B)
    if point_maps.is_cuda:
        from .. import _native
        return _native.sim3_points(point_maps.float().contiguous(), T, sc)
    p = point_maps.float() * sc.view(B, 1, 1, 1, 1)
    out = p.reshape(B, -1, 3) @ T[:, :3, :3].transpose(-1, -2) + T[:, None, :3, 3]
    return out.view(point_maps.shape)


def apply_sim3_alignment_on_c2w(poses: torch.Tensor, alignment_transform: torch.Tensor,
                                alignment_scales: torch.Tensor) -> torch.Tensor:
    """alignment.py:558-594 (scale the translation -- in place on a 4x4 input,
    as the reference -- then left-multiply T)."""
    if poses.dim() == 3:
        poses, alignment_transform, alignment_scales = poses[None], alignment_transform[None], \
            torch.as_tensor(alignment_scales).reshape(1)
    B, S = poses.shape[:2]
    if poses.shape[-2] != 4:
        poses = torch.nn.functional.pad(poses, (0, 0, 0, 1, 0, 0), mode="constant")
        poses[:, 3, 3] = 1.0  # (sic) reference indexing, alignment.py:585
    sc = torch.as_tensor(alignment_scales, dtype=poses.dtype, device=poses.device).view(B, 1, 1)
    poses[:, :, :3, 3] = poses[:, :, :3, 3] * sc
    return torch.matmul(alignment_transform.to(poses).unsqueeze(1).expand(-1, S, -1, -1), poses)


def apply_sim3_alignment_on_w2c(extr: torch.Tensor, alignment_transform: torch.Tensor,
                                alignment_scales: torch.Tensor) -> torch.Tensor:
    """alignment.py:528-556: w2c -> c2w -> Sim(3) -> w2c (B,S,4,4)."""
    if extr.dim() == 3:
        extr, alignment_transform, alignment_scales = extr[None], alignment_transform[None], \
            torch.as_tensor(alignment_scales).reshape(1)
    B, S = extr.shape[:2]
    poses = closed_form_inverse_se3(extr.reshape(B * S, *extr.shape[-2:])).reshape(B, S, 4, 4)
    poses = apply_sim3_alignment_on_c2w(poses, alignment_transform, alignment_scales)
    return closed_form_inverse_se3(poses.reshape(B * S, 4, 4)).reshape(B, S, 4, 4)


def apply_sim3_alignment(alignment_transforms, alignment_scales, pose_encodings, images_size, points=None,
                         depths=None) -> tuple:
    """alignment.py:449-489."""
    B = alignment_transforms.shape[0]
    dev = pose_encodings.device
    sc = torch.as_tensor(np.asarray(alignment_scales), dtype=torch.float32, device=dev)
    T = torch.as_tensor(np.asarray(alignment_transforms), dtype=torch.float32, device=dev)
    extr, intr = pose_encoding_to_extri_intri(pose_encodings, images_size)
    extr = apply_sim3_alignment_on_w2c(extr, T, sc)
    pose_encodings = extri_intri_to_pose_encoding(extr, intr, images_size)
    if points is not None:
        points = apply_sim3_alignment_on_point_maps(points, T, sc)
    if depths is not None:
        depths *= sc.view(B, 1, 1, 1, 1)
    return pose_encodings, points, depths


def apply_sim3_alignment_on_dict(pred: dict, images_size: tuple, alignment_poses, alignment_scales) -> None:
    """alignment.py:428-447."""
    pe, pts, d = apply_sim3_alignment(alignment_poses, alignment_scales, pred["pose_enc"], images_size,
                                      pred.get("world_points"), pred.get("depth"))
    pred["pose_enc"] = pe
    if "world_points" in pred:
        pred["world_points"] = pts
    if "depth" in pred:
        pred["depth"] = d


def umeyama_alignment_from_poses(predictions: dict, batch: dict, seq_width: int) -> None:
    """alignment.py:325-370: Sim(3) of predicted to GT camera centres."""
    B = batch["extrinsics"].shape[0]
    gt_poses = closed_form_inverse_se3(batch["extrinsics"][:, :seq_width].reshape(B * seq_width, 3, 4)).reshape(
        B, seq_width, 4, 4).detach().cpu().numpy()
    gt_positions = gt_poses[..., :3, 3]
    pred_extr, _ = pose_encoding_to_extri_intri(predictions["pose_enc"][:, :seq_width], batch["images"].shape[-2:])
    pred_positions = closed_form_inverse_se3(pred_extr.reshape(B * seq_width, 3, 4)).reshape(
        B, seq_width, 4, 4)[..., :3, 3].detach().cpu().numpy()
    transforms, scales = [], []
    for b in range(B):
        r, t, c = umeyama(pred_positions[b].transpose(), gt_positions[b].transpose())
        pose = np.pad(r, ((0, 1), (0, 1)), mode="constant")
        pose[:3, 3] = t
        pose[3, 3] = 1.0
        transforms.append(pose)
        scales.append(c)
    pe, pts, d = apply_sim3_alignment(np.array(transforms), np.array(scales), predictions["pose_enc"],
                                      batch["images"].shape[-2:], predictions.get("world_points"),
                                      predictions.get("depth"))
    predictions["pose_enc"] = pe
    if "world_points" in predictions:
        predictions["world_points"] = pts
    if "depth" in predictions:
        predictions["depth"] = d


def umeyama_alignment_from_points(pred_points, pred_confidence, target_points, target_point_mask,
                                  confidence_threshold: int) -> tuple:
    """alignment.py:372-426 (percentile-thresholded Umeyama on point maps)."""
    def np_(a):
        return a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else a
    pred_points, target_points = np_(pred_points), np_(target_points)
    pred_confidence, target_point_mask = np_(pred_confidence), np_(target_point_mask)
    poses, cs = [], []
    for b in range(pred_points.shape[0]):
        thr = np.percentile(pred_confidence[b], confidence_threshold)
        m = (target_point_mask[b] > 0) & (pred_confidence[b] >= thr) & (pred_confidence[b] > 1e-5)
        r, t, c = umeyama(pred_points[b][m].reshape(3, -1), target_points[b][m].reshape(3, -1))
        pose = np.pad(r, ((0, 1), (0, 1)), mode="constant")
        pose[:3, 3] = t
        pose[3, 3] = 1.0
        poses.append(pose)
        cs.append(c)
    return np.array(poses), np.array(cs)
