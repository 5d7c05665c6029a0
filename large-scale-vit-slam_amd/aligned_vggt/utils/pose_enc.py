"""absT_quaR_FoV pose encoding <-> extrinsics/intrinsics (VGGT
``utils/pose_enc.py``, ext).  9-d encoding = [T(3), quat xyzw(4), FoV_h, FoV_w]."""
from __future__ import annotations

import torch

from .rotation import mat_to_quat, quat_to_mat


def extri_intri_to_pose_encoding(extrinsics, intrinsics, image_size_hw=None, pose_encoding_type="absT_quaR_FoV"):
    if pose_encoding_type != "absT_quaR_FoV":
        raise NotImplementedError(pose_encoding_type)
    R = extrinsics[:, :, :3, :3]
    T = extrinsics[:, :, :3, 3]
    quat = mat_to_quat(R)
    H, W = image_size_hw
    fov_h = 2 * torch.atan((H / 2) / intrinsics[..., 1, 1])
    fov_w = 2 * torch.atan((W / 2) / intrinsics[..., 0, 0])
    return torch.cat([T, quat, fov_h[..., None], fov_w[..., None]], dim=-1).float()


def pose_encoding_to_extri_intri(pose_encoding, image_size_hw=None, pose_encoding_type="absT_quaR_FoV",
                                 build_intrinsics=True):
    if pose_encoding_type != "absT_quaR_FoV":
        raise NotImplementedError(pose_encoding_type)
    T = pose_encoding[..., :3]
    quat = pose_encoding[..., 3:7]
    fov_h = pose_encoding[..., 7]
    fov_w = pose_encoding[..., 8]
    R = quat_to_mat(quat)
    extrinsics = torch.cat([R, T[..., None]], dim=-1)
    intrinsics = None
    if build_intrinsics:
        H, W = image_size_hw
        fy = (H / 2.0) / torch.tan(fov_h / 2.0)
        fx = (W / 2.0) / torch.tan(fov_w / 2.0)
        intrinsics = torch.zeros(pose_encoding.shape[:2] + (3, 3), device=pose_encoding.device)
        intrinsics[..., 0, 0] = fx
        intrinsics[..., 1, 1] = fy
        intrinsics[..., 0, 2] = W / 2
        intrinsics[..., 1, 2] = H / 2
        intrinsics[..., 2, 2] = 1.0
    return extrinsics, intrinsics
