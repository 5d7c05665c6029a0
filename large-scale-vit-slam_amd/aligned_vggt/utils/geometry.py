"""Pose/geometry helpers: aligned_vggt/utils/geometry.py (averagePoseEncodings
:4-37, unproject :39-75, projection :77-105, relative poses :107-140, pixel
grid :142-157) plus VGGT's closed_form_inverse_se3 (ext)."""
from __future__ import annotations

import numpy as np
import torch


def closed_form_inverse_se3(se3, R=None, T=None):
    if se3.shape[-2:] != (4, 4) and se3.shape[-2:] != (3, 4):
        raise ValueError(f"se3 must be of shape (N,4,4), got {se3.shape}.")
    if R is None:
        R = se3[:, :3, :3]
    if T is None:
        T = se3[:, :3, 3:]
    if isinstance(se3, np.ndarray):
        Rt = np.transpose(R, (0, 2, 1))
        inv = np.tile(np.eye(4), (len(R), 1, 1))
        inv[:, :3, :3] = Rt
        inv[:, :3, 3:] = -np.matmul(Rt, T)
        return inv
    Rt = R.transpose(1, 2)
    inv = torch.eye(4, 4, device=R.device, dtype=R.dtype)[None].repeat(len(R), 1, 1)
    inv[:, :3, :3] = Rt
    inv[:, :3, 3:] = -torch.bmm(Rt, T)
    return inv


def averagePoseEncodings(pose_encodings: torch.Tensor) -> torch.Tensor:
    """Markley quaternion mean + translation mean (geometry.py:4-37)."""
    B, Nn, _ = pose_encodings.shape
    avg_t = pose_encodings[..., :3].mean(dim=1, keepdim=True)
    q = pose_encodings[..., 3:7]
    q = q / q.norm(dim=-1, keepdim=True).clamp(min=1e-8)
    w = (torch.ones(B, Nn, device=q.device, dtype=q.dtype) / Nn).unsqueeze(-1).unsqueeze(-1)
    M = (w * (q.unsqueeze(-1) * q.unsqueeze(-2))).sum(dim=1)
    # the (B, 4, 4) eigenproblem on the host: LAPACK, as the CPU oracle; the device
    # solver's launches, workspace fills and host round trips left the GPU idle
    # ~13 ms per chunk (profiles/r3h gap analysis); one tiny sync instead
    _, vec = torch.linalg.eigh(M.cpu())
    v = vec[..., -1].to(M.device)
    v = v / v.norm(dim=-1, keepdim=True)
    return torch.cat([avg_t, v.unsqueeze(1)], dim=-1).float()


def generate_3D_pixel_grid(H: int, W: int, device) -> torch.Tensor:
    u, v = torch.meshgrid(torch.arange(W, device=device), torch.arange(H, device=device), indexing="xy")
    return torch.stack((u, v, torch.ones_like(u)), dim=-1).float()


def unproject_depth_map_to_point_map(depth_map, extrinsics, intrinsics):
    B, S, H, W, _ = depth_map.shape
    pix = generate_3D_pixel_grid(H, W, depth_map.device).view(-1, 3)
    rays = (torch.inverse(intrinsics) @ pix.t()[None, None]).permute(0, 1, 3, 2).contiguous()
    cam = rays * depth_map.view(B, S, -1, 1)
    cam_h = torch.cat([cam, torch.ones_like(cam[..., :1])], dim=-1)
    poses = closed_form_inverse_se3(extrinsics.reshape(B * S, 3, 4)).reshape(B, S, 4, 4)
    world = (poses @ cam_h.transpose(-1, -2)).transpose(-1, -2)
    return (world[..., :3] / world[..., 3:]).view(B, S, H, W, 3)


def compute_relative_poses(extrinsics, offset: int = 1, toNext: bool = True):
    B, S, _, _ = extrinsics.shape
    if S <= offset:
        raise Exception("To small sequence for offset")
    w2c = torch.eye(4, device=extrinsics.device).unsqueeze(0).unsqueeze(0).repeat(B, S, 1, 1)
    w2c[:, :, :3, :4] = extrinsics
    c2w = torch.inverse(w2c)
    rel = w2c[:, offset:] @ c2w[:, :-offset] if toNext else w2c[:, :-offset] @ c2w[:, offset:]
    return rel[:, :, :3, :4]
