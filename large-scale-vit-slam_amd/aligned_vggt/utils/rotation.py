"""Quaternion <-> rotation matrix (VGGT ``utils/rotation.py``, ext;
scalar-last xyzw, w >= 0 after mat_to_quat).  Small per-frame host glue on
device tensors."""
from __future__ import annotations

import torch
import torch.nn.functional as F


def quat_to_mat(quaternions: torch.Tensor) -> torch.Tensor:
    i, j, k, r = torch.unbind(quaternions, -1)
    two_s = 2.0 / (quaternions * quaternions).sum(-1)
    o = torch.stack((1 - two_s * (j * j + k * k), two_s * (i * j - k * r), two_s * (i * k + j * r),
                     two_s * (i * j + k * r), 1 - two_s * (i * i + k * k), two_s * (j * k - i * r),
                     two_s * (i * k - j * r), two_s * (j * k + i * r), 1 - two_s * (i * i + j * j)), -1)
    return o.reshape(quaternions.shape[:-1] + (3, 3))


def _sqrt_positive_part(x: torch.Tensor) -> torch.Tensor:
    # sqrt(max(x, 0)) without the boolean-mask assignment (a mask index is a
    # nonzero() + device->host size read, i.e. a stream synchronisation)
    return torch.where(x > 0, torch.sqrt(x.clamp_min(0)), torch.zeros_like(x))


def mat_to_quat(matrix: torch.Tensor) -> torch.Tensor:
    """Same values as VGGT's mat_to_quat (best-conditioned candidate row,
    xyzw, w >= 0); the row is picked with gather instead of a one-hot mask
    index and the floor is a clamp, so no call synchronises the stream."""
    batch_dim = matrix.shape[:-2]
    m00, m01, m02, m10, m11, m12, m20, m21, m22 = torch.unbind(matrix.reshape(batch_dim + (9,)), dim=-1)
    q_abs = _sqrt_positive_part(torch.stack([1.0 + m00 + m11 + m22, 1.0 + m00 - m11 - m22, 1.0 - m00 + m11 - m22,
                                             1.0 - m00 - m11 + m22], dim=-1))
    cand = torch.stack([
        torch.stack([q_abs[..., 0] ** 2, m21 - m12, m02 - m20, m10 - m01], dim=-1),
        torch.stack([m21 - m12, q_abs[..., 1] ** 2, m10 + m01, m02 + m20], dim=-1),
        torch.stack([m02 - m20, m10 + m01, q_abs[..., 2] ** 2, m12 + m21], dim=-1),
        torch.stack([m10 - m01, m20 + m02, m21 + m12, q_abs[..., 3] ** 2], dim=-1)], dim=-2)
    cand = cand / (2.0 * q_abs[..., None].clamp_min(0.1))
    idx = q_abs.argmax(dim=-1)[..., None, None].expand(batch_dim + (1, 4))
    out = torch.gather(cand, -2, idx).squeeze(-2)
    out = torch.roll(out, -1, dims=-1)  # wxyz -> xyzw
    return torch.where(out[..., 3:4] < 0, -out, out)
