"""Deterministic random-init weights and synthetic inputs (BASELINE.json
configs use random-init weights and synthetic frames; no checkpoint or dataset
is available offline -- SURVEY.md §8d).

Every parameter draws from its own CPU ``torch.Generator`` seeded by
``crc32(name) ^ seed``, so a module tree gets identical weights on any device
and in any construction order.
"""
from __future__ import annotations

import zlib

import torch
import torch.nn as nn

# parameters whose constructor init is the reference's and is kept as is
_KEEP = ("gamma", "camera_token", "register_token", "register_tokens", "cls_token", "mask_token",
         "per_frame_alignment_token", "memory_token", "alpha", "empty_pose_tokens", "gate_mlp.2.")


@torch.no_grad()
def synthetic_init_(model: nn.Module, seed: int = 0, std: float = 0.02) -> nn.Module:
    for name, p in model.named_parameters():
        if any(k in name for k in _KEEP):
            continue
        g = torch.Generator().manual_seed((zlib.crc32(name.encode()) ^ seed) & 0x7FFFFFFF)
        r = torch.randn(p.shape, generator=g, dtype=torch.float32)
        is_norm_w = p.dim() == 1 and name.endswith("weight") and "norm" in name.split(".")[-2]
        if is_norm_w:
            v = 1.0 + std * r
        else:
            v = std * r
        p.copy_(v.to(p.device, p.dtype))
    return model


def synthetic_images(B: int, S: int, H: int, W: int, seed: int = 1234, device="cpu") -> torch.Tensor:
    """Uniform [0, 1) frames (B,S,3,H,W), generator seed 1234."""
    g = torch.Generator().manual_seed(seed)
    return torch.rand(B, S, 3, H, W, generator=g).to(device)


@torch.no_grad()
def condition_pose_outputs_(model: nn.Module) -> nn.Module:
    """Put the random-init pose decoders in a well-conditioned regime.

    With N(0, 0.02) weights the camera head / alignment decoders emit
    quaternions of norm ~1e-2, whose direction (all the reference uses:
    quaternions are normalised before use, data.py:45, rotation.quat_to_mat)
    is then ill-conditioned.  Trained models emit near-unit quaternions; we
    emulate that by biasing the last decoder layers towards the identity
    rotation and a ~1 rad field of view.  Only biases change."""
    cam = getattr(model, "camera_head", None)
    if cam is not None:
        b = cam.pose_branch.fc2.bias
        b.zero_()
        b[6] = 0.25  # quat w, accumulated over 4 refinement iterations
        b[7:9] = 0.25  # FoV (h, w) -> ~1 rad after 4 iterations
    ah = getattr(model, "alignment_head", None)
    if ah is not None:
        for dec in (ah.chunk_sim3_decoder, ah.frame_se3_decoder):
            b = dec.fc2.bias
            b.zero_()
            b[6] = 1.0
    return model
