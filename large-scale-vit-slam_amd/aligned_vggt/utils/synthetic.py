"""Deterministic random-init weights and synthetic inputs (BASELINE.json
configs use random-init weights and synthetic frames; no checkpoint or dataset
is available offline -- SURVEY.md §8d).

Every parameter draws from its own CPU ``torch.Generator`` seeded by
``crc32(name) ^ seed``, so a module tree gets identical weights on any device,
in any construction order and in every process (parameters with a specific
reference init -- tiny-std tokens, the orthonormal memory tokens, the gate
weight -- are redrawn from their reference distribution; constant inits are
kept).
"""
from __future__ import annotations

import zlib

import torch
import torch.nn as nn

# parameters whose constructor init is the reference's distribution, redrawn
# from the per-name generator with that same distribution (the constructors
# draw from torch's global generator, whose seed differs per process)
_REF_NORMAL = {"camera_token": 1e-6, "register_token": 1e-6, "register_tokens": 1e-6, "cls_token": 1e-6,
               "per_frame_alignment_token": 1e-6, "gate_mlp.2.weight": 0.1}
# constant constructor inits, kept as is
_KEEP = ("gamma", "mask_token", "alpha", "empty_pose_tokens", "gate_mlp.2.bias")


@torch.no_grad()
def synthetic_init_(model: nn.Module, seed: int = 0, std: float = 0.02) -> nn.Module:
    for name, p in model.named_parameters():
        if any(k in name for k in _KEEP):
            continue
        g = torch.Generator().manual_seed((zlib.crc32(name.encode()) ^ seed) & 0x7FFFFFFF)
        leaf = name.split(".")[-1]
        ref_std = _REF_NORMAL.get(leaf, _REF_NORMAL.get(".".join(name.split(".")[-3:])))
        if ref_std is not None:
            p.copy_((ref_std * torch.randn(p.shape, generator=g)).to(p.device, p.dtype))
            continue
        if leaf == "memory_token":
            # alignment_head.py:211-214: orthonormal rows, then L2-normalised
            m = torch.empty(p.shape[1:], dtype=torch.float32)
            nn.init.orthogonal_(m, generator=g)
            p.copy_(torch.nn.functional.normalize(m, dim=-1).view(p.shape).to(p.device, p.dtype))
            continue
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
def condition_pose_outputs_(model: nn.Module, translation: float = 0.0) -> nn.Module:
    """Put the random-init pose decoders in a well-conditioned regime.

    With N(0, 0.02) weights the camera head / alignment decoders emit
    quaternions of norm ~1e-2, whose direction (all the reference uses:
    quaternions are normalised before use, data.py:45, rotation.quat_to_mat)
    is then ill-conditioned.  Trained models emit near-unit quaternions; we
    emulate that by biasing the last decoder layers towards the identity
    rotation and a ~1 rad field of view.  ``translation`` (per refinement
    iteration, along the optical axis) does the same for the camera
    translation, which otherwise sits near zero, where its relative error is
    ill-conditioned; 0 keeps the earlier fixtures' init.
    Only biases change."""
    cam = getattr(model, "camera_head", None)
    if cam is not None:
        b = cam.pose_branch.fc2.bias
        b.zero_()
        b[2] = translation  # T_z: 4 x translation after the 4 refinement iterations
        b[6] = 0.25  # quat w, accumulated over 4 refinement iterations
        b[7:9] = 0.25  # FoV (h, w) -> ~1 rad after 4 iterations
    ah = getattr(model, "alignment_head", None)
    if ah is not None:
        for dec in (ah.chunk_sim3_decoder, ah.frame_se3_decoder):
            b = dec.fc2.bias
            b.zero_()
            b[6] = 1.0
    return model
