"""Chunking and pose-encoding glue (aligned_vggt/utils/data.py:12-225)."""
from __future__ import annotations

import random
from typing import List

import torch
import torch.nn.functional as F

from .rotation import mat_to_quat, quat_to_mat


def extri_to_pose_encoding(extrinsics: torch.Tensor) -> torch.Tensor:
    """data.py:12-30: (B,S,3|4,4) -> (B,S,7) [T, unit quat xyzw]."""
    quat = mat_to_quat(extrinsics[:, :, :3, :3])
    quat = quat / quat.norm(dim=-1, keepdim=True).clamp(min=1e-8)
    return torch.cat([extrinsics[:, :, :3, 3], quat], dim=-1).float()


def pose_encoding_to_extri(pose_encoding: torch.Tensor) -> torch.Tensor:
    """data.py:33-52: (B,S,7+) -> (B,S,4,4)."""
    T = pose_encoding[..., :3]
    quat = pose_encoding[..., 3:7]
    quat = quat / quat.norm(dim=-1, keepdim=True).clamp(min=1e-8)
    e = torch.cat([quat_to_mat(quat), T[..., None]], dim=-1)
    e = F.pad(e, (0, 0, 0, 1, 0, 0, 0, 0), mode="constant")
    e[:, :, 3, 3] = 1.0
    return e


def convertDictListsToTensors(chunked_dict: dict, overlap: int, out_dict: dict = None) -> None:
    """data.py:54-87: concatenate per-chunk lists along dim 1, dropping the
    `overlap` leading frames of every chunk but the first."""
    if out_dict is None:
        out_dict = chunked_dict
    keys = ["pose_enc", "pose_enc_list", "world_points", "world_points_conf", "depth", "depth_conf", "extrinsics",
            "intrinsics", "scales", "cam_points", "depths", "point_masks", "images", "ids"]
    for key in chunked_dict.keys():
        if key not in keys:
            continue
        if isinstance(chunked_dict[key][0], list):
            if overlap > 0:
                for i in range(1, len(chunked_dict[key])):
                    chunked_dict[key][i] = [item[:, overlap:] for item in chunked_dict[key][i]]
            out_dict[key] = [torch.cat(t, dim=1) for t in zip(*chunked_dict[key])]
        else:
            if overlap > 0:
                for i in range(1, len(chunked_dict[key])):
                    chunked_dict[key][i] = chunked_dict[key][i][:, overlap:]
            out_dict[key] = torch.cat(chunked_dict[key], dim=1)


def moveDictListItemToCPU(chunked_dict: dict, itemIndex: int) -> None:
    """data.py:89-106."""
    for key in chunked_dict.keys():
        v = chunked_dict[key]
        if isinstance(v, list) and len(v) >= (abs(itemIndex) if itemIndex < 0 else itemIndex + 1):
            if isinstance(v[0], list):
                v[itemIndex] = [(it.cpu() if isinstance(it, torch.Tensor) else it) for it in v[itemIndex]]
            elif isinstance(v[itemIndex], torch.Tensor):
                v[itemIndex] = v[itemIndex].cpu()


def generate_chunks(num_frames: int, mode: str, seq_width: int, overlap: int) -> List[List[int]]:
    """data.py:155-207."""
    indices = []
    if mode == "chunk_gt":
        for i in range(0, num_frames - seq_width + 1, seq_width):
            indices.append(list(range(i, i + seq_width)))
        if len(indices) * seq_width < num_frames:
            indices.append(list(range(len(indices) * seq_width, num_frames)))
    elif mode == "chunk_overlap":
        if num_frames < seq_width:
            indices.append(list(range(num_frames)))
        else:
            for i in range(0, num_frames - seq_width + 1, seq_width - overlap):
                indices.append(list(range(i, i + seq_width)))
            if len(indices) * (seq_width - overlap) < num_frames - overlap:
                indices.append(list(range(len(indices) * (seq_width - overlap), num_frames)))
    elif mode == "all":
        indices = [list(range(num_frames))]
    elif mode == "two_chunks":
        if num_frames < 2:
            raise ValueError("Number of frames must be at least 2 for two_chunks mode.")
        elif num_frames == 2:
            indices = [[0, 1]]
        else:
            all_idx = list(range(num_frames))
            first = random.sample(all_idx, random.randint(1, num_frames - 1))
            indices = [first, [i for i in all_idx if i not in first]]
    else:
        raise ValueError(f"Unknown sequence generation mode: {mode}")
    return indices


def chunk_batch(batch: dict, indices: list) -> dict:
    """data.py:209-225."""
    out = {}
    for ids in indices:
        for key in batch.keys():
            if isinstance(batch[key], torch.Tensor):
                out.setdefault(key, []).append(batch[key][:, ids])
    return out
