"""Chunking and pose-encoding glue (aligned_vggt/utils/data.py:12-225)."""
from __future__ import annotations

import random
from typing import Optional, List

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


def _to_host(t: torch.Tensor, pending: Optional[list]) -> torch.Tensor:
    if pending is None or t.device.type != "cuda":
        return t.cpu()
    # pinned destination, copied on a side stream after everything queued so far:
    # the next chunk's kernels do not wait for the PCIe transfer
    dst = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    cur = torch.cuda.current_stream(t.device)
    side = _side_stream(t.device)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        dst.copy_(t, non_blocking=True)
    t.record_stream(side)  # the allocator keeps t's memory until the copy is done
    ev = torch.cuda.Event()
    ev.record(side)
    pending.append(ev)
    return dst


_SIDE = {}


def _side_stream(device) -> "torch.cuda.Stream":
    s = _SIDE.get(device)
    if s is None:
        s = _SIDE[device] = torch.cuda.Stream(device)
    return s


def moveDictListItemToCPU(chunked_dict: dict, itemIndex: int, pending: Optional[list] = None) -> None:
    """data.py:89-106.  ``pending`` (a list): the copies run asynchronously into
    pinned host tensors and their completion events are appended -- the caller
    must wait on them (``wait_host_copies``) before reading the host tensors."""
    for key in chunked_dict.keys():
        v = chunked_dict[key]
        if isinstance(v, list) and len(v) >= (abs(itemIndex) if itemIndex < 0 else itemIndex + 1):
            if isinstance(v[0], list):
                v[itemIndex] = [(_to_host(it, pending) if isinstance(it, torch.Tensor) else it) for it in v[itemIndex]]
            elif isinstance(v[itemIndex], torch.Tensor):
                v[itemIndex] = _to_host(v[itemIndex], pending)


def wait_host_copies(pending: list) -> None:
    for ev in pending:
        ev.synchronize()
    pending.clear()


def alignAndConvertOutputs(predictions: dict, batch: dict, chunked_batch: dict, alignment_type: str, seq_width: int,
                           overlap: int) -> None:
    """data.py:108-153: optional GT-based alignment of the merged sequence
    outputs (evaluation post-processing; aligned_vggt/utils/alignment.py),
    with the per-chunk lists converted to overlap-free tensors in place."""
    from . import alignment as A
    if alignment_type == "per_chunk_scale_from_poses":
        A.per_chunk_scale_alignment_from_poses(predictions, chunked_batch)
        convertDictListsToTensors(chunked_batch, overlap, batch)
        convertDictListsToTensors(predictions, overlap)
        return
    convertDictListsToTensors(chunked_batch, overlap, batch)
    convertDictListsToTensors(predictions, overlap)
    if alignment_type == "scale_from_fc_poses":
        A.scale_alignment_from_poses(predictions, batch, seq_width)
    elif alignment_type == "scale_from_poses":
        A.scale_alignment_from_poses(predictions, batch)
    elif alignment_type == "per_frame_scale_from_poses":
        A.per_frame_scale_alignment_from_poses(predictions, batch)
    elif alignment_type == "scale_from_depths":
        if "depth" not in predictions:
            raise ValueError("scale_from_depths alignment requires depth head to be enabled.")
        A.scale_align_from_depths(predictions, batch)
    elif alignment_type == "sim3_from_poses":
        A.umeyama_alignment_from_poses(predictions, batch, seq_width)
    elif alignment_type == "sim3_from_points":
        if "world_points" not in predictions:
            raise ValueError("sim3_from_points alignment requires point head to be enabled.")
        T, sc = A.umeyama_alignment_from_points(predictions["world_points"][:, :seq_width],
                                                predictions["world_points_conf"][:, :seq_width],
                                                batch["world_points"][:, :seq_width],
                                                batch["point_masks"][:, :seq_width], confidence_threshold=50.0)
        A.apply_sim3_alignment_on_dict(predictions, batch["images"].shape[-2:], T, sc)


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
