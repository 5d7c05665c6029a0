"""Point-aligned VGGT (aligned_vggt/models/pointAligned_wrapped_vggt.py:14-305)
on MI355X -- BASELINE config 1's model family.

Same constructor / ``set_config`` / ``forward(images, num_overlap, context,
gt_poses)`` and module names (``aggregator``, ``camera_head``, ``point_head``,
``depth_head``, ``track_head``) as the reference.  Per chunk: HIP aggregator,
HIP point / depth / camera heads; consecutive chunks are aligned by a robust
Sim(3) fit between this chunk's first ``num_overlap`` point maps and the
previous chunk's last ones -- ``irls_sim3_umeyama`` runs as the HIP kernel
sequence ``vggt_irls_sim3`` for all batch elements at once, on the stream,
without the reference's per-batch host round trips; the dense Sim(3) of the
point maps is ``vggt_sim3_points`` and the depth scaling ``vggt_scale_f32``.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native as N
from ..backbone.aggregator import Aggregator
from ..backbone.camera_head import CameraHead
from ..backbone.dpt_head import DPTHead
from ..backbone.track_head import TrackHead
from ..utils.alignment import apply_sim3_alignment_on_w2c
from ..utils.pose_enc import extri_intri_to_pose_encoding, pose_encoding_to_extri_intri

try:
    from huggingface_hub import PyTorchModelHubMixin
except Exception:  # pragma: no cover
    class PyTorchModelHubMixin:  # type: ignore
        pass


class VGGT(nn.Module, PyTorchModelHubMixin):
    def __init__(self, img_size=518, patch_size=14, embed_dim=1024, enable_camera=True, enable_point=True,
                 enable_depth=True, enable_track=True):
        super().__init__()
        self.intermediate_layer_indices = [4, 11, 17, 23]
        n = len(self.intermediate_layer_indices)
        self.aggregator = Aggregator(img_size=img_size, patch_size=patch_size, embed_dim=embed_dim)
        self.camera_head = CameraHead(dim_in=2 * embed_dim) if enable_camera else None
        self.point_head = DPTHead(dim_in=2 * embed_dim, output_dim=4, activation="inv_log", conf_activation="expp1",
                                  intermediate_layer_idx=range(n)) if enable_point else None
        self.depth_head = DPTHead(dim_in=2 * embed_dim, output_dim=2, activation="exp", conf_activation="expp1",
                                  intermediate_layer_idx=range(n)) if enable_depth else None
        self.track_head = TrackHead(dim_in=2 * embed_dim, patch_size=patch_size) if enable_track else None

    def set_config(self, cfg):
        """pointAligned_wrapped_vggt.py:28-32."""
        self.camera_head = self.camera_head if cfg.enable_camera else None
        self.point_head = self.point_head if cfg.enable_point else None
        self.depth_head = self.depth_head if cfg.enable_depth else None
        self.track_head = self.track_head if cfg.enable_track else None

    @torch.no_grad()
    def forward(self, images: torch.Tensor, num_overlap: int, context: dict = None,
                gt_poses: torch.Tensor = None) -> dict:
        """pointAligned_wrapped_vggt.py:34-156 (``gt_poses`` is accepted and
        unused, as in the reference)."""
        B, S, C, H, W = images.shape
        pred = {}
        toks, psi = self.aggregator(images, keep_layers=self.intermediate_layer_indices)
        T = scales = None
        if self.point_head is not None:
            pts, pconf = self.point_head(toks, images=images, patch_start_idx=psi)
            if context is not None:
                cpm = context["world_points"][-1][:, -num_overlap:]
                cpc = context["world_points_conf"][-1][:, -num_overlap:]
                if cpm.device != pts.device:
                    raise RuntimeError("context world_points[-1] must stay on the chunk's device")
                R, t, s = N.irls_sim3(pts[:, :num_overlap].contiguous(), cpm.contiguous(),
                                      pconf[:, :num_overlap].contiguous(), cpc.contiguous())
                T = F.pad(R, (0, 1, 0, 1))
                T[:, :3, 3] = t
                T[:, 3, 3] = 1.0
                scales = s
            else:
                T = torch.eye(4, device=images.device, dtype=images.dtype).view(1, 4, 4).expand(B, -1, -1)
                scales = torch.ones(B, device=pts.device, dtype=pts.dtype)
            pts_f = N.sim3_points(pts, T, scales)
            if context is None:
                pred["world_points"], pred["world_points_conf"] = [pts_f], [pconf]
            else:
                context.setdefault("world_points", []).append(pts_f)
                pred["world_points"] = context["world_points"]
                context.setdefault("world_points_conf", []).append(pconf)
                pred["world_points_conf"] = context["world_points_conf"]

        if self.camera_head is not None:
            pose_enc = self.camera_head(toks)[-1]
            if self.point_head is not None:
                extr, intr = pose_encoding_to_extri_intri(pose_enc, image_size_hw=images.shape[-2:])
                aligned = apply_sim3_alignment_on_w2c(extr, T, scales)
                pose_enc = extri_intri_to_pose_encoding(aligned, intr, image_size_hw=images.shape[-2:])
            # (the reference leaves the encoding undefined without a point head,
            # pointAligned :117-128; the unaligned camera-head output is used here)
            if context is None:
                pred["pose_enc"] = [pose_enc]
            else:
                context.setdefault("pose_enc", []).append(pose_enc)
                pred["pose_enc"] = context["pose_enc"]

        if self.depth_head is not None:
            depth, dconf = self.depth_head(toks, images=images, patch_start_idx=psi)
            if self.point_head is not None:
                N.scale_(depth, scales)
            if context is None:
                pred["depth"], pred["depth_conf"] = [depth], [dconf]
            else:
                context.setdefault("depth", []).append(depth)
                pred["depth"] = context["depth"]
                context.setdefault("depth_conf", []).append(dconf)
                pred["depth_conf"] = context["depth_conf"]

        if not self.training:
            if context is None:
                pred["images"] = [images]
            else:
                context.setdefault("images", []).append(images)
                pred["images"] = context["images"]
        return pred


def weighted_umeyama_sim3(src: torch.Tensor, dst: torch.Tensor,
                          weights: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """pointAligned_wrapped_vggt.py:159-219 on the GPU (one solve of the
    ``vggt_irls_sim3`` sequence with the weights given directly).  NaN outputs
    where the reference raises ValueError (total weight < 1e-6)."""
    assert src.ndim == 2 and src.shape[1] == 3 and dst.shape == src.shape
    R, t, s = N.irls_sim3(src[None].contiguous(), dst[None].contiguous(), weights.reshape(1, -1).float().contiguous(),
                          None, conf_threshold_factor=0.0, max_iters=0)
    return R[0], t[0], s[0]


def irls_sim3_umeyama(src: torch.Tensor, dst: torch.Tensor, conf_src: Optional[torch.Tensor],
                      conf_dst: Optional[torch.Tensor], conf_threshold_factor: float = 0.5, delta: float = 0.1,
                      max_iters: int = 20, tol: float = 1e-9) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """pointAligned_wrapped_vggt.py:221-305 on the GPU: src/dst (N,H,W,3),
    confidences (N,H,W) -> R (3,3), t (3,), s ()."""
    assert src.shape[0] == dst.shape[0]
    R, t, s = N.irls_sim3(src.reshape(1, -1, 3).contiguous(), dst.reshape(1, -1, 3).contiguous(),
                          conf_src.reshape(1, -1).contiguous(), conf_dst.reshape(1, -1).contiguous(),
                          conf_threshold_factor, delta, max_iters, tol)
    return R[0], t[0], s[0]
