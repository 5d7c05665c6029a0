"""VGGT CameraHead (ext ``heads/camera_head.py``; called at
featureAligned_vggt.py:106 with autocast disabled) on the HIP fp32 tier.

camera tokens (B,S,2048) -> token_norm -> 4 refinement iterations of
[embed_pose 9->2048, SiLU+Linear adaLN modulation 2048->6144 (shift, scale,
gate), modulate(LN_noaffine(x)), 4 Blocks (dim 2048, 16 heads), trunk_norm,
pose_branch Mlp 2048->1024->9, activate_pose (T linear, quat linear, FoV relu)].
Linears: skinny exact-f32 MFMA kernel; attention: f32 small-window kernel.
"""
from __future__ import annotations

from typing import List

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native as N
from .layers import Block, Mlp


class CameraHead(nn.Module):
    def __init__(self, dim_in: int = 2048, trunk_depth: int = 4, pose_encoding_type: str = "absT_quaR_FoV",
                 num_heads: int = 16, mlp_ratio: int = 4, init_values: float = 0.01, trans_act: str = "linear",
                 quat_act: str = "linear", fl_act: str = "relu"):
        super().__init__()
        if pose_encoding_type != "absT_quaR_FoV":
            raise ValueError(f"Unsupported camera encoding type: {pose_encoding_type}")
        self.target_dim = 9
        self.trans_act, self.quat_act, self.fl_act = trans_act, quat_act, fl_act
        self.trunk_depth = trunk_depth
        self.trunk = nn.Sequential(*[Block(dim=dim_in, num_heads=num_heads, mlp_ratio=mlp_ratio,
                                           init_values=init_values) for _ in range(trunk_depth)])
        self.token_norm = nn.LayerNorm(dim_in)
        self.trunk_norm = nn.LayerNorm(dim_in)
        self.empty_pose_tokens = nn.Parameter(torch.zeros(1, 1, self.target_dim))
        self.embed_pose = nn.Linear(self.target_dim, dim_in)
        self.poseLN_modulation = nn.Sequential(nn.SiLU(), nn.Linear(dim_in, 3 * dim_in, bias=True))
        self.adaln_norm = nn.LayerNorm(dim_in, elementwise_affine=False, eps=1e-6)
        self.pose_branch = Mlp(in_features=dim_in, hidden_features=dim_in // 2, out_features=self.target_dim, drop=0)

    @staticmethod
    def _act(x: torch.Tensor, kind: str) -> torch.Tensor:
        if kind == "linear":
            return x
        if kind == "relu":
            return F.relu(x)
        if kind == "exp":
            return torch.exp(x)
        if kind == "inv_log":
            return torch.sign(x) * torch.expm1(torch.abs(x))
        raise ValueError(kind)

    @torch.no_grad()
    def forward(self, aggregated_tokens_list: List[torch.Tensor], num_iterations: int = 4) -> List[torch.Tensor]:
        tokens = aggregated_tokens_list[-1]
        if tokens.device.type != "cuda":
            raise RuntimeError("CameraHead: the MI355X hot path runs on HIP devices only (no CPU fallback)")
        B, S = tokens.shape[:2]
        C = tokens.shape[-1]
        dev = tokens.device
        M = B * S
        pt = tokens[:, :, 0].reshape(M, C).float().contiguous()
        N.layernorm(pt, self.token_norm.weight, self.token_norm.bias, self.token_norm.eps, pt)
        xn = torch.empty_like(pt)
        N.layernorm(pt, None, None, self.adaln_norm.eps, xn)
        pred = None
        outs = []
        inp = torch.empty(M, C, device=dev)
        mod = torch.empty(M, 3 * C, device=dev)
        delta = torch.empty(M, self.target_dim, device=dev)
        hid = torch.empty(M, self.pose_branch.fc1.out_features, device=dev)
        for _ in range(num_iterations):
            src = self.empty_pose_tokens.detach().expand(B, S, -1).reshape(M, -1).contiguous() if pred is None \
                else pred.reshape(M, -1).contiguous()
            N.linear_f32(src, self.embed_pose.weight, self.embed_pose.bias, inp)
            N.linear_f32(inp, self.poseLN_modulation[1].weight, self.poseLN_modulation[1].bias, mod, act_in=1)
            shift, scale, gate = mod[:, :C], mod[:, C:2 * C], mod[:, 2 * C:]
            x = gate * (xn * (1 + scale) + shift) + pt
            x = x.view(B, S, C)
            for blk in self.trunk:
                x = blk.forward_f32(x)
            xt = x.reshape(M, C)
            N.layernorm(xt, self.trunk_norm.weight, self.trunk_norm.bias, self.trunk_norm.eps, xt)
            N.linear_f32(xt, self.pose_branch.fc1.weight, self.pose_branch.fc1.bias, hid, N.EPI_GELU_BF16)
            N.linear_f32(hid, self.pose_branch.fc2.weight, self.pose_branch.fc2.bias, delta)
            d = delta.view(B, S, -1)
            pred = d.clone() if pred is None else pred + d
            outs.append(torch.cat([self._act(pred[..., :3], self.trans_act), self._act(pred[..., 3:7], self.quat_act),
                                   self._act(pred[..., 7:], self.fl_act)], dim=-1))
        return outs
