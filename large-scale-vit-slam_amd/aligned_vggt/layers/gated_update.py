"""Memory-token gated update (aligned_vggt/layers/gated_update.py:5-79), fp32.

The per-token delta MLPs (gated_update.py:22-31) and the gate MLP (:33-36) run
as HIP skinny fp32 linears; the per-token orthogonalise/normalise algebra
(:62-79, a few hundred floats) is device tensor glue.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native as N
from .. import autograd as AG


class GatedUpdate(nn.Module):
    def __init__(self, token_dim: int, num_tokens: int, init_gate: float = 0.5):
        super().__init__()
        self.token_dim = token_dim
        self.num_tokens = num_tokens
        self.delta_mlps = nn.ModuleList([
            nn.Sequential(nn.Linear(token_dim * 3, token_dim), nn.GELU(), nn.Linear(token_dim, token_dim))
            for _ in range(num_tokens)])
        self.gate_mlp = nn.Sequential(nn.Linear(token_dim * 2, token_dim), nn.GELU(), nn.Linear(token_dim, 1))
        bias_val = math.log(init_gate / (1 - init_gate))
        nn.init.constant_(self.gate_mlp[-1].bias, bias_val)
        nn.init.normal_(self.gate_mlp[-1].weight, mean=0.0, std=0.1)

    @torch.no_grad()
    def forward(self, memory: torch.Tensor, update: torch.Tensor) -> torch.Tensor:
        """memory (B, N, D) unit-norm, update (B, 1, D) -> new memory (B, N, D)."""
        B, Nt, D = memory.shape
        assert Nt == self.num_tokens and D == self.token_dim
        memory = memory.float().contiguous()
        scale = update.norm(dim=-1, keepdim=True)
        upd = update.expand_as(memory)
        mean_scaled = memory.mean(dim=1, keepdim=True).expand_as(memory) * scale
        mem_scaled = memory * scale
        inp = torch.cat([upd, mem_scaled, mean_scaled], dim=-1).contiguous()  # (B, N, 3D)
        hid = torch.empty(B, D, device=memory.device)
        deltas = torch.empty(B, Nt, D, device=memory.device)
        for i, mlp in enumerate(self.delta_mlps):
            N.linear_f32(inp[:, i], mlp[0].weight, mlp[0].bias, hid, N.EPI_GELU_BF16)
            N.linear_f32(hid, mlp[2].weight, mlp[2].bias, deltas[:, i], N.EPI_F32)
        diff = deltas - memory
        g_in = torch.cat([diff, mem_scaled], dim=-1).reshape(B * Nt, 2 * D).contiguous()
        gh = torch.empty(B * Nt, D, device=memory.device)
        N.linear_f32(g_in, self.gate_mlp[0].weight, self.gate_mlp[0].bias, gh, N.EPI_GELU_BF16)
        gl = torch.empty(B * Nt, 1, device=memory.device)
        N.linear_f32(gh, self.gate_mlp[2].weight, self.gate_mlp[2].bias, gl, N.EPI_F32)
        gate = torch.sigmoid(gl).view(B, Nt, 1)
        orth = diff - (diff * memory).sum(-1, keepdim=True) * memory
        d = F.normalize(orth, dim=-1)
        return F.normalize(memory + gate * d, dim=-1)

    def forward_train(self, memory: torch.Tensor, update: torch.Tensor) -> torch.Tensor:
        """gated_update.py:43-79 on fp32 HIP autograd linears (training; the
        gate input is detached as in the reference, :69)."""
        B, Nt, D = memory.shape
        assert Nt == self.num_tokens and D == self.token_dim
        memory = memory.float()
        scale = update.norm(dim=-1, keepdim=True)
        upd = update.expand_as(memory)
        mean_scaled = memory.mean(dim=1, keepdim=True).expand_as(memory) * scale
        mem_scaled = memory * scale
        inp = torch.cat([upd, mem_scaled, mean_scaled], dim=-1)
        deltas = torch.stack([AG.linear_f32(mlp[2], AG.linear_f32(mlp[0], inp[:, i], gelu=True))
                              for i, mlp in enumerate(self.delta_mlps)], dim=1)
        diff = deltas - memory
        g_in = torch.cat([diff, mem_scaled], dim=-1).detach()
        gate = torch.sigmoid(AG.linear_f32(self.gate_mlp[2], AG.linear_f32(self.gate_mlp[0], g_in, gelu=True)))
        orth = diff - (diff * memory).sum(-1, keepdim=True) * memory
        d = F.normalize(orth, dim=-1)
        return F.normalize(memory + gate * d, dim=-1)
