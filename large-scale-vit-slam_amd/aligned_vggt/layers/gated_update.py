"""Memory-token gated update (aligned_vggt/layers/gated_update.py:5-79), fp32.

The per-token delta MLPs (gated_update.py:22-31) run as two grouped HIP
skinny fp32 linears (all memory tokens in one launch each), the gate MLP
(:33-36) as two skinny linears, and the elementwise algebra around them
(:43-79: scale, concatenations, the sigmoid gate, the orthogonal step and the
normalisations) as three small HIP kernels (vggt_gated_update_*).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native as N
from .. import autograd as AG
from ..runtime import _pkey


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

    def _packed(self):
        """The per-token delta MLPs' weights stacked for the grouped linear:
        W1 [Nt, D, 3D], b1 [Nt, D], W2 [Nt, D, D], b2 [Nt, D] (fp32, cached per
        parameter version)."""
        ps = [p for mlp in self.delta_mlps for p in (mlp[0].weight, mlp[0].bias, mlp[2].weight, mlp[2].bias)]
        key = _pkey(*ps)
        c = self.__dict__.get("_mi355x_grouped")
        if c is None or c[0] != key:
            st = lambda i: torch.stack([ps[4 * t + i].detach().float() for t in range(self.num_tokens)]).contiguous()  # noqa: E731
            c = (key, st(0), st(1), st(2), st(3))
            self.__dict__["_mi355x_grouped"] = c
        return c[1:]

    @torch.no_grad()
    def forward(self, memory: torch.Tensor, update: torch.Tensor) -> torch.Tensor:
        """memory (B, N, D) unit-norm, update (B, 1, D) -> new memory (B, N, D).
        Seven launches: prep (scale, the delta MLPs' inputs, half the gate
        input), the Nt delta MLPs as two grouped linears, the gate input's
        diff half, the gate MLP, the tail (sigmoid gate, orthogonal step,
        normalisations)."""
        B, Nt, D = memory.shape
        assert Nt == self.num_tokens and D == self.token_dim
        dev = memory.device
        memory = memory.float().contiguous()
        update = update.float().contiguous()
        w1, b1, w2, b2 = self._packed()
        inp = torch.empty(B, Nt, 3 * D, device=dev)
        g_in = torch.empty(B * Nt, 2 * D, device=dev)
        N.gated_update_prep(memory, update, inp, g_in)
        hid = torch.empty(Nt, B, D, device=dev)
        N.linear_f32_grouped(inp.transpose(0, 1), w1, b1, hid, N.EPI_GELU_BF16)
        deltas = torch.empty(B, Nt, D, device=dev)
        N.linear_f32_grouped(hid, w2, b2, deltas.transpose(0, 1), N.EPI_F32)
        N.gated_update_diff(memory, deltas, g_in)
        gh = torch.empty(B * Nt, D, device=dev)
        N.linear_f32(g_in, self.gate_mlp[0].weight, self.gate_mlp[0].bias, gh, N.EPI_GELU_BF16)
        gl = torch.empty(B * Nt, 1, device=dev)
        N.linear_f32(gh, self.gate_mlp[2].weight, self.gate_mlp[2].bias, gl, N.EPI_F32)
        out = torch.empty(B, Nt, D, device=dev)
        N.gated_update_tail(memory, deltas, gl, out)
        return out

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
