"""1-D rotary position embedding (aligned_vggt/layers/rope.py:7-126).

Same frequency cache (fp32 angles, cat(angles, angles), rope.py:23-44) and
rotate-half application (rope.py:46-89); the rotation itself runs in the
HIP kernel vggt_headnorm_rope(_f32) -- usually fused with the QK-norm that
precedes it in CrossAttention (cross_attention.py:59-62).
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch
import torch.nn as nn

from .. import _native as N


class RotaryPositionEmbedding(nn.Module):
    def __init__(self, frequency: float = 100.0, scaling_factor: float = 1.0):
        super().__init__()
        self.base_frequency = frequency
        self.scaling_factor = scaling_factor
        self.frequency_cache: Dict[Tuple, Tuple[torch.Tensor, torch.Tensor]] = {}

    def _compute_frequency_components(self, dim: int, seq_len: int, device, dtype=torch.float32):
        """Host-side table (rope.py:23-44); returned as fp32 device tensors [seq_len, dim]."""
        key = (dim, seq_len, str(device))
        if key not in self.frequency_cache:
            exponents = torch.arange(0, dim, 2).float() / dim
            inv_freq = 1.0 / (self.base_frequency ** exponents)
            positions = torch.arange(seq_len, dtype=inv_freq.dtype)
            angles = torch.einsum("i,j->ij", positions, inv_freq)
            angles = torch.cat((angles, angles), dim=-1)
            self.frequency_cache[key] = (angles.cos().contiguous().to(device), angles.sin().contiguous().to(device))
        return self.frequency_cache[key]

    def tables(self, dim: int, max_pos: int, device):
        return self._compute_frequency_components(dim, max_pos + 1, device)

    @torch.no_grad()
    def forward(self, tokens: torch.Tensor, positions: torch.Tensor) -> torch.Tensor:
        """tokens (B, n_heads, N, D), positions (B, N) -> rotated copy (rope.py:91-126)."""
        assert tokens.size(-1) % 2 == 0, "Feature dimension must be even"
        B, H, Nn, D = tokens.shape
        cos, sin = self.tables(D, int(positions.max()), tokens.device)
        out = tokens.contiguous().clone().view(B * H * Nn, D)
        pos = positions.to(torch.int32)[:, None, :].expand(B, H, Nn).contiguous().view(-1)
        N.headnorm_rope_any(out, 0, 1, D, None, None, 0.0, N.ROPE_1D, pos, pos.numel(), cos, sin)
        return out.view(B, H, Nn, D)
