"""Transformer building blocks of the VGGT backbone, re-designed for the
MI355X HIP path.

Module/parameter names follow facebookresearch/vggt ``vggt/layers`` (ext,
unvendored, unpinned -- SURVEY.md §8c) so reference checkpoints load:
``norm1, attn.qkv, attn.q_norm, attn.k_norm, attn.proj, ls1.gamma, norm2,
mlp.fc1, mlp.fc2, ls2.gamma``.  The forward is NOT the reference's eager
op sequence: a Block runs as 8 fused HIP launches on a row-major fp32
residual stream (see :meth:`Block.forward_rows`), computing the bf16-mixed
autocast semantics of the reference (featureAligned_vggt.py:78 under
``precision="bf16-mixed"``, run_model.py:472).
"""
from __future__ import annotations

import os

from typing import Optional, Tuple

import torch
import torch.nn as nn

from .. import _native as N
from ..runtime import Workspace, pack_linear, yield_point


class LayerScale(nn.Module):
    def __init__(self, dim: int, init_values: float = 1e-5):
        super().__init__()
        self.gamma = nn.Parameter(init_values * torch.ones(dim))

    def forward(self, x):
        return x * self.gamma


class Mlp(nn.Module):
    """fc1 -> GELU(erf) -> fc2 (vggt layers/mlp.py, ext)."""

    def __init__(self, in_features: int, hidden_features: Optional[int] = None, out_features: Optional[int] = None,
                 act_layer=nn.GELU, drop: float = 0.0, bias: bool = True):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features, bias=bias)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, out_features, bias=bias)
        self.drop = nn.Dropout(drop)


class Attention(nn.Module):
    """Fused-qkv multi-head self-attention with optional per-head LayerNorm
    QK-norm and 2-D RoPE (vggt layers/attention.py, ext)."""

    def __init__(self, dim: int, num_heads: int = 8, qkv_bias: bool = True, proj_bias: bool = True,
                 attn_drop: float = 0.0, proj_drop: float = 0.0, norm_layer=nn.LayerNorm, qk_norm: bool = False,
                 fused_attn: bool = True, rope=None):
        super().__init__()
        assert dim % num_heads == 0
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.scale = self.head_dim ** -0.5
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.q_norm = norm_layer(self.head_dim) if qk_norm else nn.Identity()
        self.k_norm = norm_layer(self.head_dim) if qk_norm else nn.Identity()
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim, bias=proj_bias)
        self.proj_drop = nn.Dropout(proj_drop)
        self.rope = rope


# q/k norm + RoPE fused into the qkv GEMM epilogue (vggt_gemm_qkv); VGGT_FUSED_QKV=0
# selects the separate headnorm_rope launch (A/B and fallback for odd shapes).
_FUSED_QKV = os.environ.get("VGGT_FUSED_QKV", "1") != "0"
# head_dim 128 (the alignment head's frame blocks) has no persistent fused form: A/B switch
_FUSED_QKV128 = os.environ.get("VGGT_FUSED_QKV128", "1") != "0"
# VGGT_FUSED_ADD_LN bits: 1 = fc2 as a plain GEMM + one fused residual-add /
# next-LayerNorm row pass (vggt_resid_add_layernorm) instead of the GEMM's fp32
# read-modify-write epilogue + the next block's norm1; 2 = the same for proj
# (+ norm2).  Default 3 since round 2: with the persistent GEMM the plain fc2 is
# 146-150 vs 179-183 us (gemmbench: the RMW epilogue bursts on HBM after every
# round of tiles), and the aggregator step went 103.4 -> 101.8 ms (bit 1, 3 x 2
# same-box alternation, profiles/r4/ab_fused_add_ln.md), then 103.0 -> 102.5 ms
# with bit 2 as well.  Round 1 (r2c) measured the opposite with the 128x128 fc2
# form: 246.8 vs 235.2 us.  Only from _FUSED_ADD_LN_MIN_ROWS token rows: at the
# 154x518 sequence chunk (6,592 rows, fc2 = 140 tiles, less than one round) the
# sequence measured 1651 vs 1661 ms per 43 chunks (neutral to slightly worse),
# the 518^2 chunk 138.9 -> 137.8 ms and configs[2] 695 -> 689 ms (profiles/r4).
_FUSED_ADD_LN = int(os.environ.get("VGGT_FUSED_ADD_LN", "3"))
_FUSED_ADD_LN_MIN_ROWS = 16384


class RopeTables:
    """Device constants for one (rope, token layout): int32 positions
    [period, 2] and cos/sin tables [max_pos+1, D/2] computed exactly as the
    reference's frequency cache (rope.py:23-44: fp32 angles, cat(angles, angles))."""

    def __init__(self, pos: torch.Tensor, head_dim: int, freq: float, device, mode: int = N.ROPE_2D):
        self.mode = mode
        rd = head_dim // 2 if mode == N.ROPE_2D else head_dim
        maxp = int(pos.max()) + 1
        exponents = torch.arange(0, rd, 2).float() / rd
        inv_freq = 1.0 / (freq ** exponents)
        positions = torch.arange(maxp, dtype=inv_freq.dtype)
        angles = torch.einsum("i,j->ij", positions, inv_freq)
        angles = torch.cat((angles, angles), dim=-1)
        self.cos = angles.cos().contiguous().to(device)
        self.sin = angles.sin().contiguous().to(device)
        self.pos = pos.to(torch.int32).contiguous().to(device)
        self.period = pos.shape[0]


class Block(nn.Module):
    """Pre-LN transformer block with LayerScale (vggt layers/block.py, ext)."""

    def __init__(self, dim: int, num_heads: int, mlp_ratio: float = 4.0, qkv_bias: bool = True, proj_bias: bool = True,
                 ffn_bias: bool = True, drop: float = 0.0, attn_drop: float = 0.0, init_values=None,
                 drop_path: float = 0.0, act_layer=nn.GELU, norm_layer=nn.LayerNorm, attn_class=Attention,
                 ffn_layer=Mlp, qk_norm: bool = False, fused_attn: bool = True, rope=None):
        super().__init__()
        self.norm1 = norm_layer(dim)
        self.attn = attn_class(dim, num_heads=num_heads, qkv_bias=qkv_bias, proj_bias=proj_bias, attn_drop=attn_drop,
                               proj_drop=drop, qk_norm=qk_norm, fused_attn=fused_attn, rope=rope)
        self.ls1 = LayerScale(dim, init_values=init_values) if init_values else nn.Identity()
        self.norm2 = norm_layer(dim)
        self.mlp = ffn_layer(in_features=dim, hidden_features=int(dim * mlp_ratio), act_layer=act_layer, drop=drop,
                             bias=ffn_bias)
        self.ls2 = LayerScale(dim, init_values=init_values) if init_values else nn.Identity()

    def _gamma(self, ls: nn.Module, dim: int, device) -> torch.Tensor:
        if isinstance(ls, LayerScale):
            return ls.gamma.detach()
        c = self.__dict__.get("_mi355x_ones")
        if c is None or c.device != device or c.numel() != dim:
            c = torch.ones(dim, device=device)
            self.__dict__["_mi355x_ones"] = c
        return c

    @torch.no_grad()
    def forward_rows(self, x: torch.Tensor, M: int, groups: Tuple[int, int, int], rope: Optional[RopeTables],
                     ws: Workspace, out2: Optional[torch.Tensor] = None, tag: Optional[str] = None,
                     xn_ready: bool = False, next_norm: Optional[nn.LayerNorm] = None) -> bool:
        """In-place ``x[:M] = Block(x[:M])`` on the row-major fp32 residual
        stream x [>=M, C].  Attention is grouped as ``groups = (batch,
        rows_per_group, n)``: frame attention (B*S, P, P), global attention
        (B, S*P, S*P).  Optionally mirrors the block output into ``out2``
        (an fp32 [M, C] strided view, e.g. one half of a concat buffer).

        ``xn_ready``: the workspace's ``blk_xn`` already holds norm1(x) (the
        previous block fused it into its last residual add).  ``next_norm``:
        the LayerNorm the caller applies to x next (the following block's
        norm1); the fc2 residual add then also writes next_norm(x) into
        ``blk_xn`` in the same pass.  Returns True when it did."""
        C = x.shape[1]
        H = self.attn.num_heads
        D = C // H
        xs = x[:M]
        xn = ws.buf("blk_xn", M, C, torch.bfloat16)
        if not xn_ready:
            N.layernorm(xs, self.norm1.weight, self.norm1.bias, self.norm1.eps, xn)
        w, b = pack_linear(self.attn.qkv)
        qkv = ws.buf("blk_qkv", M, 3 * C, torch.bfloat16)
        yield_point(fine=True)
        qn = self.attn.q_norm if isinstance(self.attn.q_norm, nn.LayerNorm) else None
        kn = self.attn.k_norm if isinstance(self.attn.k_norm, nn.LayerNorm) else None
        mode = rope.mode if (rope is not None and self.attn.rope is not None) else N.ROPE_NONE
        fused = _FUSED_QKV and (qn is not None) == (kn is not None) and (qn is not None or mode != N.ROPE_NONE) \
            and (D == 64 or (D == 128 and _FUSED_QKV128)) and (qn is None or qn.eps == kn.eps)
        if fused:
            # qkv projection with q_norm / k_norm + RoPE in the GEMM epilogue
            rp = rope if mode != N.ROPE_NONE else None
            N.gemm_qkv(xn, w, b, qkv, H, D, qn.weight if qn is not None else None, qn.bias if qn is not None else None,
                       kn.weight if kn is not None else None, kn.bias if kn is not None else None,
                       qn.eps if qn is not None else 0.0, mode, rp.pos if rp else None, rp.period if rp else 1,
                       rp.cos if rp else None, rp.sin if rp else None)
        else:
            N.gemm_bf16(xn, w, b, qkv, N.EPI_BF16)
        if not fused and (qn is not None or mode != N.ROPE_NONE):
            rp = rope if mode != N.ROPE_NONE else None
            N.qknorm_rope(qkv, H, D, qn.weight if qn is not None else None, qn.bias if qn is not None else None,
                          kn.weight if kn is not None else None, kn.bias if kn is not None else None,
                          qn.eps if qn is not None else 0.0, mode, rp.pos if rp else None, rp.period if rp else 1,
                          rp.cos if rp else None, rp.sin if rp else None)
        ao = ws.buf("blk_ao", M, C, torch.bfloat16)
        nb, rows, n = groups
        yield_point()  # a gated encode (multi-GPU ring) pauses here while an alignment runs
        N.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], ao, nb, H, n, n, D, rows, rows, rows, tag=tag)
        w, b = pack_linear(self.attn.proj)
        fal = _FUSED_ADD_LN if M >= _FUSED_ADD_LN_MIN_ROWS else 0
        yield_point(fine=True)
        if (fal & 2) and C in (256, 512, 1024, 2048) and isinstance(self.norm2, nn.LayerNorm):
            # proj with a plain bf16 epilogue, then one row pass: x += ls1 * proj, xn = norm2(x)
            pj = ws.buf("blk_pj", M, C, torch.bfloat16)
            N.gemm_bf16(ao, w, b, pj, N.EPI_BF16)
            N.resid_add_layernorm(xs, pj, self._gamma(self.ls1, C, x.device), None, self.norm2.weight,
                                  self.norm2.bias, self.norm2.eps, xn)
        else:
            N.gemm_bf16(ao, w, b, xs, N.EPI_RESID_F32, gamma=self._gamma(self.ls1, C, x.device))
            N.layernorm(xs, self.norm2.weight, self.norm2.bias, self.norm2.eps, xn)
        w, b = pack_linear(self.mlp.fc1)
        hid = ws.buf("blk_h", M, w.shape[0], torch.bfloat16)
        yield_point()
        N.gemm_bf16(xn, w, b, hid, N.EPI_GELU_BF16)
        w, b = pack_linear(self.mlp.fc2)
        yield_point(fine=True)
        # the row pass has kernels for C / 256 in {1, 2, 4, 8} only (norm.hip)
        if not ((fal & 1) and C in (256, 512, 1024, 2048)):
            N.gemm_bf16(hid, w, b, xs, N.EPI_RESID_F32, gamma=self._gamma(self.ls2, C, x.device), out2=out2)
            return False
        # fc2 with a plain bf16 epilogue, then ONE row pass for the LayerScale
        # residual add, the kept-layer mirror and the next block's norm1 (same
        # arithmetic as the EPI_RESID_F32 epilogue).
        N.gemm_bf16(hid, w, b, ao, N.EPI_BF16)
        ln = next_norm if isinstance(next_norm, nn.LayerNorm) else None
        N.resid_add_layernorm(xs, ao, self._gamma(self.ls2, C, x.device), out2,
                              ln.weight if ln is not None else None, ln.bias if ln is not None else None,
                              ln.eps if ln is not None else 0.0, xn if ln is not None else None)
        return ln is not None

    @torch.no_grad()
    def forward_f32(self, x: torch.Tensor) -> torch.Tensor:
        """fp32 tier (autocast disabled, e.g. the camera-head trunk,
        featureAligned_vggt.py:104-106): x (B, N, C) -> new x; plain
        self-attention over the N tokens of each batch row (no QK-norm/RoPE
        unless configured)."""
        B, Nn, C = x.shape
        H = self.attn.num_heads
        D = C // H
        dev = x.device
        xs = x.reshape(B * Nn, C).float().contiguous().clone()
        xn = torch.empty_like(xs)
        N.layernorm(xs, self.norm1.weight, self.norm1.bias, self.norm1.eps, xn)
        qkv = torch.empty(B * Nn, 3 * C, device=dev)
        N.linear_f32(xn, self.attn.qkv.weight, self.attn.qkv.bias, qkv)
        for off, nm in ((0, self.attn.q_norm), (C, self.attn.k_norm)):
            if isinstance(nm, nn.LayerNorm):
                N.headnorm_rope_any(qkv, off, H, D, nm.weight, nm.bias, nm.eps)
        ao = torch.empty(B * Nn, C, device=dev)
        N.attention_small(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], ao, B, H, Nn, Nn, D, Nn, Nn, Nn)
        N.linear_f32(ao, self.attn.proj.weight, self.attn.proj.bias, xs, N.EPI_RESID_F32,
                     gamma=self._gamma(self.ls1, C, dev))
        N.layernorm(xs, self.norm2.weight, self.norm2.bias, self.norm2.eps, xn)
        hid = torch.empty(B * Nn, self.mlp.fc1.out_features, device=dev)
        N.linear_f32(xn, self.mlp.fc1.weight, self.mlp.fc1.bias, hid, N.EPI_GELU_BF16)
        N.linear_f32(hid, self.mlp.fc2.weight, self.mlp.fc2.bias, xs, N.EPI_RESID_F32,
                     gamma=self._gamma(self.ls2, C, dev))
        return xs.view(B, Nn, C)
