"""Cross attention (aligned_vggt/layers/cross_attention.py:15-200) on the
MI355X HIP path.

Same module tree (q, k, v, q_norm, k_norm, proj; norm1, norm2, norm3, ls1,
ls2, mlp) and semantics: q from x, k/v from y, per-head LayerNorm QK-norm,
1-D RoPE, softmax attention (the all-True boolean mask of
cross_attention.py:66-67 is a no-op), pre-LN block with LayerScale
(cross_attention.py:126-131).  Two execution tiers:

* ``forward_rows_bf16`` -- the temporal blocks of the alignment head, which
  run under the reference's bf16-mixed autocast: bf16 MFMA GEMMs (k and v
  fused into one GEMM), bf16 small-window attention;
* ``forward_rows_f32`` -- the decoder blocks (alignment_head.py:340 disables
  autocast): exact-f32 skinny linears + f32 attention.
"""
from __future__ import annotations

import os
from typing import Callable, Optional

import torch
import torch.nn as nn

from .. import _native as N
from ..backbone.layers import Attention, LayerScale, Mlp
from ..runtime import Workspace, _pkey, pack_linear
from .. import autograd as AG

# the temporal blocks' q_norm / k_norm + RoPE in the q and kv GEMM epilogues
# (vggt_gemm_headnorm); VGGT_FUSED_HEADNORM=0: the GEMMs, then vggt_headnorm_rope
_FUSED_HEADNORM = os.environ.get("VGGT_FUSED_HEADNORM", "1") != "0"


class CrossAttention(nn.Module):
    def __init__(self, dim: int, num_heads: int = 8, qkv_bias: bool = True, proj_bias: bool = True,
                 attn_drop: float = 0.0, proj_drop: float = 0.0, norm_layer=nn.LayerNorm, qk_norm: bool = False,
                 fused_attn: bool = True, rope=None):
        super().__init__()
        assert dim % num_heads == 0, "dim should be divisible by num_heads"
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.scale = self.head_dim ** -0.5
        self.fused_attn = fused_attn
        self.q = nn.Linear(dim, dim, bias=qkv_bias)
        self.k = nn.Linear(dim, dim, bias=qkv_bias)
        self.v = nn.Linear(dim, dim, bias=qkv_bias)
        self.q_norm = norm_layer(self.head_dim) if qk_norm else nn.Identity()
        self.k_norm = norm_layer(self.head_dim) if qk_norm else nn.Identity()
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim, bias=proj_bias)
        self.proj_drop = nn.Dropout(proj_drop)
        self.rope = rope

    def packed_kv(self):
        """bf16 [Wk; Wv] (2C x C) and rounded [bk; bv] -- one GEMM for k and v."""
        wk, bk = pack_linear(self.k)
        wv, bv = pack_linear(self.v)
        key = (self.k.__dict__["_mi355x_pack"][0], self.v.__dict__["_mi355x_pack"][0])  # parameter versions
        c = self.__dict__.get("_mi355x_kv")
        if c is None or c[0] != key:
            c = (key, torch.cat([wk, wv], 0).contiguous(), torch.cat([bk, bv], 0).contiguous())
            self.__dict__["_mi355x_kv"] = c
        return c[1], c[2]

    def f32_kv(self):
        key = _pkey(self.k.weight, self.k.bias, self.v.weight, self.v.bias)
        c = self.__dict__.get("_mi355x_kv32")
        if c is None or c[0] != key:
            c = (key, torch.cat([self.k.weight, self.v.weight], 0).detach().float().contiguous(),
                 torch.cat([self.k.bias, self.v.bias], 0).detach().float().contiguous())
            self.__dict__["_mi355x_kv32"] = c
        return c[1], c[2]


class CrossAttentionBlock(nn.Module):
    def __init__(self, dim: int, num_heads: int, mlp_ratio: float = 4.0, qkv_bias: bool = True,
                 proj_bias: bool = True, ffn_bias: bool = True, drop: float = 0.0, attn_drop: float = 0.0,
                 init_values=None, act_layer: Callable[..., nn.Module] = nn.GELU,
                 norm_layer: Callable[..., nn.Module] = nn.LayerNorm, ffn_layer: Callable[..., nn.Module] = Mlp,
                 qk_norm: bool = False, fused_attn: bool = True, rope=None):
        super().__init__()
        self.norm1 = norm_layer(dim)
        self.attn = CrossAttention(dim, num_heads=num_heads, qkv_bias=qkv_bias, proj_bias=proj_bias,
                                   attn_drop=attn_drop, proj_drop=drop, qk_norm=qk_norm, fused_attn=fused_attn,
                                   rope=rope)
        self.ls1 = LayerScale(dim, init_values=init_values) if init_values else nn.Identity()
        self.norm2 = norm_layer(dim)
        self.mlp = ffn_layer(in_features=dim, hidden_features=int(dim * mlp_ratio), act_layer=act_layer, drop=drop,
                             bias=ffn_bias)
        self.ls2 = LayerScale(dim, init_values=init_values) if init_values else nn.Identity()
        self.norm3 = norm_layer(dim)

    def _gamma(self, ls, dim, device):
        if isinstance(ls, LayerScale):
            return ls.gamma.detach()
        c = self.__dict__.get("_mi355x_ones")
        if c is None or c.device != device or c.numel() != dim:
            c = torch.ones(dim, device=device)
            self.__dict__["_mi355x_ones"] = c
        return c

    def _qk_norm(self, which):
        m = self.attn.q_norm if which == "q" else self.attn.k_norm
        if isinstance(m, nn.LayerNorm):
            return m.weight, m.bias, m.eps
        return None, None, 0.0

    @torch.no_grad()
    def forward_rows_bf16(self, x: torch.Tensor, Mx: int, y: Optional[torch.Tensor], My: int, groups: int, nq: int,
                          nk: int, rope_q, rope_k, ws: Workspace) -> None:
        """In place x[:Mx] = block(x, y) on fp32 row streams; x rows are
        ``groups`` runs of nq queries, y rows ``groups`` runs of nk keys
        (y is None: y = x).  rope_q/rope_k = (pos int32 [period], cos, sin)."""
        C = x.shape[1]
        H = self.attn.num_heads
        D = C // H
        xs = x[:Mx]
        xn = ws.buf("ca_xn", Mx, C, torch.bfloat16)
        N.layernorm(xs, self.norm1.weight, self.norm1.bias, self.norm1.eps, xn)
        ysrc = xs if y is None else y[:My]
        yn = ws.buf("ca_yn", My, C, torch.bfloat16)
        N.layernorm(ysrc, self.norm3.weight, self.norm3.bias, self.norm3.eps, yn)
        wq, bq = pack_linear(self.attn.q)
        q = ws.buf("ca_q", Mx, C, torch.bfloat16)
        wkv, bkv = self.attn.packed_kv()
        kv = ws.buf("ca_kv", My, 2 * C, torch.bfloat16)
        mode = N.ROPE_1D if self.attn.rope is not None else N.ROPE_NONE
        fused = _FUSED_HEADNORM and D in (64, 128) and C % 128 == 0 and xn.shape[1] % 32 == 0
        for a_, w_, b_, buf, which, rp in ((xn, wq, bq, q, "q", rope_q), (yn, wkv, bkv, kv, "k", rope_k)):
            w, b, eps = self._qk_norm(which)
            extra = w is not None or mode != N.ROPE_NONE
            if fused and extra:
                N.gemm_headnorm(a_, w_, b_, buf, H, D, w, b, eps, mode, rp[0] if mode else None,
                                rp[0].numel() if mode else 1, rp[1] if mode else None, rp[2] if mode else None)
                continue
            N.gemm_bf16(a_, w_, b_, buf, N.EPI_BF16)
            if extra:
                N.headnorm_rope(buf, 0, H, D, w, b, eps, mode, rp[0] if mode else None,
                                rp[0].numel() if mode else 1, rp[1] if mode else None, rp[2] if mode else None)
        ao = ws.buf("ca_ao", Mx, C, torch.bfloat16)
        N.attention_small(q, kv[:, :C], kv[:, C:], ao, groups, H, nq, nk, D, nq, nk, nq)
        wp, bp = pack_linear(self.attn.proj)
        N.gemm_bf16(ao, wp, bp, xs, N.EPI_RESID_F32, gamma=self._gamma(self.ls1, C, x.device))
        N.layernorm(xs, self.norm2.weight, self.norm2.bias, self.norm2.eps, xn)
        w1, b1 = pack_linear(self.mlp.fc1)
        hid = ws.buf("ca_h", Mx, w1.shape[0], torch.bfloat16)
        N.gemm_bf16(xn, w1, b1, hid, N.EPI_GELU_BF16)
        w2, b2 = pack_linear(self.mlp.fc2)
        N.gemm_bf16(hid, w2, b2, xs, N.EPI_RESID_F32, gamma=self._gamma(self.ls2, C, x.device))

    @torch.no_grad()
    def forward_f32(self, x: torch.Tensor, y: torch.Tensor, pos_q: torch.Tensor, pos_k: torch.Tensor,
                    rope_tabs) -> torch.Tensor:
        """fp32 tier: x (B, Nq, C), y (B, Nk, C) -> new x (B, Nq, C);
        pos_q (Nq,), pos_k (Nk,) int32 device tensors; rope_tabs = (cos, sin)."""
        B, Nq, C = x.shape
        Nk = y.shape[1]
        H = self.attn.num_heads
        D = C // H
        dev = x.device
        xs = x.reshape(B * Nq, C).float().contiguous().clone()
        ys = y.reshape(B * Nk, C).float().contiguous()
        xn = torch.empty_like(xs)
        N.layernorm(xs, self.norm1.weight, self.norm1.bias, self.norm1.eps, xn)
        yn = torch.empty_like(ys)
        N.layernorm(ys, self.norm3.weight, self.norm3.bias, self.norm3.eps, yn)
        q = torch.empty(B * Nq, C, device=dev)
        N.linear_f32(xn, self.attn.q.weight, self.attn.q.bias, q)
        wkv, bkv = self.attn.f32_kv()
        kv = torch.empty(B * Nk, 2 * C, device=dev)
        N.linear_f32(yn, wkv, bkv, kv)
        mode = N.ROPE_1D if self.attn.rope is not None else N.ROPE_NONE
        for buf, which, pos in ((q, "q", pos_q), (kv, "k", pos_k)):
            w, b, eps = self._qk_norm(which)
            if w is not None or mode != N.ROPE_NONE:
                N.headnorm_rope_any(buf, 0, H, D, w, b, eps, mode, pos if mode else None,
                                    pos.numel() if mode else 1, rope_tabs[0] if mode else None,
                                    rope_tabs[1] if mode else None)
        ao = torch.empty(B * Nq, C, device=dev)
        N.attention_small(q, kv[:, :C], kv[:, C:], ao, B, H, Nq, Nk, D, Nq, Nk, Nq)
        N.linear_f32(ao, self.attn.proj.weight, self.attn.proj.bias, xs, N.EPI_RESID_F32,
                     gamma=self._gamma(self.ls1, C, dev))
        N.layernorm(xs, self.norm2.weight, self.norm2.bias, self.norm2.eps, xn)
        hid = torch.empty(B * Nq, self.mlp.fc1.out_features, device=dev)
        N.linear_f32(xn, self.mlp.fc1.weight, self.mlp.fc1.bias, hid, N.EPI_GELU_BF16)
        N.linear_f32(hid, self.mlp.fc2.weight, self.mlp.fc2.bias, xs, N.EPI_RESID_F32,
                     gamma=self._gamma(self.ls2, C, dev))
        return xs.view(B, Nq, C)


    def forward_f32_train(self, x: torch.Tensor, y: torch.Tensor, pos_q: torch.Tensor, pos_k: torch.Tensor,
                          rope_tabs) -> torch.Tensor:
        """forward_f32 as fp32 HIP autograd Functions (decoder blocks under
        training, alignment_head.py:487-526): x (B, Nq, C), y (B, Nk, C)."""
        B, Nq, C = x.shape
        Nk = y.shape[1]
        H = self.attn.num_heads
        D = C // H
        a = self.attn
        xn = AG.layernorm_f32(self.norm1, x)
        yn = AG.layernorm_f32(self.norm3, y)
        q = AG.linear_f32(a.q, xn).reshape(B * Nq, C)
        k = AG.linear_f32(a.k, yn).reshape(B * Nk, C)
        v = AG.linear_f32(a.v, yn).reshape(B * Nk, C)
        mode = N.ROPE_1D if a.rope is not None else N.ROPE_NONE
        qn, kn = a.q_norm, a.k_norm
        if isinstance(qn, nn.LayerNorm) or mode != N.ROPE_NONE:
            hn = isinstance(qn, nn.LayerNorm)
            q = AG.HeadNormRopeF32Fn.apply(q, qn.weight if hn else None, qn.bias if hn else None,
                                           qn.eps if hn else 0.0, H, D, mode, pos_q, rope_tabs)
            k = AG.HeadNormRopeF32Fn.apply(k, kn.weight if hn else None, kn.bias if hn else None,
                                           kn.eps if hn else 0.0, H, D, mode, pos_k, rope_tabs)
        o = AG.AttnSmallF32Fn.apply(q, k, v, B, H, Nq, Nk, D)
        x = x + self.ls1.gamma * AG.linear_f32(a.proj, o).view(B, Nq, C)
        h = AG.linear_f32(self.mlp.fc1, AG.layernorm_f32(self.norm2, x), gelu=True)
        return x + self.ls2.gamma * AG.linear_f32(self.mlp.fc2, h)


class DecoderBlock(nn.Module):
    """Defined in the reference (cross_attention.py:134-200) but never
    instantiated; kept for state-dict/API parity.  Not on any hot path."""

    def __init__(self, dim: int, num_heads: int, mlp_ratio: float = 4.0, qkv_bias: bool = True,
                 proj_bias: bool = True, ffn_bias: bool = True, drop: float = 0.0, attn_drop: float = 0.0,
                 init_values=None, act_layer=nn.GELU, norm_layer=nn.LayerNorm, ffn_layer=Mlp, qk_norm: bool = False,
                 fused_attn: bool = True, rope=None):
        super().__init__()
        self.norm1 = norm_layer(dim)
        self.cross_attn = CrossAttention(dim, num_heads=num_heads, qkv_bias=qkv_bias, proj_bias=proj_bias,
                                         attn_drop=attn_drop, proj_drop=drop, qk_norm=qk_norm, fused_attn=fused_attn,
                                         rope=rope)
        self.attn = Attention(dim, num_heads=num_heads, qkv_bias=qkv_bias, proj_bias=proj_bias, attn_drop=attn_drop,
                              proj_drop=drop, qk_norm=qk_norm, fused_attn=fused_attn, rope=rope)
        self.ls1 = LayerScale(dim, init_values=init_values) if init_values else nn.Identity()
        self.norm2 = norm_layer(dim)
        self.norm3 = norm_layer(dim)
        self.mlp = ffn_layer(in_features=dim, hidden_features=int(dim * mlp_ratio), act_layer=act_layer, drop=drop,
                             bias=ffn_bias)
        self.ls2 = LayerScale(dim, init_values=init_values) if init_values else nn.Identity()
        self.norm_y = norm_layer(dim)

    def forward(self, *args, **kwargs):
        raise NotImplementedError("DecoderBlock is never instantiated by the reference (SURVEY.md §2)")
