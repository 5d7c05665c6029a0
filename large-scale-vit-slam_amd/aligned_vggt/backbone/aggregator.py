"""VGGT Aggregator (alternating frame/global attention over DINOv2-L/14-reg
patch tokens) on the MI355X HIP path.

Restated from facebookresearch/vggt ``models/aggregator.py`` and the DINOv2
``vision_transformer.py`` it embeds (ext, unpinned; assumptions in
SPEC_ASSUMPTIONS.md).  Called by FeatureAlignedVGGT.forward
(featureAligned_vggt.py:78) and the point-aligned VGGT (pointAligned_wrapped_vggt.py:60).

Execution: the whole chunk lives as one row-major fp32 residual stream
``x[B*S*P, 1024]`` in HBM; frame and global blocks differ only in how the
attention kernel groups rows (per frame vs per chunk), so no permutes or
copies happen between them.  Only the layers the callers keep
(featureAligned_vggt.py:24,79) are materialised, written by the fc2 GEMM
epilogue straight into their half of the (B,S,P,2C) concat buffer.
"""
from __future__ import annotations

import math
from functools import partial
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native as N
from ..runtime import Workspace, pack_linear, round_up, yield_point
from .layers import Block, RopeTables

_RESNET_MEAN = (0.485, 0.456, 0.406)
_RESNET_STD = (0.229, 0.224, 0.225)


class PatchEmbed(nn.Module):
    def __init__(self, img_size=518, patch_size=14, in_chans=3, embed_dim=1024):
        super().__init__()
        self.patch_size = (patch_size, patch_size)
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)
        self.norm = nn.Identity()


class DinoVisionTransformer(nn.Module):
    """DINOv2 ViT with register tokens (ext ``layers/vision_transformer.py``):
    parameter names cls_token, pos_embed, register_tokens, mask_token,
    patch_embed.proj, blocks.{i}, norm."""

    def __init__(self, img_size=518, patch_size=14, embed_dim=1024, depth=24, num_heads=16, mlp_ratio=4.0,
                 num_register_tokens=4, init_values=1.0, interpolate_antialias=True, interpolate_offset=0.0):
        super().__init__()
        self.patch_size = patch_size
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.num_register_tokens = num_register_tokens
        self.interpolate_antialias = interpolate_antialias
        self.interpolate_offset = interpolate_offset
        self.patch_embed = PatchEmbed(img_size, patch_size, 3, embed_dim)
        n = (img_size // patch_size) ** 2
        self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
        self.pos_embed = nn.Parameter(torch.zeros(1, n + 1, embed_dim))
        self.register_tokens = nn.Parameter(torch.zeros(1, num_register_tokens, embed_dim))
        self.mask_token = nn.Parameter(torch.zeros(1, embed_dim), requires_grad=False)
        blk = partial(Block, norm_layer=partial(nn.LayerNorm, eps=1e-6))
        self.blocks = nn.ModuleList([blk(dim=embed_dim, num_heads=num_heads, mlp_ratio=mlp_ratio, qkv_bias=True,
                                         proj_bias=True, ffn_bias=True, init_values=init_values) for _ in range(depth)])
        self.norm = nn.LayerNorm(embed_dim, eps=1e-6)
        self.head = nn.Identity()
        nn.init.trunc_normal_(self.pos_embed, std=0.02)
        nn.init.normal_(self.cls_token, std=1e-6)
        nn.init.normal_(self.register_tokens, std=1e-6)

    def pos_embed_for(self, h: int, w: int) -> torch.Tensor:
        """Positional table [1 + h*w, C] (DINOv2 interpolate_pos_encoding:
        bicubic, antialias, offset 0 -> explicit size; identity at the native
        square grid).  Weight preprocessing, cached per (h, w, version)."""
        pe = self.pos_embed
        key = (h, w, pe.data_ptr(), pe._version)
        c = self.__dict__.get("_mi355x_pe")
        if c is not None and c[0] == key:
            return c[1]
        n = pe.shape[1] - 1
        m = int(math.sqrt(n))
        with torch.no_grad():
            if h * w == n and h == w:
                out = pe[0].float().contiguous()
            else:
                grid = pe[0, 1:].float().reshape(1, m, m, -1).permute(0, 3, 1, 2)
                grid = F.interpolate(grid, size=(h, w), mode="bicubic", antialias=self.interpolate_antialias)
                out = torch.cat([pe[0, :1].float(), grid.permute(0, 2, 3, 1).reshape(h * w, -1)], 0).contiguous()
        self.__dict__["_mi355x_pe"] = (key, out)
        return out


def slice_expand_and_flatten(token_tensor: torch.Tensor, B: int, S: int) -> torch.Tensor:
    """(1,2,X,C) -> (B*S,X,C): frame 0 takes index 0, others index 1."""
    query = token_tensor[:, 0:1, ...].expand(B, 1, *token_tensor.shape[2:])
    others = token_tensor[:, 1:, ...].expand(B, S - 1, *token_tensor.shape[2:])
    return torch.cat([query, others], dim=1).reshape(B * S, *token_tensor.shape[2:])


class Aggregator(nn.Module):
    def __init__(self, img_size=518, patch_size=14, embed_dim=1024, depth=24, num_heads=16, mlp_ratio=4.0,
                 num_register_tokens=4, block_fn=Block, qkv_bias=True, proj_bias=True, ffn_bias=True,
                 patch_embed="dinov2_vitl14_reg", aa_order=("frame", "global"), aa_block_size=1, qk_norm=True,
                 rope_freq=100, init_values=0.01, dino_depth: int = 24):
        super().__init__()
        if patch_embed != "dinov2_vitl14_reg":
            raise NotImplementedError("only the dinov2_vitl14_reg patch embed used by every reference config")
        if list(aa_order) != ["frame", "global"] or aa_block_size != 1:
            raise NotImplementedError("aa_order ['frame','global'] with aa_block_size 1 (VGGT defaults)")
        self.patch_embed = DinoVisionTransformer(img_size, patch_size, embed_dim, dino_depth, num_heads, mlp_ratio,
                                                 num_register_tokens, init_values=1.0)
        self.rope_freq = rope_freq
        self.rope = True if rope_freq > 0 else None
        self.frame_blocks = nn.ModuleList([
            block_fn(dim=embed_dim, num_heads=num_heads, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, proj_bias=proj_bias,
                     ffn_bias=ffn_bias, init_values=init_values, qk_norm=qk_norm, rope=self.rope)
            for _ in range(depth)])
        self.global_blocks = nn.ModuleList([
            block_fn(dim=embed_dim, num_heads=num_heads, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, proj_bias=proj_bias,
                     ffn_bias=ffn_bias, init_values=init_values, qk_norm=qk_norm, rope=self.rope)
            for _ in range(depth)])
        self.depth = depth
        self.aa_order = list(aa_order)
        self.patch_size = patch_size
        self.aa_block_size = aa_block_size
        self.aa_block_num = depth // aa_block_size
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.camera_token = nn.Parameter(torch.randn(1, 2, 1, embed_dim))
        self.register_token = nn.Parameter(torch.randn(1, 2, num_register_tokens, embed_dim))
        self.patch_start_idx = 1 + num_register_tokens
        nn.init.normal_(self.camera_token, std=1e-6)
        nn.init.normal_(self.register_token, std=1e-6)
        self.register_buffer("_resnet_mean", torch.FloatTensor(_RESNET_MEAN).view(1, 1, 3, 1, 1), persistent=False)
        self.register_buffer("_resnet_std", torch.FloatTensor(_RESNET_STD).view(1, 1, 3, 1, 1), persistent=False)

    # -------------------------------------------------------------- helpers
    def _rope_tables(self, h: int, w: int, device) -> RopeTables:
        key = (h, w, device)
        c = self.__dict__.get("_mi355x_rope")
        if c is None or c[0] != key:
            yy, xx = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
            pos = torch.stack([yy.reshape(-1), xx.reshape(-1)], -1) + 1
            pos = torch.cat([torch.zeros(self.patch_start_idx, 2, dtype=pos.dtype), pos], 0)
            c = (key, RopeTables(pos, self.embed_dim // self.num_heads, float(self.rope_freq), device))
            self.__dict__["_mi355x_rope"] = c
        return c[1]

    def _special_tokens(self) -> torch.Tensor:
        return torch.cat([self.camera_token, self.register_token], dim=2)[0].detach().float().contiguous()

    @torch.no_grad()
    def forward(self, images: torch.Tensor, keep_layers: Optional[Sequence[int]] = None
                ) -> Tuple[List[torch.Tensor], int]:
        """images (B,S,3,H,W) in [0,1] -> (list of (B,S,P,2C) fp32, patch_start_idx).

        Returns all ``depth`` concat outputs like the reference unless
        ``keep_layers`` selects a subset (the callers keep [4, 11, 17, 23])."""
        B, S, C_in, H, W = images.shape
        if images.device.type != "cuda":
            raise RuntimeError("Aggregator: the MI355X hot path runs on HIP devices only (no CPU fallback)")
        keep = list(range(self.depth)) if keep_layers is None else list(keep_layers)
        ps = self.patch_size
        h, w = H // ps, W // ps
        hw = h * w
        F_ = B * S
        C = self.embed_dim
        dino = self.patch_embed
        nreg = dino.num_register_tokens
        P = 1 + nreg + hw  # == patch_start_idx + hw
        M = F_ * P
        ws = Workspace.get(images.device)

        # ---- DINOv2 patch embed: normalise + im2col -> bf16 GEMM -> assemble
        kk = 3 * ps * ps
        Kp = round_up(kk, 64)
        A = ws.buf("pe_a", F_ * hw, Kp, torch.bfloat16)
        N.patch_im2col(images.reshape(F_, C_in, H, W).float().contiguous(), ps, _RESNET_MEAN, _RESNET_STD, A)
        wpe, bpe = pack_linear(dino.patch_embed.proj, k_pad=Kp - kk)
        pe = ws.buf("pe_out", F_ * hw, C, torch.bfloat16)
        N.gemm_bf16(A, wpe, bpe, pe, N.EPI_BF16)
        x = ws.buf("dino_x", round_up(M, 256), C)
        N.dino_assemble(pe, dino.cls_token.detach().float().contiguous(),
                        dino.register_tokens.detach().float().contiguous(), dino.pos_embed_for(h, w), F_, hw, nreg, C,
                        x)
        ready = False
        for j, blk in enumerate(dino.blocks):
            yield_point()  # the multi-GPU pipeline's gated encode pauses here while an alignment runs
            nxt = dino.blocks[j + 1].norm1 if j + 1 < len(dino.blocks) else None
            ready = blk.forward_rows(x, M, (F_, P, P), None, ws, tag="dino_attn", xn_ready=ready, next_norm=nxt)

        # ---- aggregator tokens: final DINOv2 norm + camera/register tokens
        y = ws.buf("agg_x", round_up(M, 256), C)
        N.layernorm(x[:M], dino.norm.weight, dino.norm.bias, dino.norm.eps, y[:M])
        N.special_tokens(y, F_, S, P, self._special_tokens())
        rope = self._rope_tables(h, w, images.device) if self.rope is not None else None

        outs = {i: torch.empty(B, S, P, 2 * C, device=images.device, dtype=torch.float32) for i in keep}
        # each block's last residual add also writes the next block's norm1(y)
        ready = False
        for i in range(self.depth):
            yield_point()
            o = outs[i].view(M, 2 * C) if i in outs else None
            ready = self.frame_blocks[i].forward_rows(y, M, (F_, P, P), rope, ws,
                                                      out2=o[:, :C] if o is not None else None, tag="frame_attn",
                                                      xn_ready=ready, next_norm=self.global_blocks[i].norm1)
            nxt = self.frame_blocks[i + 1].norm1 if i + 1 < self.depth else None
            yield_point()
            ready = self.global_blocks[i].forward_rows(y, M, (B, S * P, S * P), rope, ws,
                                                       out2=o[:, C:] if o is not None else None, tag="global_attn",
                                                       xn_ready=ready, next_norm=nxt)
        return [outs[i] for i in keep], self.patch_start_idx
