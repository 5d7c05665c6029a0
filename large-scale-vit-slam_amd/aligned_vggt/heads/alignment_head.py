"""AlignmentHead (aligned_vggt/heads/alignment_head.py:19-568) on the MI355X
HIP path: same constructor kwargs, forward signature, return tuple and
state-dict names.

Trunk (bf16-mixed tier, alignment_head.py:242-338):
  project_in (fp32 tokens -> bf16 cast -> bf16 MFMA GEMM) -> token_norm
  written straight behind the per-frame alignment token of every frame (row
  remapped LayerNorm) -> 4 x [frame Block (D=128, QK-norm, RoPE-2D) ;
  temporal CrossAttentionBlock].  The temporal block reproduces the
  reference's raw ``.view(B*P, S, C)`` of the (B,S,P,C) token tensor
  (alignment_head.py:372-380, Appendix A of SURVEY.md): queries are runs of S
  consecutive rows of the row-major token stream and keys runs of T rows of
  the overlap tokens -- exactly how this path lays them out in HBM, so no
  copies are needed.
Decoder (fp32 tier, alignment_head.py:427-540): skinny fp32 MFMA linears,
f32 small attention; memory hybrid init / GatedUpdate glue on device tensors.
"""
from __future__ import annotations

import logging
from typing import List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native as N
from ..backbone.layers import Block, Mlp, RopeTables
from ..layers.cross_attention import CrossAttentionBlock
from ..layers.gated_update import GatedUpdate
from ..layers.rope import RotaryPositionEmbedding
from ..runtime import Workspace, pack_linear, round_up
from .. import autograd as AG

logger = logging.getLogger(__name__)


class AlignmentHead(nn.Module):
    def __init__(self, patch_size=14, in_dim=2048, embed_dim=1024, dec_dim=512, depth_aa=4, depth_decoder=2,
                 num_heads=8, mlp_ratio=4.0, num_register_tokens=4, qkv_bias=True, proj_bias=True, ffn_bias=True,
                 aa_order=["frame", "temporal"], aa_block_size=1, qk_norm=True, rope_freq=100, init_values=0.01,
                 num_memory_tokens=8, temporal_attention=True):
        super().__init__()
        self.num_memory_tokens = num_memory_tokens
        self.temporal_attention = temporal_attention
        self.depth_aa = depth_aa
        self.aa_order = aa_order
        self.aa_block_size = aa_block_size
        self.patch_size = patch_size
        if self.depth_aa % self.aa_block_size != 0:
            raise ValueError(f"depth ({depth_aa}) must be divisible by aa_block_size ({aa_block_size})")
        self.aa_block_num = self.depth_aa // self.aa_block_size
        self.depth_decoder = depth_decoder
        self.patch_start_idx = 1 + 1 + num_register_tokens
        self.drop_prob_nonoverlap = 0.2
        self.use_reentrant = False
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.rope_freq = rope_freq
        self.project_in = nn.Linear(in_dim, embed_dim)
        self.project_dec = nn.Linear(embed_dim, dec_dim)
        self.rope1d = RotaryPositionEmbedding(frequency=rope_freq) if rope_freq > 0 else None
        self.rope2d = True if rope_freq > 0 else None
        self.frame_blocks = nn.ModuleList([
            Block(dim=embed_dim, num_heads=num_heads, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, proj_bias=proj_bias,
                  ffn_bias=ffn_bias, init_values=init_values, qk_norm=qk_norm, rope=self.rope2d)
            for _ in range(depth_aa)])
        if temporal_attention:
            self.temporal_blocks = nn.ModuleList([
                CrossAttentionBlock(dim=embed_dim, num_heads=num_heads, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias,
                                    proj_bias=proj_bias, ffn_bias=ffn_bias, init_values=init_values, qk_norm=qk_norm,
                                    rope=self.rope1d)
                for _ in range(depth_aa)])
        else:
            self.global_blocks = nn.ModuleList([
                Block(dim=embed_dim, num_heads=num_heads, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, proj_bias=proj_bias,
                      ffn_bias=ffn_bias, init_values=init_values, qk_norm=qk_norm, rope=self.rope2d)
                for _ in range(depth_aa)])
        self.chunk_cross_blocks = nn.ModuleList([
            CrossAttentionBlock(dim=dec_dim, num_heads=num_heads, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias,
                                proj_bias=proj_bias, ffn_bias=ffn_bias, init_values=init_values, qk_norm=qk_norm,
                                rope=self.rope1d)
            for _ in range(depth_decoder)])
        self.frame_cross_blocks = nn.ModuleList([
            CrossAttentionBlock(dim=dec_dim, num_heads=num_heads, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias,
                                proj_bias=proj_bias, ffn_bias=ffn_bias, init_values=init_values, qk_norm=qk_norm,
                                rope=self.rope1d)
            for _ in range(depth_decoder)])
        self.chunk_sim3_decoder = Mlp(in_features=dec_dim, hidden_features=dec_dim // 2, out_features=8, drop=0)
        self.frame_se3_decoder = Mlp(in_features=dec_dim, hidden_features=dec_dim // 2, out_features=7, drop=0)
        self.token_norm = nn.LayerNorm(embed_dim)
        self.dec_norm = nn.LayerNorm(dec_dim)
        self.chunk_norm = nn.LayerNorm(dec_dim)
        self.frame_norm = nn.LayerNorm(dec_dim)
        self.per_frame_alignment_token = nn.Parameter(torch.randn(1, 2, 1, embed_dim))
        nn.init.normal_(self.per_frame_alignment_token, std=1e-6)
        if self.num_memory_tokens > 0:
            self.memory_token = nn.Parameter(torch.empty(1, num_memory_tokens, dec_dim))
            nn.init.orthogonal_(self.memory_token[0])
            self.memory_token.data = F.normalize(self.memory_token.data, dim=-1)
            self.frame_proj = nn.Linear(dec_dim, num_memory_tokens * dec_dim)
            self.alpha = nn.Parameter(torch.tensor(0.1))
            self.gated_update = GatedUpdate(dec_dim, num_memory_tokens)

    # ------------------------------------------------------------------
    def _rope2d(self, h: int, w: int, device) -> RopeTables:
        """2-D RoPE tables per patch grid, kept for every grid seen: a HIP graph
        captured for one grid reads them on each replay, so they must outlive
        a switch to another grid (a one-entry cache freed them under it)."""
        cache = self.__dict__.setdefault("_mi355x_rope2d", {})
        key = (h, w, str(device))
        c = cache.get(key)
        if c is None:
            yy, xx = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
            pos = torch.stack([yy.reshape(-1), xx.reshape(-1)], -1) + 1
            pos = torch.cat([torch.zeros(self.patch_start_idx, 2, dtype=pos.dtype), pos], 0)
            c = cache[key] = RopeTables(pos, self.embed_dim // self.num_heads, float(self.rope_freq), device)
        return c

    def _i32(self, pos: torch.Tensor, device) -> torch.Tensor:
        """Device int32 copy of a small host position vector, cached per value
        (a per-chunk host->device copy would synchronise the stream)."""
        cache = self.__dict__.setdefault("_mi355x_pos", {})
        key = (tuple(pos.tolist()), str(device))
        c = cache.get(key)
        if c is None:
            c = cache[key] = pos.to(torch.int32).to(device)
        return c

    def _rope1d(self, pos: torch.Tensor, dim: int, device):
        cos, sin = self.rope1d.tables(dim, int(pos.max()), device)
        return self._i32(pos, device), cos, sin

    def trainable(self) -> bool:
        """A training step for this head: train mode, autograd enabled and
        trainable parameters (Lightning's training_step, run_model.py:232).
        In eval mode the fused inference path runs and builds no graph, as
        Lightning's validation / test steps run under no_grad anyway."""
        return self.training and torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())

    def forward(self, tokens: torch.Tensor, image_size: Tuple[int, int], next_num_overlap: int,
                overlap_tokens: torch.Tensor = None, memory_tokens: torch.Tensor = None):
        """alignment_head.py:224-345 -> (chunk_sim3 (B,1,8), frame_se3 (B,S-1,7),
        memory (B,N,dec)|None, new_overlap_tokens (B, ov+1, P+1, C)).

        With gradients enabled and trainable parameters this runs the
        autograd path (aligned_vggt.autograd: checkpoint-style block Functions
        with HIP backward kernels); otherwise the fused inference path."""
        if self.trainable():
            return self._forward_train(tokens, image_size, next_num_overlap, overlap_tokens, memory_tokens)
        with torch.no_grad():
            return self._forward_infer(tokens, image_size, next_num_overlap, overlap_tokens, memory_tokens)

    def _positions(self, S: int, T: Optional[int], dev):
        """Temporal 1-D RoPE positions (alignment_head.py:274-286): queries
        att_ids, keys cross_ids (previous chunk's first frame at 0)."""
        C = self.embed_dim
        seq = torch.arange(S)
        if T is not None:
            att = seq + (S - (T - 1))
            cross = torch.cat([seq[:1], seq[-(T - 1):]])
            return self._rope1d(att, C // self.num_heads, dev), self._rope1d(cross, C // self.num_heads, dev)
        r = self._rope1d(seq, C // self.num_heads, dev)
        return r, r

    def _forward_train(self, tokens, image_size, next_num_overlap, overlap_tokens, memory_tokens):
        if tokens.device.type != "cuda":
            raise RuntimeError("AlignmentHead: the MI355X hot path runs on HIP devices only (no CPU fallback)")
        if not self.temporal_attention:
            raise NotImplementedError("temporal_attention=False is not supported (see forward)")
        if tokens.requires_grad:
            raise NotImplementedError("gradients into the aggregator tokens: the reference training config freezes "
                                      "the aggregator (train_featureAlignedVGGT_vkitti.yaml:80-83)")
        H_img, W_img = image_size
        B, S, P, Cin = tokens.shape
        C = self.embed_dim
        dev = tokens.device
        P1 = P + 1
        M = B * S * P1
        x = AG.ProjectInFn.apply(tokens.detach().float().contiguous(), self, round_up(M, 256),
                                 self.project_in.weight, self.project_in.bias, self.token_norm.weight,
                                 self.token_norm.bias, self.per_frame_alignment_token)
        first_chunk = overlap_tokens is None
        if not first_chunk:
            assert overlap_tokens.shape[0] == B and overlap_tokens.shape[2] == 1 + P and \
                overlap_tokens.shape[3] == C, "Size of tokens and overlap tokens must match"
            if overlap_tokens.device != dev:
                raise RuntimeError("overlap_tokens must already be on the chunk's device "
                                   "(the reference's .to() at alignment_head.py:256-257 is a no-op)")
            T = overlap_tokens.shape[1]
            # detached, alignment_head.py:262
            y = overlap_tokens.detach().reshape(B * T * P1, C).float().contiguous()
            nk = T
        else:
            T, y, nk = None, None, S
        rq, rk = self._positions(S, T, dev)
        r2 = self._rope2d(H_img // self.patch_size, W_img // self.patch_size, dev)
        for i in range(self.aa_block_num):
            fb = self.frame_blocks[i]
            x = AG.FrameBlockFn.apply(x, fb, (B * S, P1), r2, *AG.frame_block_params(fb))
            tb = self.temporal_blocks[i]
            x = AG.TemporalBlockFn.apply(x, y, tb, B * P1, S, nk, rq, rk, *AG.temporal_block_params(tb))
        tok4 = x.view(B, S, P1, C)
        chunk_sim3, frame_se3, memory = self._decode_train(tok4[..., 0, :], next_num_overlap, first_chunk,
                                                           memory_tokens)
        new_overlap = torch.cat([tok4[:, :1], tok4[:, -next_num_overlap:]], dim=1).contiguous()
        return chunk_sim3, frame_se3, memory, new_overlap

    def _frame_dropout(self, frame_tokens: torch.Tensor, num_overlap: int, is_first_chunk: bool) -> torch.Tensor:
        """alignment_head.py:500-510: training-mode dropout of non-overlap frame
        tokens (not for the first chunk, never the overlap frames)."""
        B, S1, _ = frame_tokens.shape
        if self.training and self.drop_prob_nonoverlap > 0.0 and not is_first_chunk and (S1 - num_overlap) > 1:
            keep = self._dropout_mask(B, S1 - num_overlap, frame_tokens.device)
            mask = torch.cat((keep, torch.ones((B, num_overlap, 1), device=frame_tokens.device)), dim=1)
            return frame_tokens * mask * (1.0 / (1.0 - self.drop_prob_nonoverlap))
        return frame_tokens

    def _dropout_mask(self, B: int, n: int, device) -> torch.Tensor:
        return (torch.rand(B, n, device=device) > self.drop_prob_nonoverlap).float().unsqueeze(-1)

    def _decode_train(self, frame_alignment_tokens, num_overlap, is_first_chunk, memory_tokens=None):
        """_decode_alignments (alignment_head.py:427-540) on fp32 HIP autograd
        Functions; memory tokens keep their gradient (:482-484)."""
        B, S, Ce = frame_alignment_tokens.shape
        dev = frame_alignment_tokens.device
        dec = self.project_dec.out_features
        nm = self.num_memory_tokens
        seq = torch.arange(1, S)
        cross = torch.arange(0, S + nm) if nm > 0 else torch.arange(0, S)
        if nm > 0:
            cross[-nm:] += S
        hd = dec // self.num_heads
        maxp = int(max(cross.max(), seq.max() if S > 1 else 0))
        tabs = self.rope1d.tables(hd, maxp, dev)
        i32 = lambda t: self._i32(t, dev)
        tok = AG.linear_f32(self.project_dec, frame_alignment_tokens.float())
        tok = AG.layernorm_f32(self.dec_norm, tok)
        directional = None
        if nm > 0:
            norm_t = tok.norm(dim=-1).mean(dim=-1, keepdim=True).unsqueeze(1)
            if memory_tokens is None:
                mem = self.memory_token.expand(B, *self.memory_token.shape[1:])
                fi = AG.linear_f32(self.frame_proj, tok[:, 0]).view(B, nm, dec)
                fdir = fi / fi.norm(dim=-1, keepdim=True).clamp_min(1e-6)
                a = torch.sigmoid(self.alpha)
                directional = (1 - a) * mem + a * fdir
                eff = mem * norm_t
            else:
                directional = memory_tokens
                eff = memory_tokens * norm_t
            cross_tok = torch.cat([tok, eff], dim=1)
        else:
            cross_tok = tok
        first = tok[:, :1]
        pq, pk = i32(torch.zeros(1, dtype=cross.dtype)), i32(cross)
        for blk in self.chunk_cross_blocks:
            first = blk.forward_f32_train(first, cross_tok, pq, pk, tabs)
        memory = self.gated_update.forward_train(directional, first) if nm > 0 else None
        chunk_tok = AG.layernorm_f32(self.chunk_norm, first)
        frame_tokens = self._frame_dropout(tok[:, 1:], num_overlap, is_first_chunk)
        fq, fk = i32(seq), i32(torch.zeros(1, dtype=seq.dtype))
        for blk in self.frame_cross_blocks:
            frame_tokens = blk.forward_f32_train(frame_tokens, chunk_tok, fq, fk, tabs)
        frame_tokens = AG.layernorm_f32(self.frame_norm, frame_tokens)
        d = self.frame_se3_decoder
        frame_se3 = AG.linear_f32(d.fc2, AG.linear_f32(d.fc1, frame_tokens, gelu=True))
        d = self.chunk_sim3_decoder
        cs = AG.linear_f32(d.fc2, AG.linear_f32(d.fc1, chunk_tok, gelu=True))
        chunk_sim3 = torch.cat([cs[..., :-1], torch.exp(cs[..., -1:])], dim=-1)
        return chunk_sim3, frame_se3, memory

    def _forward_infer(self, tokens: torch.Tensor, image_size: Tuple[int, int], next_num_overlap: int,
                       overlap_tokens: torch.Tensor = None, memory_tokens: torch.Tensor = None):
        x = self.prepare_infer(tokens, image_size)
        B, S, P, _ = tokens.shape
        return self.forward_prepared(x, (B, S, P), image_size, next_num_overlap, overlap_tokens, memory_tokens)

    @torch.no_grad()
    def prepare_infer(self, tokens: torch.Tensor, image_size: Tuple[int, int]) -> torch.Tensor:
        """The context-free prefix of the inference forward (alignment_head.py:242-270
        and the first frame block, :347-366): project_in, token_norm, the
        per-frame alignment tokens and frame block 0 depend only on this
        chunk's aggregator tokens, not on the previous chunk -- the multi-GPU
        pipeline runs them with the encode, off the alignment recurrence.
        Returns the fp32 residual rows [round_up(B*S*(P+1), 256), C]."""
        if tokens.device.type != "cuda":
            raise RuntimeError("AlignmentHead: the MI355X hot path runs on HIP devices only (no CPU fallback)")
        if not self.temporal_attention:
            raise NotImplementedError("temporal_attention=False: the reference builds global_blocks but keeps aa_order="
                                      "['frame', 'temporal'] (alignment_head.py:80, :146), so its forward fails; "
                                      "not part of any BASELINE configuration")
        H_img, W_img = image_size
        B, S, P, Cin = tokens.shape
        C = self.embed_dim
        dev = tokens.device
        ws = Workspace.get(dev)
        P1 = P + 1
        M_in = B * S * P
        M = B * S * P1
        # project_in under autocast: fp32 tokens -> bf16 -> GEMM -> bf16
        tin = ws.buf("ah_in", M_in, Cin, torch.bfloat16)
        N.cast_f32_bf16(tokens.reshape(M_in, Cin), tin)
        w, b = pack_linear(self.project_in)
        pr = ws.buf("ah_proj", M_in, C, torch.bfloat16)
        N.gemm_bf16(tin, w, b, pr, N.EPI_BF16)
        # token_norm -> rows f*P1 + 1 + p; alignment token -> row f*P1
        x = torch.empty(round_up(M, 256), C, device=dev, dtype=torch.float32)
        N.layernorm_grouped(pr, self.token_norm.weight, self.token_norm.bias, self.token_norm.eps, x, M_in, C, P, P, 0,
                            P1, 1)
        al = self.per_frame_alignment_token[0].detach().float().contiguous()  # (2, 1, C)
        N.special_tokens(x, B * S, S, P1, al)
        r2 = self._rope2d(H_img // self.patch_size, W_img // self.patch_size, dev)
        self.frame_blocks[0].forward_rows(x, M, (B * S, P1, P1), r2, ws, tag="align_frame_attn")
        return x

    @torch.no_grad()
    def forward_prepared(self, x: torch.Tensor, bsp: Tuple[int, int, int], image_size: Tuple[int, int],
                         next_num_overlap: int, overlap_tokens: torch.Tensor = None,
                         memory_tokens: torch.Tensor = None):
        """The recurrent part of the inference forward (alignment_head.py:270-345
        from the first temporal block on), on the rows ``prepare_infer`` made
        (updated in place).  ``bsp`` = (B, S, P) of the aggregator tokens."""
        B, S, P = bsp
        H_img, W_img = image_size
        C = self.embed_dim
        dev = x.device
        ws = Workspace.get(dev)
        P1 = P + 1
        M = B * S * P1
        assert x.shape[0] >= M and x.shape[1] == C and x.dtype == torch.float32
        first_chunk = overlap_tokens is None
        if not first_chunk:
            assert overlap_tokens.shape[0] == B and overlap_tokens.shape[2] == 1 + P and \
                overlap_tokens.shape[3] == C, "Size of tokens and overlap tokens must match"
            T = overlap_tokens.shape[1]
            if overlap_tokens.device != dev:
                raise RuntimeError("overlap_tokens must already be on the chunk's device "
                                   "(the reference's .to() at alignment_head.py:256-257 is a no-op)")
            y = overlap_tokens.detach().reshape(B * T * P1, C).float().contiguous()
            seq = torch.arange(S)
            att = seq + (S - (T - 1))
            cross = torch.cat([seq[:1], seq[-(T - 1):]])
            rq = self._rope1d(att, C // self.num_heads, dev)
            rk = self._rope1d(cross, C // self.num_heads, dev)
            My, nk = B * T * P1, T
        else:
            y = None
            seq = torch.arange(S)
            rq = rk = self._rope1d(seq, C // self.num_heads, dev)
            My, nk = M, S

        ph, pw = H_img // self.patch_size, W_img // self.patch_size
        r2 = self._rope2d(ph, pw, dev)
        for i in range(self.aa_block_num):
            if i > 0:  # frame block 0 ran in prepare_infer
                self.frame_blocks[i].forward_rows(x, M, (B * S, P1, P1), r2, ws, tag="align_frame_attn")
            self.temporal_blocks[i].forward_rows_bf16(x, M, y, My, B * P1, S, nk, rq, rk, ws)

        tok4 = x[:M].view(B, S, P1, C)
        frame_tok = tok4[..., 0, :].contiguous()
        chunk_sim3, frame_se3, memory = self._decode_alignments(frame_tok, next_num_overlap, first_chunk,
                                                                memory_tokens)
        new_overlap = torch.cat([tok4[:, :1], tok4[:, -next_num_overlap:]], dim=1).contiguous()
        return chunk_sim3, frame_se3, memory, new_overlap

    # ------------------------------------------------------------------
    @torch.no_grad()
    def _decode_alignments(self, frame_alignment_tokens: torch.Tensor, num_overlap: int, is_first_chunk: bool,
                           memory_tokens: torch.Tensor = None):
        """alignment_head.py:427-540 (fp32; frame dropout in training mode)."""
        B, S, Ce = frame_alignment_tokens.shape
        dev = frame_alignment_tokens.device
        dec = self.project_dec.out_features
        nm = self.num_memory_tokens
        seq = torch.arange(1, S)
        pos_frame_q, pos_frame_k = seq, torch.zeros(1, dtype=seq.dtype)
        cross = torch.arange(0, S + nm) if nm > 0 else torch.arange(0, S)
        if nm > 0:
            cross[-nm:] += S
        pos_cross_q = torch.zeros(1, dtype=cross.dtype)
        hd = dec // self.num_heads
        maxp = int(max(cross.max(), seq.max() if S > 1 else 0))
        tabs = self.rope1d.tables(hd, maxp, dev)
        i32 = lambda t: self._i32(t, dev)

        ft = frame_alignment_tokens.reshape(B * S, Ce).float().contiguous()
        tok = torch.empty(B * S, dec, device=dev)
        N.linear_f32(ft, self.project_dec.weight, self.project_dec.bias, tok)
        N.layernorm(tok, self.dec_norm.weight, self.dec_norm.bias, self.dec_norm.eps, tok)
        tok = tok.view(B, S, dec)
        directional = None
        if nm > 0:
            norm_t = tok.norm(dim=-1).mean(dim=-1, keepdim=True).unsqueeze(1)
            if memory_tokens is None:
                mem = self.memory_token.detach().expand(B, *self.memory_token.shape[1:])
                fi = torch.empty(B, nm * dec, device=dev)
                N.linear_f32(tok[:, 0], self.frame_proj.weight, self.frame_proj.bias, fi)
                fi = fi.view(B, nm, dec)
                fdir = fi / fi.norm(dim=-1, keepdim=True).clamp_min(1e-6)
                a = torch.sigmoid(self.alpha.detach())
                directional = (1 - a) * mem + a * fdir
                eff = mem * norm_t
            else:
                directional = memory_tokens
                eff = memory_tokens * norm_t
            cross_tok = torch.cat([tok, eff], dim=1)
        else:
            cross_tok = tok
        first = tok[:, :1]
        for blk in self.chunk_cross_blocks:
            first = blk.forward_f32(first, cross_tok, i32(pos_cross_q), i32(cross), tabs)
        memory = self.gated_update(directional, first) if nm > 0 else None
        chunk_tok = torch.empty(B, dec, device=dev)
        N.layernorm(first.reshape(B, dec), self.chunk_norm.weight, self.chunk_norm.bias, self.chunk_norm.eps,
                    chunk_tok)
        chunk_tok = chunk_tok.view(B, 1, dec)
        frame_tokens = self._frame_dropout(tok[:, 1:], num_overlap, is_first_chunk)
        for blk in self.frame_cross_blocks:
            frame_tokens = blk.forward_f32(frame_tokens, chunk_tok, i32(pos_frame_q), i32(pos_frame_k), tabs)
        fr = frame_tokens.reshape(B * (S - 1), dec)
        N.layernorm(fr, self.frame_norm.weight, self.frame_norm.bias, self.frame_norm.eps, fr)
        frame_se3 = _mlp_f32(self.frame_se3_decoder, fr).view(B, S - 1, -1)
        chunk_sim3 = _mlp_f32(self.chunk_sim3_decoder, chunk_tok.reshape(B, dec)).view(B, 1, -1)
        chunk_sim3[:, :, -1] = torch.exp(chunk_sim3[:, :, -1])
        return chunk_sim3, frame_se3, memory


def _mlp_f32(mlp: Mlp, x: torch.Tensor) -> torch.Tensor:
    h = torch.empty(x.shape[0], mlp.fc1.out_features, device=x.device)
    N.linear_f32(x, mlp.fc1.weight, mlp.fc1.bias, h, N.EPI_GELU_BF16)
    o = torch.empty(x.shape[0], mlp.fc2.out_features, device=x.device)
    N.linear_f32(h, mlp.fc2.weight, mlp.fc2.bias, o, N.EPI_F32)
    return o


def slice_expand_and_flatten(token_tensor: torch.Tensor, B: int, S: int) -> torch.Tensor:
    """alignment_head.py:543-568: (1,2,X,C) -> (B,S,X,C)."""
    query = token_tensor[:, 0:1, ...].expand(B, 1, *token_tensor.shape[2:])
    others = token_tensor[:, 1:, ...].expand(B, S - 1, *token_tensor.shape[2:])
    return torch.cat([query, others], dim=1)
