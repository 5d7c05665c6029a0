"""Autograd for training the alignment head on the HIP path (SURVEY.md §8f
row 4).

The reference trains only ``alignment_head.*`` (train_featureAlignedVGGT_vkitti.yaml:
80-83 freezes the aggregator, camera and depth heads) under bf16-mixed
autocast (run_model.py:472), with every trunk / decoder block wrapped in
``torch.utils.checkpoint`` (alignment_head.py:351-426, use_reentrant=False).
This module mirrors that structure MI355X-first:

* Trunk blocks (frame Block, temporal CrossAttentionBlock; bf16 tier) are ONE
  ``torch.autograd.Function`` each.  Forward saves only the block input (the
  checkpoint contract); backward recomputes the block with the unfused
  training kernels (plain bf16 GEMMs, q/k norm + RoPE, LSE-emitting attention,
  GELU, LayerScale residual) and then runs the whole backward chain as HIP
  launches: LayerScale / bias reductions, GELU backward, dX = dY W and
  dW = dY^T X bf16 GEMMs (vggt_gemm_bf16 on transposed operands), flash
  attention backward (frame blocks) or small-window attention backward
  (temporal blocks), per-head norm + RoPE backward, LayerNorm backward.
* project_in + token_norm + alignment tokens: one Function.
* Decoder (fp32 tier, autocast disabled, alignment_head.py:340): fp32 HIP
  Functions per Linear / LayerNorm / q-k norm + RoPE / small attention,
  composed by torch autograd with the decoder's small tensor glue (memory
  init, GatedUpdate algebra), exactly like the inference path.

Gradient numerics follow autocast: gradients of bf16 activations are bf16,
parameter gradients are the bf16 GEMM results widened to fp32.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn as nn

from . import _native as N
from .runtime import Workspace, pack_linear, round_up


# ----------------------------------------------------------------- helpers
def _transposed(w: torch.Tensor) -> torch.Tensor:
    """Dense row-major copy of w^T (``.t().contiguous()`` keeps a stride-N
    inner dim when N == 1, which the C ABI's leading-dimension check rejects)."""
    out = torch.empty(w.shape[1], w.shape[0], device=w.device, dtype=w.dtype)
    out.copy_(w.t())
    return out


def _zeros(n: int, device) -> torch.Tensor:
    key = ("_zeros", str(device))
    t = _CACHE.get(key)
    if t is None or t.numel() < n:
        t = torch.zeros(max(n, 4096), device=device)
        _CACHE[key] = t
    return t[:n]


_CACHE = {}


def _wt_bf16(lin: nn.Linear) -> torch.Tensor:
    """bf16 W^T [K, N] of a Linear (dX = dY W as vggt_gemm_bf16(dY, W^T)); cached per weight version."""
    w, _ = pack_linear(lin)
    key = lin.__dict__["_mi355x_pack"][0]  # the parameters' versions
    c = lin.__dict__.get("_mi355x_wt")
    if c is None or c[0] != key:
        c = (key, _transposed(w))
        lin.__dict__["_mi355x_wt"] = c
    return c[1]


def _wt_f32(w: torch.Tensor, owner: nn.Module, name: str) -> torch.Tensor:
    key = (w.data_ptr(), w._version)
    attr = "_mi355x_wt32_" + name
    c = owner.__dict__.get(attr)
    if c is None or c[0] != key:
        c = (key, _transposed(w.detach().float()))
        owner.__dict__[attr] = c
    return c[1]


class _LinBwd:
    """bf16-tier Linear backward:
    dX = dY . W  through the forward GEMM kernel (W^T packed once per weight version),
    dW = dY^T . X by the split-K weight-gradient kernel (vggt_wgrad_bf16: row-major
    operands, the token dimension as the MFMA reduction, no transposes); shapes
    it does not cover go through transposed operands + the forward GEMM."""

    def __init__(self, ws: Workspace, M: int):
        self.ws = ws
        self.M = M
        self.Mp = round_up(max(M, 1), 64)

    def dx(self, dy: torch.Tensor, lin: nn.Linear, out: torch.Tensor) -> None:
        wt = _wt_bf16(lin)
        N.gemm_bf16(dy, wt, _zeros(wt.shape[0], dy.device), out, N.EPI_BF16)

    def dw(self, dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor) -> None:
        """out [N, K] fp32 = dy[M, N]^T x[M, K] (bf16-rounded like autocast's bf16 weight gradient)."""
        Nn, K = dy.shape[1], x.shape[1]
        if Nn % 128 == 0 and K % 128 == 0:
            N.wgrad_bf16(dy, x, out, False)
            return
        a = self.ws.buf("tr_a", Nn, self.Mp, torch.bfloat16)
        b = self.ws.buf("tr_b", K, self.Mp, torch.bfloat16)
        N.transpose_b16(dy, a, self.Mp)
        N.transpose_b16(x, b, self.Mp)
        N.gemm_bf16(a, b, _zeros(K, dy.device), out, N.EPI_F32)


_ARENA = os.environ.get("VGGT_GRAD_ARENA", "1") != "0"


class _GradArena:
    """The zero-initialised fp32 parameter gradients of one backward, carved out of
    ONE zero-filled buffer: one fill launch instead of one per parameter (the
    training step issued ~670 fills of ~4 us each, plus their dispatch gaps).
    The views are contiguous and shaped like their parameters, so autograd's
    AccumulateGrad adopts them as .grad without a copy."""

    def __init__(self, device, tensors):
        self.buf = torch.zeros(sum(t.numel() for t in tensors if t is not None), device=device) if _ARENA else None
        self.off = 0

    def like(self, t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        if t is None:
            return None
        if self.buf is None:  # VGGT_GRAD_ARENA=0: one zero fill per parameter (A/B)
            return torch.zeros_like(t, dtype=torch.float32)
        v = self.buf[self.off:self.off + t.numel()].view(t.shape)
        self.off += t.numel()
        return v

    def lin(self, lin: nn.Linear):
        return self.like(lin.weight), self.like(lin.bias)

    def ln(self, ln: nn.LayerNorm):
        return self.like(ln.weight), self.like(ln.bias)


def _params_of(*mods) -> list:
    out = []
    for m in mods:
        if isinstance(m, torch.Tensor):
            out.append(m)
        elif isinstance(m, (nn.Linear, nn.LayerNorm)):
            out += [m.weight, m.bias]
    return out


def _mlp_fwd(blk, x1: torch.Tensor, ws: Workspace, pfx: str):
    """Shared second half of the bf16-tier blocks: LN2 -> fc1 -> GELU -> fc2 (branch)."""
    M, C = x1.shape
    xn2 = ws.buf(pfx + "xn2", M, C, torch.bfloat16)
    N.layernorm(x1, blk.norm2.weight, blk.norm2.bias, blk.norm2.eps, xn2)
    w1, b1 = pack_linear(blk.mlp.fc1)
    hpre = ws.buf(pfx + "hpre", M, w1.shape[0], torch.bfloat16)
    h = ws.buf(pfx + "h", M, w1.shape[0], torch.bfloat16)
    N.gemm_bf16_gelu_pre(xn2, w1, b1, h, hpre)  # GELU in the epilogue, pre-activation kept for the backward
    w2, b2 = pack_linear(blk.mlp.fc2)
    br2 = ws.buf(pfx + "br2", M, C, torch.bfloat16)
    N.gemm_bf16(h, w2, b2, br2, N.EPI_BF16)
    return xn2, hpre, h, br2


def _mlp_bwd(blk, dx: torch.Tensor, x1, xn2, hpre, h, br2, g, lb: _LinBwd, ws: Workspace, pfx: str):
    """dx (fp32, holds d(out)) -> dx holds d(x1); fills g[...] for ls2, fc2, fc1, norm2."""
    M, C = dx.shape
    dbr = ws.buf(pfx + "dbr", M, C, torch.bfloat16)
    N.layerscale_bwd(dx, br2, blk.ls2.gamma.detach(), dbr, g["ls2"], g["fc2.b"])
    lb.dw(dbr, h, g["fc2.w"])
    dh = ws.buf(pfx + "dh", M, blk.mlp.fc1.out_features, torch.bfloat16)
    lb.dx(dbr, blk.mlp.fc2, dh)
    N.gelu_bwd(dh, hpre, dh, g["fc1.b"])
    lb.dw(dh, xn2, g["fc1.w"])
    dxn = ws.buf(pfx + "dxn", M, C, torch.bfloat16)
    lb.dx(dh, blk.mlp.fc1, dxn)
    N.layernorm_bwd(x1, blk.norm2.weight, blk.norm2.eps, dxn, dx, True, g["norm2.w"], g["norm2.b"])


# ----------------------------------------------------------------- frame Block (bf16 tier)
class FrameBlockFn(torch.autograd.Function):
    """vggt Block (ext layers/block.py) with QK-norm + RoPE-2D, as the
    alignment head's frame blocks (alignment_head.py:347-366 under
    checkpoint).  x: fp32 rows [M, C]; attention over ``groups`` = (nb, rows)."""

    @staticmethod
    def _recompute(blk, x, groups, rope, ws):
        M, C = x.shape
        H = blk.attn.num_heads
        D = C // H
        nb, rows = groups
        xn1 = ws.buf("fb_xn1", M, C, torch.bfloat16)
        N.layernorm(x, blk.norm1.weight, blk.norm1.bias, blk.norm1.eps, xn1)
        w, b = pack_linear(blk.attn.qkv)
        qpre = ws.buf("fb_qkvpre", M, 3 * C, torch.bfloat16)
        N.gemm_bf16(xn1, w, b, qpre, N.EPI_BF16)
        qn, kn = blk.attn.q_norm, blk.attn.k_norm
        has_norm = isinstance(qn, nn.LayerNorm)
        mode = rope.mode if (rope is not None and blk.attn.rope is not None) else N.ROPE_NONE
        if has_norm or mode != N.ROPE_NONE:
            # q|k normalised out of place (the backward needs the pre-norm
            # values); v is read from the projection itself
            qk = ws.buf("fb_qk", M, 2 * C, torch.bfloat16)
            N.qknorm_rope_out(qpre, qk, H, D, qn.weight if has_norm else None, qn.bias if has_norm else None,
                              kn.weight if has_norm else None, kn.bias if has_norm else None,
                              qn.eps if has_norm else 0.0, mode, rope.pos if mode else None,
                              rope.period if mode else 1, rope.cos if mode else None, rope.sin if mode else None)
            qkv = (qk[:, :C], qk[:, C:], qpre[:, 2 * C:])
        else:
            qkv = (qpre[:, :C], qpre[:, C:2 * C], qpre[:, 2 * C:])
        ao = ws.buf("fb_ao", M, C, torch.bfloat16)
        lse = ws.buf("fb_lse", 1, nb * H * rows, torch.float32)
        N.attention_fwd_lse(qkv[0], qkv[1], qkv[2], ao, lse, nb, H, rows, rows, D, rows, rows, rows)
        wp, bp = pack_linear(blk.attn.proj)
        br1 = ws.buf("fb_br1", M, C, torch.bfloat16)
        N.gemm_bf16(ao, wp, bp, br1, N.EPI_BF16)
        x1 = ws.buf("fb_x1", M, C, torch.float32)
        N.resid_scale_add_from(x1, x, br1, blk.ls1.gamma.detach())
        xn2, hpre, h, br2 = _mlp_fwd(blk, x1, ws, "fb_")
        return dict(xn1=xn1, qpre=qpre, qkv=qkv, ao=ao, lse=lse, br1=br1, x1=x1, xn2=xn2, hpre=hpre, h=h, br2=br2,
                    has_norm=has_norm, mode=mode)

    @staticmethod
    def forward(ctx, x, blk, groups, rope, *params):
        ws = Workspace.get(x.device)
        t = FrameBlockFn._recompute(blk, x, groups, rope, ws)
        out = torch.empty_like(t["x1"])
        N.resid_scale_add_from(out, t["x1"], t["br2"], blk.ls2.gamma.detach())
        ctx.save_for_backward(x)
        ctx.blk, ctx.groups, ctx.rope = blk, groups, rope
        return out

    @staticmethod
    def backward(ctx, dout):
        (x,) = ctx.saved_tensors
        blk, groups, rope = ctx.blk, ctx.groups, ctx.rope
        ws = Workspace.get(x.device)
        M, C = x.shape
        H = blk.attn.num_heads
        D = C // H
        nb, rows = groups
        t = FrameBlockFn._recompute(blk, x, groups, rope, ws)
        g = {}
        qn, kn = blk.attn.q_norm, blk.attn.k_norm
        ar = _GradArena(x.device, _params_of(blk.norm1, blk.attn.qkv, *((qn, kn) if t["has_norm"] else ()),
                                             blk.attn.proj, blk.ls1.gamma, blk.norm2, blk.mlp.fc1, blk.mlp.fc2,
                                             blk.ls2.gamma))
        g["norm1.w"], g["norm1.b"] = ar.ln(blk.norm1)
        g["qkv.w"], g["qkv.b"] = ar.lin(blk.attn.qkv)
        if t["has_norm"]:
            g["qn.w"], g["qn.b"] = ar.ln(qn)
            g["kn.w"], g["kn.b"] = ar.ln(kn)
        g["proj.w"], g["proj.b"] = ar.lin(blk.attn.proj)
        g["ls1"] = ar.like(blk.ls1.gamma)
        g["norm2.w"], g["norm2.b"] = ar.ln(blk.norm2)
        g["fc1.w"], g["fc1.b"] = ar.lin(blk.mlp.fc1)
        g["fc2.w"], g["fc2.b"] = ar.lin(blk.mlp.fc2)
        g["ls2"] = ar.like(blk.ls2.gamma)
        lb = _LinBwd(ws, M)
        dx = dout.float().contiguous().clone()
        _mlp_bwd(blk, dx, t["x1"], t["xn2"], t["hpre"], t["h"], t["br2"], g, lb, ws, "fbb_")
        # attention branch: x1 = x + ls1 * proj(attn)
        dbr = ws.buf("fbb_dbr", M, C, torch.bfloat16)
        N.layerscale_bwd(dx, t["br1"], blk.ls1.gamma.detach(), dbr, g["ls1"], g["proj.b"])
        lb.dw(dbr, t["ao"], g["proj.w"])
        dao = ws.buf("fbb_dxn", M, C, torch.bfloat16)
        lb.dx(dbr, blk.attn.proj, dao)
        qkv = t["qkv"]
        dqkv = ws.buf("fbb_dqkv", M, 3 * C, torch.bfloat16)
        N.attention_bwd(qkv[0], qkv[1], qkv[2], t["ao"], dao, t["lse"], dqkv[:, :C],
                        dqkv[:, C:2 * C], dqkv[:, 2 * C:], nb, H, rows, rows, D, rows, rows, rows)
        mode = t["mode"]
        if t["has_norm"] or mode != N.ROPE_NONE:
            hn = t["has_norm"]
            N.headnorm_rope_bwd(t["qpre"][:, :2 * C], dqkv[:, :2 * C], 2 * H, H, D, qn.weight if hn else None,
                                kn.weight if hn else None, qn.eps if hn else 0.0, mode,
                                rope.pos if mode else None, rope.period if mode else 1, rope.cos if mode else None,
                                rope.sin if mode else None, g.get("qn.w"), g.get("qn.b"), g.get("kn.w"),
                                g.get("kn.b"))
        N.colsum(dqkv, g["qkv.b"])
        lb.dw(dqkv, t["xn1"], g["qkv.w"])
        dxn1 = ws.buf("fbb_dxn", M, C, torch.bfloat16)
        lb.dx(dqkv, blk.attn.qkv, dxn1)
        N.layernorm_bwd(x, blk.norm1.weight, blk.norm1.eps, dxn1, dx, True, g["norm1.w"], g["norm1.b"])
        grads = [g["norm1.w"], g["norm1.b"], g["qkv.w"], g["qkv.b"]]
        grads += [g["qn.w"], g["qn.b"], g["kn.w"], g["kn.b"]] if t["has_norm"] else []
        grads += [g["proj.w"], g["proj.b"], g["ls1"], g["norm2.w"], g["norm2.b"], g["fc1.w"], g["fc1.b"],
                  g["fc2.w"], g["fc2.b"], g["ls2"]]
        return (dx, None, None, None, *grads)


def frame_block_params(blk) -> list:
    p = [blk.norm1.weight, blk.norm1.bias, blk.attn.qkv.weight, blk.attn.qkv.bias]
    if isinstance(blk.attn.q_norm, nn.LayerNorm):
        p += [blk.attn.q_norm.weight, blk.attn.q_norm.bias, blk.attn.k_norm.weight, blk.attn.k_norm.bias]
    p += [blk.attn.proj.weight, blk.attn.proj.bias, blk.ls1.gamma, blk.norm2.weight, blk.norm2.bias,
          blk.mlp.fc1.weight, blk.mlp.fc1.bias, blk.mlp.fc2.weight, blk.mlp.fc2.bias, blk.ls2.gamma]
    return p


# ----------------------------------------------------------------- temporal CrossAttentionBlock (bf16 tier)
class TemporalBlockFn(torch.autograd.Function):
    """CrossAttentionBlock (cross_attention.py:84-131) as the alignment head's
    temporal blocks (alignment_head.py:368-393 under checkpoint): queries are
    ``groups`` runs of nq rows of x, keys runs of nk rows of y (y None: y = x,
    the first chunk's time-aware self attention; otherwise the detached
    overlap tokens, alignment_head.py:262)."""

    @staticmethod
    def _recompute(blk, x, y, groups, nq, nk, rq, rk, ws):
        Mx, C = x.shape
        H = blk.attn.num_heads
        D = C // H
        ysrc = x if y is None else y
        My = ysrc.shape[0]
        xn1 = ws.buf("tb_xn1", Mx, C, torch.bfloat16)
        N.layernorm(x, blk.norm1.weight, blk.norm1.bias, blk.norm1.eps, xn1)
        yn = ws.buf("tb_yn", My, C, torch.bfloat16)
        N.layernorm(ysrc, blk.norm3.weight, blk.norm3.bias, blk.norm3.eps, yn)
        wq, bq = pack_linear(blk.attn.q)
        qpre = ws.buf("tb_qpre", Mx, C, torch.bfloat16)
        N.gemm_bf16(xn1, wq, bq, qpre, N.EPI_BF16)
        wkv, bkv = blk.attn.packed_kv()
        kvpre = ws.buf("tb_kvpre", My, 2 * C, torch.bfloat16)
        N.gemm_bf16(yn, wkv, bkv, kvpre, N.EPI_BF16)
        mode = N.ROPE_1D if blk.attn.rope is not None else N.ROPE_NONE
        q, k = qpre, kvpre[:, :C]
        for which, rp, src, nm in (("q", rq, qpre, "tb_q"), ("k", rk, kvpre, "tb_k")):
            w, b, eps = blk._qk_norm(which)
            if w is not None or mode != N.ROPE_NONE:
                # normalised out of place: the backward needs the pre-norm projections
                dst = ws.buf(nm, src.shape[0], C, torch.bfloat16)
                N.headnorm_rope_out(src, dst, H, D, w, b, eps, mode, rp[0] if mode else None,
                                    rp[0].numel() if mode else 1, rp[1] if mode else None, rp[2] if mode else None)
                if which == "q":
                    q = dst
                else:
                    k = dst
        v = kvpre[:, C:]
        ao = ws.buf("tb_ao", Mx, C, torch.bfloat16)
        N.attention_small(q, k, v, ao, groups, H, nq, nk, D, nq, nk, nq, exact=True)  # the backward's formula
        wp, bp = pack_linear(blk.attn.proj)
        br1 = ws.buf("tb_br1", Mx, C, torch.bfloat16)
        N.gemm_bf16(ao, wp, bp, br1, N.EPI_BF16)
        x1 = ws.buf("tb_x1", Mx, C, torch.float32)
        N.resid_scale_add_from(x1, x, br1, blk.ls1.gamma.detach())
        xn2, hpre, h, br2 = _mlp_fwd(blk, x1, ws, "tb_")
        return dict(ysrc=ysrc, xn1=xn1, yn=yn, qpre=qpre, kvpre=kvpre, q=q, k=k, v=v, ao=ao, br1=br1, x1=x1, xn2=xn2,
                    hpre=hpre, h=h, br2=br2, mode=mode)

    @staticmethod
    def forward(ctx, x, y, blk, groups, nq, nk, rq, rk, *params):
        ws = Workspace.get(x.device)
        t = TemporalBlockFn._recompute(blk, x, y, groups, nq, nk, rq, rk, ws)
        out = torch.empty_like(t["x1"])
        N.resid_scale_add_from(out, t["x1"], t["br2"], blk.ls2.gamma.detach())
        if y is None:
            ctx.save_for_backward(x)
        else:
            ctx.save_for_backward(x, y)
        ctx.self_attn = y is None
        ctx.blk, ctx.groups, ctx.nq, ctx.nk, ctx.rq, ctx.rk = blk, groups, nq, nk, rq, rk
        return out

    @staticmethod
    def backward(ctx, dout):
        if ctx.self_attn:
            (x,) = ctx.saved_tensors
            y = None
        else:
            x, y = ctx.saved_tensors
        blk = ctx.blk
        groups, nq, nk, rq, rk = ctx.groups, ctx.nq, ctx.nk, ctx.rq, ctx.rk
        ws = Workspace.get(x.device)
        Mx, C = x.shape
        H = blk.attn.num_heads
        D = C // H
        t = TemporalBlockFn._recompute(blk, x, y, groups, nq, nk, rq, rk, ws)
        My = t["ysrc"].shape[0]
        g = {}
        qn, kn = blk.attn.q_norm, blk.attn.k_norm
        has_norm = isinstance(qn, nn.LayerNorm)
        ar = _GradArena(x.device, _params_of(blk.norm1, blk.norm3, blk.norm2, blk.attn.q, blk.attn.k, blk.attn.v,
                                             blk.attn.proj, *((qn, kn) if has_norm else ()), blk.ls1.gamma,
                                             blk.mlp.fc1, blk.mlp.fc2, blk.ls2.gamma))
        for nm in ("norm1", "norm3", "norm2"):
            g[nm + ".w"], g[nm + ".b"] = ar.ln(getattr(blk, nm))
        for nm in ("q", "k", "v", "proj"):
            g[nm + ".w"], g[nm + ".b"] = ar.lin(getattr(blk.attn, nm))
        if has_norm:
            g["qn.w"], g["qn.b"] = ar.ln(qn)
            g["kn.w"], g["kn.b"] = ar.ln(kn)
        g["ls1"] = ar.like(blk.ls1.gamma)
        g["fc1.w"], g["fc1.b"] = ar.lin(blk.mlp.fc1)
        g["fc2.w"], g["fc2.b"] = ar.lin(blk.mlp.fc2)
        g["ls2"] = ar.like(blk.ls2.gamma)
        lb = _LinBwd(ws, Mx)
        dx = dout.float().contiguous().clone()
        _mlp_bwd(blk, dx, t["x1"], t["xn2"], t["hpre"], t["h"], t["br2"], g, lb, ws, "tbb_")
        dbr = ws.buf("tbb_dbr", Mx, C, torch.bfloat16)
        N.layerscale_bwd(dx, t["br1"], blk.ls1.gamma.detach(), dbr, g["ls1"], g["proj.b"])
        lb.dw(dbr, t["ao"], g["proj.w"])
        dao = ws.buf("tbb_dxn", Mx, C, torch.bfloat16)
        lb.dx(dbr, blk.attn.proj, dao)
        dq = ws.buf("tbb_dq", Mx, C, torch.bfloat16)
        dkv = ws.buf("tbb_dkv", My, 2 * C, torch.bfloat16)
        N.attention_small_bwd(t["q"], t["k"], t["v"], dao, dq, dkv[:, :C], dkv[:, C:], groups, H, nq, nk, D, nq, nk,
                              nq, nq, nk)
        mode = t["mode"]
        if has_norm or mode != N.ROPE_NONE:
            N.headnorm_rope_bwd(t["qpre"], dq, H, H, D, qn.weight if has_norm else None, None,
                                qn.eps if has_norm else 0.0, mode, rq[0] if mode else None,
                                rq[0].numel() if mode else 1, rq[1] if mode else None, rq[2] if mode else None,
                                g.get("qn.w"), g.get("qn.b"))
            N.headnorm_rope_bwd(t["kvpre"][:, :C], dkv[:, :C], H, H, D, kn.weight if has_norm else None, None,
                                kn.eps if has_norm else 0.0, mode, rk[0] if mode else None,
                                rk[0].numel() if mode else 1, rk[1] if mode else None, rk[2] if mode else None,
                                g.get("kn.w"), g.get("kn.b"))
        N.colsum(dq, g["q.b"])
        N.colsum(dkv[:, :C], g["k.b"])
        N.colsum(dkv[:, C:], g["v.b"])
        lb.dw(dq, t["xn1"], g["q.w"])
        lby = _LinBwd(ws, My)
        lby.dw(dkv[:, :C], t["yn"], g["k.w"])
        lby.dw(dkv[:, C:], t["yn"], g["v.w"])
        dxn1 = ws.buf("tbb_dxn", Mx, C, torch.bfloat16)
        lb.dx(dq, blk.attn.q, dxn1)
        N.layernorm_bwd(x, blk.norm1.weight, blk.norm1.eps, dxn1, dx, True, g["norm1.w"], g["norm1.b"])
        # k/v path: dyn = dk Wk + dv Wv
        dyn = ws.buf("tbb_dyn", My, C, torch.bfloat16)
        wkv_t = _kv_wt(blk.attn)
        N.gemm_bf16(dkv, wkv_t, _zeros(C, x.device), dyn, N.EPI_BF16)
        if y is None:
            N.layernorm_bwd(x, blk.norm3.weight, blk.norm3.eps, dyn, dx, True, g["norm3.w"], g["norm3.b"])
            dy = None
        else:
            dys = ws.buf("tbb_dys", My, C, torch.float32)
            N.layernorm_bwd(y, blk.norm3.weight, blk.norm3.eps, dyn, dys, False, g["norm3.w"], g["norm3.b"])
            dy = dys.clone() if ctx.needs_input_grad[1] else None
        grads = [g["norm1.w"], g["norm1.b"], g["norm3.w"], g["norm3.b"], g["q.w"], g["q.b"], g["k.w"], g["k.b"],
                 g["v.w"], g["v.b"]]
        grads += [g["qn.w"], g["qn.b"], g["kn.w"], g["kn.b"]] if has_norm else []
        grads += [g["proj.w"], g["proj.b"], g["ls1"], g["norm2.w"], g["norm2.b"], g["fc1.w"], g["fc1.b"],
                  g["fc2.w"], g["fc2.b"], g["ls2"]]
        return (dx, dy, None, None, None, None, None, None, *grads)


def _kv_wt(attn) -> torch.Tensor:
    """bf16 [Wk; Wv]^T = [C, 2C]: dyn = [dk | dv] . [Wk; Wv] in one GEMM."""
    wkv, _ = attn.packed_kv()
    key = attn.__dict__["_mi355x_kv"][0]
    c = attn.__dict__.get("_mi355x_kv_t")
    if c is None or c[0] != key:
        c = (key, _transposed(wkv))
        attn.__dict__["_mi355x_kv_t"] = c
    return c[1]


def temporal_block_params(blk) -> list:
    a = blk.attn
    p = [blk.norm1.weight, blk.norm1.bias, blk.norm3.weight, blk.norm3.bias, a.q.weight, a.q.bias, a.k.weight, a.k.bias,
         a.v.weight, a.v.bias]
    if isinstance(a.q_norm, nn.LayerNorm):
        p += [a.q_norm.weight, a.q_norm.bias, a.k_norm.weight, a.k_norm.bias]
    p += [a.proj.weight, a.proj.bias, blk.ls1.gamma, blk.norm2.weight, blk.norm2.bias, blk.mlp.fc1.weight,
          blk.mlp.fc1.bias, blk.mlp.fc2.weight, blk.mlp.fc2.bias, blk.ls2.gamma]
    return p


# ----------------------------------------------------------------- project_in + token_norm + alignment tokens
class ProjectInFn(torch.autograd.Function):
    """alignment_head.py:242-272: tokens (B,S,P,Cin) fp32 (frozen aggregator
    output, no gradient) -> project_in (bf16 autocast) -> token_norm (fp32)
    -> rows f*(P+1) + 1 + p of the residual stream, alignment token
    (slice_expand_and_flatten, :543-568) at rows f*(P+1)."""

    @staticmethod
    def forward(ctx, tokens, head, M_pad, w_in, b_in, tn_w, tn_b, al_tok):
        B, S, P, Cin = tokens.shape
        C = head.embed_dim
        dev = tokens.device
        ws = Workspace.get(dev)
        P1, M_in = P + 1, B * S * P
        M = B * S * P1
        tin = ws.buf("pi_in", M_in, Cin, torch.bfloat16)
        N.cast_f32_bf16(tokens.reshape(M_in, Cin), tin)
        w, b = pack_linear(head.project_in)
        pr = torch.empty(M_in, C, device=dev, dtype=torch.bfloat16)
        N.gemm_bf16(tin, w, b, pr, N.EPI_BF16)
        x = torch.empty(M_pad, C, device=dev, dtype=torch.float32)
        N.layernorm_grouped(pr, head.token_norm.weight, head.token_norm.bias, head.token_norm.eps, x, M_in, C, P, P, 0,
                            P1, 1)
        N.special_tokens(x, B * S, S, P1, al_tok.detach()[0].float().contiguous())
        ctx.save_for_backward(pr)
        ctx.head, ctx.shape = head, (B, S, P, Cin)
        ctx.tokens = tokens
        return x[:M]

    @staticmethod
    def backward(ctx, dx):
        (pr,) = ctx.saved_tensors
        head = ctx.head
        B, S, P, Cin = ctx.shape
        C = head.embed_dim
        dev = pr.device
        ws = Workspace.get(dev)
        P1, M_in = P + 1, B * S * P
        dx = dx.float().contiguous()
        ar = _GradArena(dev, _params_of(head.token_norm, head.project_in))
        dtw, dtb = ar.ln(head.token_norm)
        dpr = ws.buf("pib_dpr", M_in, C, torch.bfloat16)
        N.layernorm_bwd(pr, head.token_norm.weight, head.token_norm.eps, dx, dpr, False, dtw, dtb, M=M_in, group=P,
                        x_gstride=P, x_off=0, y_gstride=P1, y_off=1)
        dw, db = ar.lin(head.project_in)
        N.colsum(dpr, db)
        tin = ws.buf("pi_in", M_in, Cin, torch.bfloat16)
        N.cast_f32_bf16(ctx.tokens.reshape(M_in, Cin), tin)
        _LinBwd(ws, M_in).dw(dpr, tin, dw)
        d4 = dx.view(B, S, P1, C)[:, :, 0]
        dal = torch.zeros_like(head.per_frame_alignment_token)
        dal[0, 0, 0] = d4[:, 0].sum(0)
        if S > 1:
            dal[0, 1, 0] = d4[:, 1:].sum((0, 1))
        return None, None, None, dw, db, dtw, dtb, dal


# ----------------------------------------------------------------- fp32 tier (decoder)
class LinearF32Fn(torch.autograd.Function):
    """fp32 nn.Linear (+ exact GELU) of the alignment decoder / GatedUpdate
    (autocast disabled, alignment_head.py:340): vggt_linear_f32 forward,
    backward dX = dY W (linear_f32 on W^T), dW = dY^T X (vggt_wgrad_f32),
    db = column sums."""

    @staticmethod
    def forward(ctx, x, w, b, gelu, owner, name):
        x2 = x.reshape(-1, x.shape[-1]).float().contiguous()
        M = x2.shape[0]
        pre = torch.empty(M, w.shape[0], device=x.device)
        N.linear_f32(x2, w.detach(), b.detach() if b is not None else None, pre, N.EPI_F32)
        if gelu:
            out = torch.empty_like(pre)
            N.gelu_fwd(pre, out) if pre.shape[1] % 4 == 0 else out.copy_(torch.nn.functional.gelu(pre))
        else:
            out = pre
        ctx.save_for_backward(x2, w, pre if gelu else None)
        ctx.gelu, ctx.owner, ctx.name, ctx.has_b = gelu, owner, name, b is not None
        ctx.in_shape = x.shape
        return out.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w, pre = ctx.saved_tensors
        dy2 = dy.reshape(-1, w.shape[0]).float().contiguous()
        Nn = w.shape[0]
        if ctx.gelu:
            dpre = torch.empty_like(dy2)
            if Nn % 4 == 0:
                N.gelu_bwd(dy2, pre, dpre, None)
            else:
                xx = pre
                cdf = 0.5 * (1 + torch.erf(xx * 0.7071067811865476))
                dpre.copy_(dy2 * (cdf + xx * torch.exp(-0.5 * xx * xx) * 0.3989422804014327))
        else:
            dpre = dy2
        dw = torch.empty_like(w, dtype=torch.float32)  # written (not accumulated): every element
        db = None
        if ctx.has_b:  # weight and bias gradients in one launch
            db = torch.empty(Nn, device=dy.device)
            N.wgrad_bias_f32(dpre, x2, dw, db, False)
        else:
            N.wgrad_f32(dpre, x2, dw, False)
        dx = None
        if ctx.needs_input_grad[0]:
            wt = _wt_f32(w, ctx.owner, ctx.name)
            dx = torch.empty(x2.shape, device=dy.device)
            N.linear_f32(dpre, wt, None, dx, N.EPI_F32)
            dx = dx.view(ctx.in_shape)
        return dx, dw, db, None, None, None


def linear_f32(lin: nn.Linear, x: torch.Tensor, gelu: bool = False) -> torch.Tensor:
    return LinearF32Fn.apply(x, lin.weight, lin.bias, gelu, lin, "w")


class LayerNormF32Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        x2 = x.reshape(-1, x.shape[-1]).float().contiguous()
        out = torch.empty_like(x2)
        N.layernorm(x2, w.detach(), b.detach(), eps, out)
        ctx.save_for_backward(x2, w)
        ctx.eps, ctx.shape = eps, x.shape
        return out.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        dy2 = dy.reshape(x2.shape).float().contiguous()
        dx = torch.empty_like(x2)
        dw, db = torch.empty_like(x2[0]), torch.empty_like(x2[0])  # written by the finalize (no zero fill)
        N.layernorm_bwd(x2, w.detach(), ctx.eps, dy2, dx, False, dw, db, params_write=True)
        return dx.view(ctx.shape), dw, db, None


def layernorm_f32(ln: nn.LayerNorm, x: torch.Tensor) -> torch.Tensor:
    return LayerNormF32Fn.apply(x, ln.weight, ln.bias, ln.eps)


class HeadNormRopeF32Fn(torch.autograd.Function):
    """Per-head LayerNorm + 1-D RoPE on fp32 [M, H*D] rows (decoder q_norm/k_norm + rope1d)."""

    @staticmethod
    def forward(ctx, t, w, b, eps, H, D, mode, pos, tabs):
        t2 = t.contiguous()
        out = t2.clone()
        N.headnorm_rope_any(out, 0, H, D, w.detach() if w is not None else None,
                            b.detach() if b is not None else None, eps, mode, pos if mode else None,
                            pos.numel() if mode else 1, tabs[0] if mode else None, tabs[1] if mode else None)
        ctx.save_for_backward(t2, w)
        ctx.args = (eps, H, D, mode, pos, tabs, b is not None)
        return out

    @staticmethod
    def backward(ctx, dout):
        t2, w = ctx.saved_tensors
        eps, H, D, mode, pos, tabs, has_b = ctx.args
        grad = dout.float().contiguous().clone()
        ar = _GradArena(grad.device, [w, w if has_b else None])
        dw = ar.like(w)
        db = ar.like(w) if has_b else None
        N.headnorm_rope_bwd(t2, grad, H, H, D, w.detach() if w is not None else None, None, eps, mode,
                            pos if mode else None, pos.numel() if mode else 1, tabs[0] if mode else None,
                            tabs[1] if mode else None, dw, db)
        return grad, dw, db, None, None, None, None, None, None


class AttnSmallF32Fn(torch.autograd.Function):
    """softmax(q k^T / sqrt(D)) v for [B*nq, H*D] / [B*nk, H*D] fp32 rows (decoder cross attention)."""

    @staticmethod
    def forward(ctx, q, k, v, B, H, nq, nk, D):
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        o = torch.empty_like(q)
        N.attention_small(q, k, v, o, B, H, nq, nk, D, nq, nk, nq)
        ctx.save_for_backward(q, k, v)
        ctx.dims = (B, H, nq, nk, D)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v = ctx.saved_tensors
        B, H, nq, nk, D = ctx.dims
        do = do.float().contiguous()
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        N.attention_small_bwd(q, k, v, do, dq, dk, dv, B, H, nq, nk, D, nq, nk, nq, nq, nk)
        return dq, dk, dv, None, None, None, None, None


class ScaleFn(torch.autograd.Function):
    """out[b] = x[b] * scale[b] with x frozen (depth *= chunk_scale,
    featureAligned_vggt.py:171 in training): d scale[b] = sum(dout[b] * x[b])."""

    @staticmethod
    def forward(ctx, x, scale):
        out = x.detach().contiguous().clone()
        N.scale_(out, scale.detach())
        ctx.save_for_backward(x.detach().contiguous())
        ctx.sshape = scale.shape
        return out

    @staticmethod
    def backward(ctx, dout):
        (x,) = ctx.saved_tensors
        B = x.shape[0]
        ds = torch.empty(B, device=x.device)
        N.batch_dot_f32(dout.float().contiguous(), x, ds)
        return None, ds.view(ctx.sshape)
