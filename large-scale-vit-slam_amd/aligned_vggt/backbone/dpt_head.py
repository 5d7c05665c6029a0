"""VGGT DPTHead (ext ``heads/dpt_head.py`` + ``heads/utils.py``; depth head
at featureAligned_vggt.py:166, point head at :183 / pointAligned :70) on the
HIP fp32 tier (autocast disabled in the reference, featureAligned_vggt.py:104).

All activations are NHWC rows in HBM -- fp32 where a residual or an upsample
reads them, else only as the split bf16 halves (hi, lo) the next convolution
gathers; every convolution is one implicit-GEMM launch (split-bf16 on the bf16
matrix path by default, or exact-f32 MFMA, VGGT_CONV=fp32) with the surrounding
elementwise work fused into it: the positional embedding add after the 1x1
projections, the stride==kernel ConvTranspose2d as a pixel-shuffle store,
the in-place-ReLU semantics of ResidualConvUnit (relu on the conv input,
relu on the output, relu'd skip add) and the FeatureFusionBlock residual.
Module names (norm, projects, resize_layers, scratch.layer*_rn,
scratch.refinenet*, scratch.output_conv*) follow the reference checkpoint.
All frames of a chunk are processed at once (288 GB of HBM; the reference
chunks 8 frames at a time only to bound memory -- the arithmetic is identical).
"""
from __future__ import annotations

import os

from typing import List, Optional, Tuple

import torch
import torch.nn as nn

from .. import _native as N
from ..runtime import Workspace, yield_point


def _make_sincos(embed_dim: int, pos: torch.Tensor, omega_0: float = 100) -> torch.Tensor:
    omega = torch.arange(embed_dim // 2, dtype=torch.double)
    omega /= embed_dim / 2.0
    omega = 1.0 / omega_0 ** omega
    out = torch.einsum("m,d->md", pos.reshape(-1), omega)
    return torch.cat([torch.sin(out), torch.cos(out)], dim=1).float()


def _uv_grid(width: int, height: int, aspect_ratio: float) -> torch.Tensor:
    diag = (aspect_ratio ** 2 + 1.0) ** 0.5
    span_x, span_y = aspect_ratio / diag, 1.0 / diag
    xs = torch.linspace(-span_x * (width - 1) / width, span_x * (width - 1) / width, steps=width)
    ys = torch.linspace(-span_y * (height - 1) / height, span_y * (height - 1) / height, steps=height)
    uu, vv = torch.meshgrid(xs, ys, indexing="xy")
    return torch.stack((uu, vv), dim=-1)


def pos_table(C: int, h: int, w: int, W_img: int, H_img: int, ratio: float = 0.1) -> torch.Tensor:
    """DPTHead._apply_pos_embed as an NHWC table [h*w, C] (host-side constant)."""
    grid = _uv_grid(w, h, W_img / H_img).reshape(-1, 2)
    emb = torch.cat([_make_sincos(C // 2, grid[:, 0]), _make_sincos(C // 2, grid[:, 1])], dim=-1)
    return (emb * ratio).contiguous()


def pos_table_sep(C: int, h: int, w: int, W_img: int, H_img: int, ratio: float = 0.1) -> torch.Tensor:
    """pos_table in separable form [w + h, C/2]: the first C/2 channels of the
    embedding depend only on the pixel's u (x), the last C/2 only on v (y), so
    rows 0..w-1 hold the x part and rows w..w+h-1 the y part -- the same
    floats as pos_table's entries."""
    grid = _uv_grid(w, h, W_img / H_img)  # (h, w, 2)
    u = _make_sincos(C // 2, grid[0, :, 0])  # (w, C/2)
    v = _make_sincos(C // 2, grid[:, 0, 1])  # (h, C/2)
    return (torch.cat([u, v], 0) * ratio).contiguous()


class ResidualConvUnit(nn.Module):
    def __init__(self, features, activation=None, bn=False, groups=1):
        super().__init__()
        self.bn = bn
        self.groups = groups
        self.conv1 = nn.Conv2d(features, features, kernel_size=3, stride=1, padding=1, bias=True, groups=groups)
        self.conv2 = nn.Conv2d(features, features, kernel_size=3, stride=1, padding=1, bias=True, groups=groups)
        self.norm1 = None
        self.norm2 = None
        self.activation = activation


class FeatureFusionBlock(nn.Module):
    def __init__(self, features, activation=None, deconv=False, bn=False, expand=False, align_corners=True,
                 size=None, has_residual=True, groups=1):
        super().__init__()
        self.deconv = deconv
        self.align_corners = align_corners
        self.groups = groups
        self.expand = expand
        out_features = features // 2 if expand else features
        self.out_conv = nn.Conv2d(features, out_features, kernel_size=1, stride=1, padding=0, bias=True, groups=groups)
        if has_residual:
            self.resConfUnit1 = ResidualConvUnit(features, activation, bn, groups=groups)
        self.has_residual = has_residual
        self.resConfUnit2 = ResidualConvUnit(features, activation, bn, groups=groups)
        self.size = size


def _fusion(features: int, has_residual: bool = True) -> FeatureFusionBlock:
    return FeatureFusionBlock(features, nn.ReLU(inplace=True), deconv=False, bn=False, expand=False,
                              align_corners=True, size=None, has_residual=has_residual)


def _scratch(in_shape, out_shape) -> nn.Module:
    s = nn.Module()
    s.layer1_rn = nn.Conv2d(in_shape[0], out_shape, kernel_size=3, stride=1, padding=1, bias=False)
    s.layer2_rn = nn.Conv2d(in_shape[1], out_shape, kernel_size=3, stride=1, padding=1, bias=False)
    s.layer3_rn = nn.Conv2d(in_shape[2], out_shape, kernel_size=3, stride=1, padding=1, bias=False)
    s.layer4_rn = nn.Conv2d(in_shape[3], out_shape, kernel_size=3, stride=1, padding=1, bias=False)
    return s


# DPT convolutions: "bf16x3pre" (default: split-bf16 operands on the bf16 matrix
# path, the activation split once by its producer -- conv epilogue, upsample or a
# split pass -- and gathered by LDS-DMA), "bf16x3" (the same products with the
# split done in the conv's register-staged gather; bitwise equal) or "fp32"
# (exact f32 MFMA).
CONV_PRECISION = os.environ.get("VGGT_CONV", "bf16x3pre")

# FeatureFusionBlock: run the 1x1 out_conv before the bilinear resize (the two
# commute; see DPTHead._fuse); VGGT_DPT_REORDER=0 keeps the reference's order.
REORDER_OUT_CONV = os.environ.get("VGGT_DPT_REORDER", "1") != "0"
# final upsample: the positional table in separable [w + h, C/2] form (bitwise the
# same values; VGGT_DPT_SEP_POS=0 reads the full [h*w, C] table per frame)
SEPARABLE_POS = os.environ.get("VGGT_DPT_SEP_POS", "1") != "0"
# output_conv1 -> resize -> + pos -> output_conv2[0] as one fused launch
# (vggt_conv2d_upsample_bf16x3: the resized 518^2 map is never written);
# VGGT_DPT_FUSE_UP=0 runs the separate upsample + conv
FUSE_UPSAMPLE_CONV = os.environ.get("VGGT_DPT_FUSE_UP", "1") != "0"

# The convolutions address their operands with 32-bit byte offsets
# (conv.hip: VGGT_ERR_SHAPE at 2 GiB); a forward whose widest map reaches this
# runs in groups of frames.  Module-level so tests can lower it.
MAP_BYTES_LIMIT = 1 << 31


def _pre() -> bool:
    return CONV_PRECISION == "bf16x3pre"


def _pack_conv(conv: nn.Module, transpose: bool = False):
    """Conv2d [co,ci,kh,kw] -> [roundup(co,128), kh*kw*ci]; ConvTranspose2d
    [ci,co,k,k] -> [roundup(k*k*co,128), ci] with column (ky*k+kx)*co + c.
    Returns (w_f32, bias, w_hi, w_lo): the split bf16 halves are made once."""
    w = conv.weight
    key = (w.data_ptr(), w._version, transpose)
    c = conv.__dict__.get("_mi355x_conv")
    if c is not None and c[0] == key:
        return c[1:]
    with torch.no_grad():
        if transpose:
            ci, co, kh, kw = w.shape
            wp = w.detach().float().permute(2, 3, 1, 0).reshape(kh * kw * co, ci)
        else:
            co, ci, kh, kw = w.shape
            wp = w.detach().float().permute(0, 2, 3, 1).reshape(co, kh * kw * ci)
        rows = (wp.shape[0] + 127) // 128 * 128  # (the f32 kernel needs 64, the split one 128)
        if rows != wp.shape[0]:
            wp = torch.cat([wp, wp.new_zeros(rows - wp.shape[0], wp.shape[1])], 0)
        wp = wp.contiguous()
        b = conv.bias.detach().float().contiguous() if conv.bias is not None else None
        w_hi, w_lo = N.split_bf16x2(wp) if wp.is_cuda else (None, None)
        c = (key, wp, b, w_hi, w_lo)
    conv.__dict__["_mi355x_conv"] = c
    return c[1:]


class _Map:
    """An NHWC activation: rows [n*h*w, c] fp32 (``t``) and/or its split bf16
    halves ``sp`` = (hi, lo) of relu(x) (``sp_relu``) or of x -- the form the
    next convolution gathers."""

    __slots__ = ("t", "n", "h", "w", "c", "sp", "sp_relu")

    def __init__(self, t, n, h, w, c, sp=None, sp_relu=False):
        self.t, self.n, self.h, self.w, self.c = t, n, h, w, c
        self.sp, self.sp_relu = sp, sp_relu


def _split_of(x: _Map, relu: bool):
    if x.sp is not None and x.sp_relu == relu:
        return x.sp
    assert x.t is not None, "DPT map has neither its f32 rows nor the split this conv needs"
    return N.split_act_bf16x2(x.t, relu)


def _outputs(rows: int, co: int, dev, f32: bool, split):
    """(y, y_split) buffers for a producer: split None / "plain" / "relu"."""
    if not _pre():
        f32, split = True, None
    y = torch.empty(rows, co, device=dev) if f32 else None
    ys = None
    if split is not None:
        ys = (torch.empty(rows, co, device=dev, dtype=torch.bfloat16),
              torch.empty(rows, co, device=dev, dtype=torch.bfloat16))
    return y, ys


def _conv_call(x: _Map, packed, co, kh, kw, stride, pad, y, ys, split_relu, relu_in=False, relu_out=False, res1=None,
               res1_relu=False, res2=None, pos=None, shuffle=0):
    wp, b, w_hi, w_lo = packed
    n, h, w_, c = x.n, x.h, x.w, x.c
    if CONV_PRECISION == "fp32":
        N.conv2d_f32(x.t, n, h, w_, c, wp, b, co, kh, kw, stride, pad, y, relu_in, relu_out, res1, res1_relu, res2,
                     pos, shuffle=shuffle)
    elif _pre():
        xh, xl = _split_of(x, relu_in)
        N.conv2d_bf16x3_pre(xh, xl, n, h, w_, c, w_hi, w_lo, b, co, kh, kw, stride, pad, y, relu_out, res1, res1_relu,
                            res2, pos, shuffle=shuffle, y_split=ys, split_relu=split_relu)
    else:
        N.conv2d_bf16x3(x.t, n, h, w_, c, w_hi, w_lo, b, co, kh, kw, stride, pad, y, relu_in, relu_out, res1,
                        res1_relu, res2, pos, shuffle=shuffle)


def _conv(x: _Map, conv: nn.Conv2d, stride=1, pad=None, relu_in=False, relu_out=False, res1: _Map = None,
          res1_relu=False, res2: _Map = None, pos=None, f32=True, split=None) -> _Map:
    """split: the consumer's gather form to write besides (or, f32=False, instead
    of) the f32 rows -- None, "plain" or "relu" (the consumer's relu_in)."""
    yield_point(fine=True)
    packed = _pack_conv(conv)
    co, _, kh, kw = conv.weight.shape
    pad = conv.padding[0] if pad is None else pad
    ho = (x.h + 2 * pad - kh) // stride + 1
    wo = (x.w + 2 * pad - kw) // stride + 1
    y, ys = _outputs(x.n * ho * wo, co, x.t.device if x.t is not None else x.sp[0].device, f32, split)
    _conv_call(x, packed, co, kh, kw, stride, pad, y, ys, split == "relu", relu_in, relu_out,
               res1.t if res1 else None, res1_relu, res2.t if res2 else None, pos)
    return _Map(y, x.n, ho, wo, co, ys, split == "relu")


def _convT(x: _Map, conv: nn.ConvTranspose2d, f32=True, split=None) -> _Map:
    yield_point(fine=True)
    packed = _pack_conv(conv, transpose=True)
    ci, co, k, _ = conv.weight.shape
    assert conv.stride[0] == k and conv.padding[0] == 0
    y, ys = _outputs(x.n * x.h * k * x.w * k, co, x.t.device if x.t is not None else x.sp[0].device, f32, split)
    _conv_call(x, packed, co, 1, 1, 1, 0, y, ys, split == "relu", shuffle=k)
    return _Map(y, x.n, x.h * k, x.w * k, co, ys, split == "relu")


def _upsample(x: _Map, ho: int, wo: int, pos=None, f32=True, split=None, pos_sep=None) -> _Map:
    y, ys = _outputs(x.n * ho * wo, x.c, x.t.device, f32, split)
    if pos_sep is not None and ys is not None:
        N.upsample_bilinear_split_sep(x.t, x.n, x.h, x.w, x.c, y, ho, wo, pos_sep, y_split=ys,
                                      split_relu=split == "relu")
    elif ys is None:
        N.upsample_bilinear_f32(x.t, x.n, x.h, x.w, x.c, y, ho, wo, pos)
    else:
        N.upsample_bilinear_split(x.t, x.n, x.h, x.w, x.c, y, ho, wo, pos, y_split=ys, split_relu=split == "relu")
    return _Map(y, x.n, ho, wo, x.c, ys, split == "relu")


def _conv_upsample(x: _Map, conv: nn.Conv2d, ho: int, wo: int, pos_sep, relu_out=False, f32=True, split=None) -> _Map:
    """conv3x3(resize(x) + pos) as one launch (vggt_conv2d_upsample_bf16x3): x's f32 rows
    at the source resolution, the resized map never materialised."""
    yield_point(fine=True)
    _, b, w_hi, w_lo = _pack_conv(conv)
    co = conv.weight.shape[0]
    y, ys = _outputs(x.n * ho * wo, co, x.t.device, f32, split)
    N.conv2d_upsample_bf16x3(x.t, x.n, x.h, x.w, x.c, pos_sep, ho, wo, w_hi, w_lo, b, co, y, relu_out=relu_out,
                             y_split=ys, split_relu=split == "relu")
    return _Map(y, x.n, ho, wo, co, ys, split == "relu")


class DPTHead(nn.Module):
    def __init__(self, dim_in: int, patch_size: int = 14, output_dim: int = 4, activation: str = "inv_log",
                 conf_activation: str = "expp1", features: int = 256, out_channels=(256, 512, 1024, 1024),
                 intermediate_layer_idx=(4, 11, 17, 23), pos_embed: bool = True, feature_only: bool = False,
                 down_ratio: int = 1):
        super().__init__()
        if feature_only or down_ratio != 1:
            raise NotImplementedError("feature_only / down_ratio are not used by any reference model")
        if activation not in ("exp", "inv_log") or conf_activation != "expp1":
            raise NotImplementedError(f"activation {activation}/{conf_activation}")
        self.patch_size = patch_size
        self.activation = activation
        self.conf_activation = conf_activation
        self.pos_embed = pos_embed
        self.feature_only = feature_only
        self.down_ratio = down_ratio
        self.intermediate_layer_idx = list(intermediate_layer_idx)
        self.output_dim = output_dim
        out_channels = list(out_channels)
        self.out_channels = out_channels
        self.norm = nn.LayerNorm(dim_in)
        self.projects = nn.ModuleList([nn.Conv2d(dim_in, oc, kernel_size=1, stride=1, padding=0) for oc in out_channels])
        self.resize_layers = nn.ModuleList([
            nn.ConvTranspose2d(out_channels[0], out_channels[0], kernel_size=4, stride=4, padding=0),
            nn.ConvTranspose2d(out_channels[1], out_channels[1], kernel_size=2, stride=2, padding=0),
            nn.Identity(),
            nn.Conv2d(out_channels[3], out_channels[3], kernel_size=3, stride=2, padding=1)])
        self.scratch = _scratch(out_channels, features)
        self.scratch.stem_transpose = None
        self.scratch.refinenet1 = _fusion(features)
        self.scratch.refinenet2 = _fusion(features)
        self.scratch.refinenet3 = _fusion(features)
        self.scratch.refinenet4 = _fusion(features, has_residual=False)
        self.scratch.output_conv1 = nn.Conv2d(features, features // 2, kernel_size=3, stride=1, padding=1)
        self.scratch.output_conv2 = nn.Sequential(
            nn.Conv2d(features // 2, 32, kernel_size=3, stride=1, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(32, output_dim, kernel_size=1, stride=1, padding=0))

    def _pos(self, C: int, h: int, w: int, W_img: int, H_img: int, device, sep: bool = False) -> torch.Tensor:
        cache = self.__dict__.setdefault("_mi355x_pos", {})
        key = (C, h, w, W_img, H_img, str(device), sep)
        if key not in cache:
            cache[key] = (pos_table_sep if sep else pos_table)(C, h, w, W_img, H_img).to(device)
        return cache[key]

    def _fuse(self, blk: FeatureFusionBlock, x0: _Map, x1: Optional[_Map], size, f32=True, split=None) -> _Map:
        """x1 (and x0 when x1 is None) arrive with their f32 rows and the ReLU'd split;
        (f32, split) select the output forms for the consumer."""
        out = x0
        if x1 is not None:
            t = _conv(x1, blk.resConfUnit1.conv1, relu_in=True, relu_out=True, f32=False, split="plain")
            out = _conv(t, blk.resConfUnit1.conv2, res1=x1, res1_relu=True, res2=x0, split="relu")
        t = _conv(out, blk.resConfUnit2.conv1, relu_in=True, relu_out=True, f32=False, split="plain")
        ho, wo = size if size is not None else (out.h * 2, out.w * 2)
        if REORDER_OUT_CONV:
            # out_conv (1x1) before the bilinear resize instead of after: both are
            # linear, the resize acts per channel with weights summing to 1
            # (align_corners=True), so conv1x1(resize(x)) == resize(conv1x1(x)) in
            # exact arithmetic (bias included) -- at the input resolution the 1x1
            # conv touches 1/4 of the pixels (refinenet1: 148^2 instead of 296^2)
            out = _conv(t, blk.resConfUnit2.conv2, res1=out, res1_relu=True, f32=False, split="plain")
            y = _conv(out, blk.out_conv)
            return _upsample(y, ho, wo, f32=f32, split=split)
        out = _conv(t, blk.resConfUnit2.conv2, res1=out, res1_relu=True)
        up = _upsample(out, ho, wo, f32=False, split="plain")
        return _conv(up, blk.out_conv, f32=f32, split=split)

    @torch.no_grad()
    def forward(self, aggregated_tokens_list: List[torch.Tensor], images: torch.Tensor, patch_start_idx: int,
                frames_chunk_size: int = 8, _scale: Optional[torch.Tensor] = None):
        """-> (preds (B,S,H,W,output_dim-1), conf (B,S,H,W)).  ``_scale`` (B,)
        optionally multiplies preds (the chunk-scale fusion of
        featureAligned_vggt.py:171)."""
        B, S, _, H, W = images.shape
        if images.device.type != "cuda":
            raise RuntimeError("DPTHead: the MI355X hot path runs on HIP devices only (no CPU fallback)")
        per_frame = H * W * 128 * 2  # widest activation: 128 channels at full resolution, bf16 halves
        if B * S > 1 and B * S * per_frame >= MAP_BYTES_LIMIT:
            # the widest map would pass the convolutions' 32-bit offsets (a long
            # chunk, or a batch of chunks from ChunkPipeline's grouped encode):
            # groups of frames instead -- every DPT op is per frame, so the
            # results are identical (the reference itself runs frames_chunk_size
            # frames at a time)
            fpg = max(1, (MAP_BYTES_LIMIT - 1) // per_frame)
            tl = [t.reshape(1, B * S, *t.shape[2:]) for t in aggregated_tokens_list]
            im = images.reshape(1, B * S, *images.shape[2:])
            fs = _scale.float().reshape(B, 1).expand(B, S).reshape(1, B * S) if _scale is not None else None
            outs = [self._forward_frames([t[:, f0:f0 + fpg] for t in tl], im[:, f0:f0 + fpg], patch_start_idx,
                                         fs[:, f0:f0 + fpg] if fs is not None else None)
                    for f0 in range(0, B * S, fpg)]
            preds = torch.cat([o[0] for o in outs], 1)
            conf = torch.cat([o[1] for o in outs], 1)
            return preds.view(B, S, *preds.shape[2:]), conf.view(B, S, *conf.shape[2:])
        return self._forward_frames(aggregated_tokens_list, images, patch_start_idx, _scale)

    def _forward_frames(self, aggregated_tokens_list: List[torch.Tensor], images: torch.Tensor, patch_start_idx: int,
                        _scale: Optional[torch.Tensor]):
        """``_scale``: (B,) per chunk or (B, S) per frame."""
        B, S, _, H, W = images.shape
        dev = images.device
        ph, pw = H // self.patch_size, W // self.patch_size
        F_ = B * S
        hw = ph * pw
        ws = Workspace.get(dev)
        feats = []
        # yield points (the multi-GPU pipeline's gated encode pauses there while an
        # alignment runs): every reassemble layer, fusion block and the output stage
        for li, layer_idx in enumerate(self.intermediate_layer_idx):
            yield_point()
            tk = aggregated_tokens_list[layer_idx]
            P, Cin = tk.shape[2], tk.shape[3]
            xl = ws.buf("dpt_ln", F_ * hw, Cin)
            N.layernorm_grouped(tk.reshape(F_ * P, Cin), self.norm.weight, self.norm.bias, self.norm.eps, xl, F_ * hw,
                                Cin, hw, P, patch_start_idx, hw, 0)
            oc = self.out_channels[li]
            pos = self._pos(oc, ph, pw, W, H, dev) if self.pos_embed else None
            # every producer below writes the form its consumer gathers (f32 rows only
            # where a residual / upsample reads them)
            x = _conv(_Map(xl, F_, ph, pw, Cin), self.projects[li], pos=pos, f32=False, split="plain")
            if li == 0 or li == 1:
                x = _convT(x, self.resize_layers[li], f32=False, split="plain")
            elif li == 3:
                x = _conv(x, self.resize_layers[3], stride=2, pad=1, f32=False, split="plain")
            feats.append(x)
        sc = self.scratch
        l1 = _conv(feats[0], sc.layer1_rn, split="relu")
        l2 = _conv(feats[1], sc.layer2_rn, split="relu")
        l3 = _conv(feats[2], sc.layer3_rn, split="relu")
        l4 = _conv(feats[3], sc.layer4_rn, split="relu")
        yield_point()
        out = self._fuse(sc.refinenet4, l4, None, (l3.h, l3.w))
        yield_point()
        out = self._fuse(sc.refinenet3, out, l3, (l2.h, l2.w))
        yield_point()
        out = self._fuse(sc.refinenet2, out, l2, (l1.h, l1.w))
        yield_point()
        out = self._fuse(sc.refinenet1, out, l1, None, f32=False, split="plain")
        yield_point()
        out = _conv(out, sc.output_conv1)
        Ho, Wo = int(ph * self.patch_size / self.down_ratio), int(pw * self.patch_size / self.down_ratio)
        c2 = sc.output_conv2[0]
        if (FUSE_UPSAMPLE_CONV and _pre() and self.pos_embed and out.c % 32 == 0 and c2.weight.shape[0] <= 32
                and c2.kernel_size == (3, 3) and c2.padding == (1, 1) and c2.stride == (1, 1)):
            out = _conv_upsample(out, c2, Ho, Wo, self._pos(out.c, Ho, Wo, W, H, dev, sep=True), relu_out=True,
                                 f32=False, split="plain")
        else:
            if self.pos_embed and _pre() and SEPARABLE_POS and out.c % 8 == 0:
                out = _upsample(out, Ho, Wo, f32=False, split="plain",
                                pos_sep=self._pos(out.c, Ho, Wo, W, H, dev, sep=True))
            else:
                out = _upsample(out, Ho, Wo, self._pos(out.c, Ho, Wo, W, H, dev) if self.pos_embed else None,
                                f32=False, split="plain")
            out = _conv(out, c2, relu_out=True, f32=False, split="plain")
        out = _conv(out, sc.output_conv2[2])
        ncl = self.output_dim
        npix = F_ * Ho * Wo
        preds = torch.empty(B, S, Ho, Wo, ncl - 1, device=dev)
        conf = torch.empty(B, S, Ho, Wo, device=dev)
        scale = _scale.float().reshape(B, -1).expand(B, S).contiguous().view(-1) if _scale is not None else None
        N.dpt_activate(out.t, npix, Ho * Wo, ncl, 0 if self.activation == "exp" else 1, scale, preds, conf)
        return preds, conf
