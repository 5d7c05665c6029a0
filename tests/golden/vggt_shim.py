"""Test-only stand-in for the absent ``vggt`` package (facebookresearch/vggt,
unpinned; README.md:45-46) so that the reference's OWN alignment-path modules
import and run in the build container:

    aligned_vggt/heads/alignment_head.py       (AlignmentHead, :19-568)
    aligned_vggt/layers/cross_attention.py     (CrossAttention[Block], :15-131)
    aligned_vggt/models/featureAligned_vggt.py (FeatureAlignedVGGT.forward, :48-225)

It supplies only the VGGT primitives those files import -- Block, Mlp,
LayerScale, Attention, RotaryPositionEmbedding2D, PositionGetter, the pose
encoding / rotation / SE(3) helpers -- as thin nn.Modules / functions over the
build's CPU oracle (oracle/vggt_oracle.py), plus parameter-free stubs for the
aggregator, camera / DPT / track heads whose outputs the generator feeds in.
The reference's control flow, shapes, token layouts, positions, decoder,
memory mechanic and pose composition run unchanged; what the fixtures pin is
that reference-authored arithmetic (the VGGT internals stay "parity unpinned").

``bf16_mixed()`` emulates Lightning's bf16-mixed CUDA autocast
(test_featureAlignedVGGT_vkitti.yaml:86) on the CPU with a TorchFunctionMode:
F.linear / SDPA take bf16-rounded operands, accumulate in fp32 and return bf16;
F.layer_norm runs in fp32; ``torch.amp.autocast("cuda", enabled=False)``
blocks (alignment_head.py:340, featureAligned_vggt.py:104) switch the
emulation off, as they switch autocast off on the GPU.  The oracle primitives
follow the same rounding points (oracle bf16=True).

Never shipped to the GPU box (listed in .gpurunignore); used only by
tests/golden/gen_golden.py.
"""
from __future__ import annotations

import contextlib
import sys
import types

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.overrides import TorchFunctionMode

from oracle import vggt_oracle as O

_EMU = {"on": False}


def _bf16_on() -> bool:
    return _EMU["on"]


# ----------------------------------------------------------------------------
# autocast emulation
# ----------------------------------------------------------------------------
class _Bf16MixedMode(TorchFunctionMode):
    def __torch_function__(self, func, types_, args=(), kwargs=None):
        kwargs = kwargs or {}
        if not _EMU["on"]:
            return func(*args, **kwargs)
        if func is F.linear:
            x, w = args[0], args[1]
            b = args[2] if len(args) > 2 else kwargs.get("bias")
            y = O.linear(x.float(), w.float(), b.float() if b is not None else None, True)
            return y.to(torch.bfloat16)
        if func is F.scaled_dot_product_attention:
            q, k, v = args[:3]
            mask = args[3] if len(args) > 3 else kwargs.get("attn_mask")
            assert mask is None or (mask.dtype == torch.bool and bool(mask.all())), "only the all-True mask"
            assert not kwargs.get("is_causal", False) and kwargs.get("scale") is None
            return O.sdpa(q.float(), k.float(), v.float(), True).to(torch.bfloat16)
        if func is F.layer_norm:
            x, shape = args[0], args[1]
            w = args[2] if len(args) > 2 else kwargs.get("weight")
            b = args[3] if len(args) > 3 else kwargs.get("bias")
            eps = args[4] if len(args) > 4 else kwargs.get("eps", 1e-5)
            return F.layer_norm(x.float(), shape, w.float() if w is not None else None,
                                b.float() if b is not None else None, eps)
        return func(*args, **kwargs)


class _AutocastSwitch:
    """torch.amp.autocast stand-in while emulating: a CUDA autocast block sets
    the emulation state for its extent."""

    def __init__(self, device_type="cuda", dtype=None, enabled=True, cache_enabled=None):
        self.device_type, self.enabled = device_type, enabled

    def __enter__(self):
        self.prev = _EMU["on"]
        if self.device_type == "cuda":
            _EMU["on"] = self.prev and bool(self.enabled)
        return self

    def __exit__(self, *exc):
        _EMU["on"] = self.prev
        return False


@contextlib.contextmanager
def bf16_mixed(enabled: bool = True):
    if not enabled:
        yield
        return
    real = torch.amp.autocast
    torch.amp.autocast = _AutocastSwitch
    _EMU["on"] = True
    try:
        with _Bf16MixedMode():
            yield
    finally:
        _EMU["on"] = False
        torch.amp.autocast = real


# ----------------------------------------------------------------------------
# vggt.vggt.layers
# ----------------------------------------------------------------------------
def _sd(m: nn.Module):
    return dict(m.named_parameters())


class LayerScale(nn.Module):
    def __init__(self, dim, init_values=1e-5, inplace=False):
        super().__init__()
        self.gamma = nn.Parameter(init_values * torch.ones(dim))

    def forward(self, x):
        return x * self.gamma


class Mlp(nn.Module):
    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU, drop=0.0, bias=True):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features, bias=bias)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, out_features, bias=bias)
        self.drop = nn.Dropout(drop)

    def forward(self, x):
        return O.mlp(_sd(self), "", x.float(), _bf16_on())


class Attention(nn.Module):
    def __init__(self, dim, num_heads=8, qkv_bias=True, proj_bias=True, attn_drop=0.0, proj_drop=0.0,
                 norm_layer=nn.LayerNorm, qk_norm=False, fused_attn=True, rope=None):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.q_norm = norm_layer(self.head_dim) if qk_norm else nn.Identity()
        self.k_norm = norm_layer(self.head_dim) if qk_norm else nn.Identity()
        self.proj = nn.Linear(dim, dim, bias=proj_bias)
        self.rope = rope
        self.qk_norm = qk_norm

    def forward(self, x, pos=None):
        return O.attention(_sd(self), "", x.float(), self.num_heads, pos, "2d" if self.rope is not None else None,
                           self.qk_norm, _bf16_on())


class Block(nn.Module):
    def __init__(self, dim, num_heads, mlp_ratio=4.0, qkv_bias=True, proj_bias=True, ffn_bias=True, drop=0.0,
                 attn_drop=0.0, init_values=None, drop_path=0.0, act_layer=nn.GELU, norm_layer=nn.LayerNorm,
                 attn_class=Attention, ffn_layer=Mlp, qk_norm=False, fused_attn=True, rope=None):
        super().__init__()
        self.norm1 = norm_layer(dim)
        self.attn = attn_class(dim, num_heads=num_heads, qkv_bias=qkv_bias, proj_bias=proj_bias, qk_norm=qk_norm,
                               rope=rope)
        self.ls1 = LayerScale(dim, init_values=init_values) if init_values else nn.Identity()
        self.norm2 = norm_layer(dim)
        self.mlp = ffn_layer(in_features=dim, hidden_features=int(dim * mlp_ratio), act_layer=act_layer, drop=drop,
                             bias=ffn_bias)
        self.ls2 = LayerScale(dim, init_values=init_values) if init_values else nn.Identity()
        self.num_heads = num_heads
        self.qk_norm = qk_norm
        self.rope = rope

    def forward(self, x, pos=None):
        return O.block(_sd(self), "", x.float(), self.num_heads, pos, "2d" if self.rope is not None else None,
                       self.qk_norm, eps=self.norm1.eps, bf16=_bf16_on())


class RotaryPositionEmbedding2D(nn.Module):
    def __init__(self, frequency: float = 100.0, scaling_factor: float = 1.0):
        super().__init__()
        self.frequency = frequency

    def forward(self, tokens, positions):
        return O.rope2d(tokens, positions, self.frequency)


class PositionGetter:
    """(batch, h*w, 2) integer (y, x) grid, cartesian_prod(arange(h), arange(w))."""

    def __call__(self, batch_size, height, width, device):
        yy, xx = torch.meshgrid(torch.arange(height), torch.arange(width), indexing="ij")
        pos = torch.stack([yy.reshape(-1), xx.reshape(-1)], dim=-1).to(device)
        return pos.view(1, height * width, 2).expand(batch_size, -1, -1).clone()


# ----------------------------------------------------------------------------
# vggt.vggt.utils
# ----------------------------------------------------------------------------
def closed_form_inverse_se3(se3, R=None, T=None):
    return O.closed_form_inverse_se3(se3)


def pose_encoding_to_extri_intri(pose_encoding, image_size_hw=None, pose_encoding_type="absT_quaR_FoV",
                                 build_intrinsics=True):
    return O.pose_encoding_to_extri_intri(pose_encoding, tuple(int(v) for v in image_size_hw))


def extri_intri_to_pose_encoding(extrinsics, intrinsics, image_size_hw=None, pose_encoding_type="absT_quaR_FoV"):
    return O.extri_intri_to_pose_encoding(extrinsics, intrinsics, tuple(int(v) for v in image_size_hw))


def check_and_fix_inf_nan(x, name=None, hard_max=None):
    return torch.nan_to_num(x)


# ----------------------------------------------------------------------------
# stubs for the encoder side (outputs fed by the generator)
# ----------------------------------------------------------------------------
class _Feed:
    """Per-call outputs for the stub aggregator / heads (set by the generator)."""
    tokens = None       # list of 4 kept (B,S,P,2C) tensors -> layers 4/11/17/23
    pose_enc = None     # (B,S,9)
    depth = None        # (B,S,H,W,1), conf (B,S,H,W)
    depth_conf = None
    points = None       # (B,S,H,W,3), conf (B,S,H,W)
    points_conf = None


class Aggregator(nn.Module):
    def __init__(self, img_size=518, patch_size=14, embed_dim=1024, **kw):
        super().__init__()

    def forward(self, images):
        out = [None] * 24
        for i, t in zip((4, 11, 17, 23), _Feed.tokens):
            out[i] = t.clone()
        return out, 5


class CameraHead(nn.Module):
    def __init__(self, dim_in=2048, **kw):
        super().__init__()

    def forward(self, tokens_list, num_iterations=4):
        return [_Feed.pose_enc.clone()]


class DPTHead(nn.Module):
    def __init__(self, dim_in, output_dim=4, activation="inv_log", conf_activation="expp1", **kw):
        super().__init__()
        self.points = output_dim == 4

    def forward(self, tokens_list, images, patch_start_idx, frames_chunk_size=8):
        if self.points:
            return _Feed.points.clone(), _Feed.points_conf.clone()
        return _Feed.depth.clone(), _Feed.depth_conf.clone()


class TrackHead(nn.Module):
    def __init__(self, dim_in=2048, patch_size=14, **kw):
        super().__init__()


# ----------------------------------------------------------------------------
def install():
    """Register the shim as ``vggt`` in sys.modules (idempotent)."""
    if "vggt" in sys.modules and getattr(sys.modules["vggt"], "__shim__", False):
        return
    me = sys.modules[__name__]

    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        m.__path__ = []  # package
        sys.modules[name] = m
        return m

    mod("vggt", __shim__=True)
    mod("vggt.vggt")
    mod("vggt.vggt.layers", Mlp=Mlp, Block=Block, LayerScale=LayerScale, Attention=Attention)
    mod("vggt.vggt.layers.block", Block=Block)
    mod("vggt.vggt.layers.mlp", Mlp=Mlp)
    mod("vggt.vggt.layers.layer_scale", LayerScale=LayerScale)
    mod("vggt.vggt.layers.attention", Attention=Attention)
    mod("vggt.vggt.layers.rope", RotaryPositionEmbedding2D=RotaryPositionEmbedding2D, PositionGetter=PositionGetter)
    mod("vggt.vggt.utils")
    mod("vggt.vggt.utils.pose_enc", pose_encoding_to_extri_intri=pose_encoding_to_extri_intri,
        extri_intri_to_pose_encoding=extri_intri_to_pose_encoding)
    mod("vggt.vggt.utils.geometry", closed_form_inverse_se3=closed_form_inverse_se3)
    mod("vggt.vggt.utils.rotation", quat_to_mat=O.quat_to_mat, mat_to_quat=O.mat_to_quat)
    mod("vggt.vggt.models")
    mod("vggt.vggt.models.aggregator", Aggregator=Aggregator)
    mod("vggt.vggt.heads")
    mod("vggt.vggt.heads.camera_head", CameraHead=CameraHead)
    mod("vggt.vggt.heads.dpt_head", DPTHead=DPTHead)
    mod("vggt.vggt.heads.track_head", TrackHead=TrackHead)
    mod("vggt.training")
    mod("vggt.training.train_utils")
    mod("vggt.training.train_utils.general", check_and_fix_inf_nan=check_and_fix_inf_nan)
    me.installed = True
