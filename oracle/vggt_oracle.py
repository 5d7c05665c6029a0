"""CPU oracle for the per-chunk VGGT forward + feature-alignment head.

TEST INFRASTRUCTURE ONLY.  Nothing in the product (``large-scale-vit-slam_amd``)
imports this module; only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may use it, and only as the checker / the
timed CPU baseline, never as the thing measured or shipped.

This is a plain functional fp32 PyTorch-on-CPU restatement of the reference
path, operating on a state dict whose keys are the reference module-tree names
(``aggregator.*``, ``camera_head.*``, ``depth_head.*``, ``alignment_head.*``).

Two numeric tiers (SURVEY.md §7 hard part 3):
  * ``bf16=False``: plain fp32 everywhere (what the reference computes on CPU,
    where ``torch.amp.autocast("cuda")`` is inert) -- the CPU baseline.
  * ``bf16=True``: emulates the reference under Lightning ``bf16-mixed``
    autocast (test_featureAlignedVGGT_vkitti.yaml:86): Linear/Conv/SDPA inputs
    (and Linear bias) rounded to bf16 with fp32 accumulation and bf16 outputs,
    LayerNorm in fp32, fp32 residual stream, LayerScale promoting to fp32.
    The camera/depth/point heads and the alignment decoder run with autocast
    disabled in the reference (featureAligned_vggt.py:104, alignment_head.py:340),
    so they stay fp32 in both tiers.

Parity status
-------------
Reference-authored arithmetic (alignment head, cross attention, 1-D RoPE, gated
update, pose/Sim(3) glue, chunking) follows the files cited per function and is
pinned by ``tests/golden`` fixtures produced by running the reference's own
importable modules / AST-extracted functions in the build container.
The VGGT backbone and heads live in the unvendored, unpinned third-party
``facebookresearch/vggt`` package (README.md:45-46); they are restated from its
public source and are **parity unpinned** except for the DINOv2 stage, which is
pinned against the in-container ``transformers`` Dinov2WithRegistersModel.
Every unpinned assumption is listed in SPEC_ASSUMPTIONS.md.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor
SD = Dict[str, Tensor]

RESNET_MEAN = (0.485, 0.456, 0.406)
RESNET_STD = (0.229, 0.224, 0.225)


# ----------------------------------------------------------------------------
# numeric helpers (autocast emulation)
# ----------------------------------------------------------------------------
def _r(x: Tensor, bf16: bool) -> Tensor:
    """Round to bf16 and back (the autocast cast points)."""
    return x.to(torch.bfloat16).to(torch.float32) if bf16 else x


def linear(x: Tensor, w: Tensor, b: Optional[Tensor], bf16: bool) -> Tensor:
    """nn.Linear; under autocast inputs, weight and bias are cast to bf16,
    accumulation is fp32, output bf16."""
    y = _r(x, bf16) @ _r(w, bf16).t()
    if b is not None:
        y = y + _r(b, bf16)
    return _r(y, bf16)


def layer_norm(x: Tensor, w: Optional[Tensor], b: Optional[Tensor], eps: float) -> Tensor:
    # autocast runs layer_norm in fp32
    return F.layer_norm(x.float(), (x.shape[-1],), w, b, eps)


def gelu(x: Tensor, bf16: bool) -> Tensor:
    # nn.GELU (exact erf); on a bf16 tensor torch computes in fp32, rounds output
    return _r(F.gelu(x), bf16)


def sdpa(q: Tensor, k: Tensor, v: Tensor, bf16: bool, max_score_bytes: int = 1 << 31) -> Tensor:
    """softmax(q k^T / sqrt(d)) v over (..., N, D); fp32 softmax.  Rows are
    independent, so a score matrix larger than max_score_bytes (the global
    attention of a 16 x 518^2 chunk: 16 x 21,984^2 fp32 = 31 GB) is formed in
    blocks of query rows."""
    q, k, v = _r(q, bf16), _r(k, bf16), _r(v, bf16)
    nq, nk = q.shape[-2], k.shape[-2]
    per_row = 4 * nk * max(1, q.numel() // (nq * q.shape[-1]))
    step = max(1, min(nq, max_score_bytes // max(1, per_row)))
    outs = []
    for r0 in range(0, nq, step):
        s = (q[..., r0:r0 + step, :] @ k.transpose(-1, -2)) * (q.shape[-1] ** -0.5)
        p = torch.softmax(s, dim=-1)
        outs.append(p @ v)
        del s, p
    return _r(outs[0] if len(outs) == 1 else torch.cat(outs, dim=-2), bf16)


# ----------------------------------------------------------------------------
# RoPE (vggt layers/rope.py, restated; 1-D variant = aligned_vggt/layers/rope.py)
# ----------------------------------------------------------------------------
def rope_cos_sin(dim: int, seq_len: int, freq: float, dtype=torch.float32) -> Tuple[Tensor, Tensor]:
    """aligned_vggt/layers/rope.py:23-44 (same as VGGT RoPE2D's cache)."""
    exponents = torch.arange(0, dim, 2).float() / dim
    inv_freq = 1.0 / (freq ** exponents)
    positions = torch.arange(seq_len, dtype=inv_freq.dtype)
    angles = torch.einsum("i,j->ij", positions, inv_freq).to(dtype)
    angles = torch.cat((angles, angles), dim=-1)
    return angles.cos().to(dtype), angles.sin().to(dtype)


def _rotate_half(x: Tensor) -> Tensor:
    d = x.shape[-1]
    return torch.cat((-x[..., d // 2:], x[..., : d // 2]), dim=-1)


def _rope_apply(x: Tensor, pos: Tensor, cos: Tensor, sin: Tensor) -> Tensor:
    """rope.py:70-89: tokens (B,H,N,D), positions (B,N) -> x*cos + rot(x)*sin."""
    c = F.embedding(pos, cos)[:, None]
    s = F.embedding(pos, sin)[:, None]
    return x * c + _rotate_half(x) * s


def rope1d(x: Tensor, pos: Tensor, freq: float = 100.0) -> Tensor:
    """aligned_vggt/layers/rope.py:91-126."""
    cos, sin = rope_cos_sin(x.shape[-1], int(pos.max()) + 1, freq, x.dtype)
    return _rope_apply(x, pos, cos, sin)


def rope2d(x: Tensor, pos: Tensor, freq: float = 100.0) -> Tensor:
    """VGGT RotaryPositionEmbedding2D (ext, unpinned): first half of head_dim
    rotated by the y position, second half by x (SPEC_ASSUMPTIONS.md A3)."""
    half = x.shape[-1] // 2
    cos, sin = rope_cos_sin(half, int(pos.max()) + 1, freq, x.dtype)
    v, h = x[..., :half], x[..., half:]
    return torch.cat((_rope_apply(v, pos[..., 0], cos, sin), _rope_apply(h, pos[..., 1], cos, sin)), dim=-1)


def position_grid(n: int, h: int, w: int, n_special: int) -> Tensor:
    """VGGT PositionGetter (cartesian_prod(y, x)) + 1, zeros for the special
    tokens (aggregator; alignment_head.py:301-310)."""
    yy, xx = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    pos = torch.stack([yy.reshape(-1), xx.reshape(-1)], dim=-1) + 1
    pos = torch.cat([torch.zeros(n_special, 2, dtype=pos.dtype), pos], dim=0)
    return pos.unsqueeze(0).expand(n, -1, -1).contiguous()


# ----------------------------------------------------------------------------
# transformer blocks
# ----------------------------------------------------------------------------
def attention(sd: SD, p: str, x: Tensor, num_heads: int, pos: Optional[Tensor], rope: Optional[str],
              qk_norm: bool, bf16: bool) -> Tensor:
    """VGGT layers/attention.py Attention (ext): fused qkv, optional per-head
    LayerNorm QK-norm (eps 1e-5), optional RoPE-2D, SDPA, proj."""
    B, N, C = x.shape
    hd = C // num_heads
    qkv = linear(x, sd[p + "qkv.weight"], sd.get(p + "qkv.bias"), bf16)
    qkv = qkv.reshape(B, N, 3, num_heads, hd).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    if qk_norm:
        q = layer_norm(q, sd[p + "q_norm.weight"], sd[p + "q_norm.bias"], 1e-5)
        k = layer_norm(k, sd[p + "k_norm.weight"], sd[p + "k_norm.bias"], 1e-5)
    if rope == "2d":
        q = rope2d(q, pos)
        k = rope2d(k, pos)
    o = sdpa(q, k, v, bf16)
    o = o.transpose(1, 2).reshape(B, N, C)
    return linear(o, sd[p + "proj.weight"], sd.get(p + "proj.bias"), bf16)


def mlp(sd: SD, p: str, x: Tensor, bf16: bool) -> Tensor:
    """VGGT layers/mlp.py Mlp: fc1 -> GELU -> fc2."""
    h = linear(x, sd[p + "fc1.weight"], sd[p + "fc1.bias"], bf16)
    h = gelu(h, bf16)
    return linear(h, sd[p + "fc2.weight"], sd[p + "fc2.bias"], bf16)


def _ls(sd: SD, key: str, y: Tensor) -> Tensor:
    g = sd.get(key)
    return y * g if g is not None else y


def block(sd: SD, p: str, x: Tensor, num_heads: int, pos: Optional[Tensor] = None, rope: Optional[str] = None,
          qk_norm: bool = False, eps: float = 1e-5, bf16: bool = False) -> Tensor:
    """VGGT layers/block.py Block: pre-LN, LayerScale, residual (fp32 stream)."""
    y = layer_norm(x, sd[p + "norm1.weight"], sd[p + "norm1.bias"], eps)
    x = x + _ls(sd, p + "ls1.gamma", attention(sd, p + "attn.", y, num_heads, pos, rope, qk_norm, bf16))
    y = layer_norm(x, sd[p + "norm2.weight"], sd[p + "norm2.bias"], eps)
    x = x + _ls(sd, p + "ls2.gamma", mlp(sd, p + "mlp.", y, bf16))
    return x


def cross_attention(sd: SD, p: str, x: Tensor, y: Tensor, num_heads: int, pos_q: Tensor, pos_k: Tensor,
                    bf16: bool) -> Tensor:
    """aligned_vggt/layers/cross_attention.py:47-78 (q from x, k/v from y,
    per-head LN QK-norm, 1-D RoPE; the all-True mask of :66-67 is a no-op)."""
    B, N, C = x.shape
    M = y.shape[1]
    hd = C // num_heads
    q = linear(x, sd[p + "q.weight"], sd[p + "q.bias"], bf16).reshape(B, N, num_heads, hd).transpose(1, 2)
    k = linear(y, sd[p + "k.weight"], sd[p + "k.bias"], bf16).reshape(B, M, num_heads, hd).transpose(1, 2)
    v = linear(y, sd[p + "v.weight"], sd[p + "v.bias"], bf16).reshape(B, M, num_heads, hd).transpose(1, 2)
    q = layer_norm(q, sd[p + "q_norm.weight"], sd[p + "q_norm.bias"], 1e-5)
    k = layer_norm(k, sd[p + "k_norm.weight"], sd[p + "k_norm.bias"], 1e-5)
    q = rope1d(q, pos_q)
    k = rope1d(k, pos_k)
    o = sdpa(q, k, v, bf16)
    o = o.transpose(1, 2).reshape(B, N, C)
    return linear(o, sd[p + "proj.weight"], sd[p + "proj.bias"], bf16)


def cross_attention_block(sd: SD, p: str, x: Tensor, y: Tensor, num_heads: int, pos: Tuple[Tensor, Tensor],
                          bf16: bool) -> Tensor:
    """cross_attention.py:126-131: x += ls1(attn(norm1 x, norm3 y)); x += ls2(mlp(norm2 x))."""
    xn = layer_norm(x, sd[p + "norm1.weight"], sd[p + "norm1.bias"], 1e-5)
    yn = layer_norm(y, sd[p + "norm3.weight"], sd[p + "norm3.bias"], 1e-5)
    x = x + _ls(sd, p + "ls1.gamma", cross_attention(sd, p + "attn.", xn, yn, num_heads, pos[0], pos[1], bf16))
    xn = layer_norm(x, sd[p + "norm2.weight"], sd[p + "norm2.bias"], 1e-5)
    x = x + _ls(sd, p + "ls2.gamma", mlp(sd, p + "mlp.", xn, bf16))
    return x


def slice_expand_and_flatten(tok: Tensor, B: int, S: int) -> Tensor:
    """alignment_head.py:543-568 (returns (B,S,X,C); the aggregator flattens)."""
    query = tok[:, 0:1].expand(B, 1, *tok.shape[2:])
    others = tok[:, 1:].expand(B, S - 1, *tok.shape[2:])
    return torch.cat([query, others], dim=1)


# ----------------------------------------------------------------------------
# aggregator (VGGT models/aggregator.py, ext) incl. DINOv2 ViT-L/14-reg
# ----------------------------------------------------------------------------
def interpolated_pos_embed(pos_embed: Tensor, h: int, w: int) -> Tensor:
    """DINOv2 interpolate_pos_encoding with offset 0 / antialias (ext)."""
    N = pos_embed.shape[1] - 1
    M = int(math.sqrt(N))
    if h * w == N and h == w:
        return pos_embed
    cls_pe = pos_embed[:, :1].float()
    pe = pos_embed[:, 1:].float().reshape(1, M, M, -1).permute(0, 3, 1, 2)
    pe = F.interpolate(pe, size=(h, w), mode="bicubic", antialias=True, align_corners=False)
    pe = pe.permute(0, 2, 3, 1).reshape(1, h * w, -1)
    return torch.cat([cls_pe, pe], dim=1).to(pos_embed.dtype)


def dinov2(sd: SD, p: str, imgs: Tensor, bf16: bool, depth: int = 24, num_heads: int = 16) -> Tensor:
    """DINOv2 ViT-L/14 with 4 registers (ext): returns x_norm_patchtokens
    (N, h*w, C).  ``imgs`` are already ResNet-normalised (N,3,H,W)."""
    N, _, H, W = imgs.shape
    ps = sd[p + "patch_embed.proj.weight"].shape[-1]
    h, w = H // ps, W // ps
    x = F.conv2d(_r(imgs, bf16), _r(sd[p + "patch_embed.proj.weight"], bf16), _r(sd[p + "patch_embed.proj.bias"], bf16),
                 stride=ps)
    x = _r(x, bf16).flatten(2).transpose(1, 2)
    x = torch.cat([sd[p + "cls_token"].expand(N, -1, -1), x], dim=1)
    x = x + interpolated_pos_embed(sd[p + "pos_embed"], h, w)
    nreg = sd[p + "register_tokens"].shape[1]
    x = torch.cat([x[:, :1], sd[p + "register_tokens"].expand(N, -1, -1), x[:, 1:]], dim=1)
    for i in range(depth):
        x = block(sd, f"{p}blocks.{i}.", x, num_heads, eps=1e-6, bf16=bf16)
    x = layer_norm(x, sd[p + "norm.weight"], sd[p + "norm.bias"], 1e-6)
    return x[:, 1 + nreg:]


def aggregator(sd: SD, images: Tensor, bf16: bool = False, keep: Tuple[int, ...] = (4, 11, 17, 23),
               depth: int = 24, num_heads: int = 16, dino_depth: int = 24) -> Tuple[List[Tensor], int]:
    """VGGT Aggregator.forward (ext), called at featureAligned_vggt.py:78.
    Returns only the concatenated (frame, global) outputs of the ``keep``
    layers (featureAligned_vggt.py:24,79), each (B,S,P,2C) fp32, and
    patch_start_idx."""
    p = "aggregator."
    B, S, _, H, W = images.shape
    mean = torch.tensor(RESNET_MEAN).view(1, 1, 3, 1, 1)
    std = torch.tensor(RESNET_STD).view(1, 1, 3, 1, 1)
    x = ((images - mean) / std).view(B * S, 3, H, W)
    patch = dinov2(sd, p + "patch_embed.", x, bf16, depth=dino_depth, num_heads=num_heads)
    cam = slice_expand_and_flatten(sd[p + "camera_token"], B, S).reshape(B * S, 1, -1)
    reg = slice_expand_and_flatten(sd[p + "register_token"], B, S)
    reg = reg.reshape(B * S, reg.shape[2], -1)
    tokens = torch.cat([cam, reg, patch], dim=1)
    psi = 1 + reg.shape[1]
    ps = sd[p + "patch_embed.patch_embed.proj.weight"].shape[-1]
    pos = position_grid(B * S, H // ps, W // ps, psi)
    _, P, C = tokens.shape
    outs = []
    for i in range(depth):
        tokens = block(sd, f"{p}frame_blocks.{i}.", tokens.view(B * S, P, C), num_heads, pos, "2d", True, bf16=bf16)
        fr = tokens.view(B, S, P, C)
        tokens = block(sd, f"{p}global_blocks.{i}.", tokens.view(B, S * P, C), num_heads,
                       pos.view(B, S * P, 2), "2d", True, bf16=bf16)
        gl = tokens.view(B, S, P, C)
        if i in keep:
            outs.append(torch.cat([fr, gl], dim=-1))
    return outs, psi


# ----------------------------------------------------------------------------
# rotation / pose utilities (VGGT utils/rotation.py, pose_enc.py, geometry.py;
# aligned_vggt/utils/data.py:12-52, geometry.py:4-37)
# ----------------------------------------------------------------------------
def quat_to_mat(q: Tensor) -> Tensor:
    """VGGT rotation.quat_to_mat, scalar-last xyzw (ext)."""
    i, j, k, r = torch.unbind(q, -1)
    two_s = 2.0 / (q * q).sum(-1)
    o = torch.stack((
        1 - two_s * (j * j + k * k), two_s * (i * j - k * r), two_s * (i * k + j * r),
        two_s * (i * j + k * r), 1 - two_s * (i * i + k * k), two_s * (j * k - i * r),
        two_s * (i * k - j * r), two_s * (j * k + i * r), 1 - two_s * (i * i + j * j)), -1)
    return o.reshape(q.shape[:-1] + (3, 3))


def _sqrt_pos(x: Tensor) -> Tensor:
    ret = torch.zeros_like(x)
    m = x > 0
    ret[m] = torch.sqrt(x[m])
    return ret


def mat_to_quat(m: Tensor) -> Tensor:
    """VGGT rotation.mat_to_quat -> xyzw with w >= 0 (ext)."""
    bd = m.shape[:-2]
    m00, m01, m02, m10, m11, m12, m20, m21, m22 = torch.unbind(m.reshape(bd + (9,)), -1)
    q_abs = _sqrt_pos(torch.stack([1.0 + m00 + m11 + m22, 1.0 + m00 - m11 - m22,
                                   1.0 - m00 + m11 - m22, 1.0 - m00 - m11 + m22], -1))
    cand = torch.stack([
        torch.stack([q_abs[..., 0] ** 2, m21 - m12, m02 - m20, m10 - m01], -1),
        torch.stack([m21 - m12, q_abs[..., 1] ** 2, m10 + m01, m02 + m20], -1),
        torch.stack([m02 - m20, m10 + m01, q_abs[..., 2] ** 2, m12 + m21], -1),
        torch.stack([m10 - m01, m20 + m02, m21 + m12, q_abs[..., 3] ** 2], -1)], -2)
    flr = torch.tensor(0.1, dtype=q_abs.dtype)
    cand = cand / (2.0 * q_abs[..., None].max(flr))
    out = cand[F.one_hot(q_abs.argmax(-1), num_classes=4) > 0.5, :].reshape(bd + (4,))
    out = out[..., [1, 2, 3, 0]]
    return torch.where(out[..., 3:4] < 0, -out, out)


def closed_form_inverse_se3(se3: Tensor) -> Tensor:
    """VGGT geometry.closed_form_inverse_se3 over (N,4,4)/(N,3,4) (ext)."""
    R = se3[:, :3, :3]
    T = se3[:, :3, 3:]
    Rt = R.transpose(1, 2)
    inv = torch.eye(4, dtype=se3.dtype).unsqueeze(0).repeat(se3.shape[0], 1, 1)
    inv[:, :3, :3] = Rt
    inv[:, :3, 3:] = -torch.bmm(Rt, T)
    return inv


def extri_to_pose_encoding(extr: Tensor) -> Tensor:
    """aligned_vggt/utils/data.py:12-30."""
    quat = mat_to_quat(extr[:, :, :3, :3])
    quat = quat / quat.norm(dim=-1, keepdim=True).clamp(min=1e-8)
    return torch.cat([extr[:, :, :3, 3], quat], dim=-1).float()


def pose_encoding_to_extri(enc: Tensor) -> Tensor:
    """aligned_vggt/utils/data.py:33-52 -> (B,S,4,4)."""
    T = enc[..., :3]
    quat = enc[..., 3:7]
    quat = quat / quat.norm(dim=-1, keepdim=True).clamp(min=1e-8)
    e = torch.cat([quat_to_mat(quat), T[..., None]], dim=-1)
    e = F.pad(e, (0, 0, 0, 1, 0, 0, 0, 0))
    e[:, :, 3, 3] = 1.0
    return e


def pose_encoding_to_extri_intri(enc: Tensor, hw) -> Tuple[Tensor, Tensor]:
    """VGGT pose_enc.pose_encoding_to_extri_intri, absT_quaR_FoV (ext)."""
    H, W = hw
    R = quat_to_mat(enc[..., 3:7])
    extr = torch.cat([R, enc[..., :3, None]], dim=-1)
    fy = (H / 2.0) / torch.tan(enc[..., 7] / 2.0)
    fx = (W / 2.0) / torch.tan(enc[..., 8] / 2.0)
    intr = torch.zeros(enc.shape[:2] + (3, 3), dtype=enc.dtype)
    intr[..., 0, 0] = fx
    intr[..., 1, 1] = fy
    intr[..., 0, 2] = W / 2
    intr[..., 1, 2] = H / 2
    intr[..., 2, 2] = 1.0
    return extr, intr


def extri_intri_to_pose_encoding(extr: Tensor, intr: Tensor, hw) -> Tensor:
    """VGGT pose_enc.extri_intri_to_pose_encoding, absT_quaR_FoV (ext)."""
    H, W = hw
    quat = mat_to_quat(extr[:, :, :3, :3])
    fov_h = 2 * torch.atan((H / 2) / intr[..., 1, 1])
    fov_w = 2 * torch.atan((W / 2) / intr[..., 0, 0])
    return torch.cat([extr[:, :, :3, 3], quat, fov_h[..., None], fov_w[..., None]], dim=-1).float()


def average_pose_encodings(enc: Tensor) -> Tensor:
    """aligned_vggt/utils/geometry.py:4-37 (Markley quaternion mean)."""
    B, N, _ = enc.shape
    t = enc[..., :3].mean(dim=1, keepdim=True)
    q = enc[..., 3:7]
    q = q / q.norm(dim=-1, keepdim=True).clamp(min=1e-8)
    wts = (torch.ones(B, N, dtype=q.dtype) / N)[..., None, None]
    M = (wts * (q.unsqueeze(-1) * q.unsqueeze(-2))).sum(dim=1)
    _, vec = torch.linalg.eigh(M)
    v = vec[..., -1]
    v = v / v.norm(dim=-1, keepdim=True)
    return torch.cat([t, v.unsqueeze(1)], dim=-1).float()


# ----------------------------------------------------------------------------
# camera head (VGGT heads/camera_head.py, ext)
# ----------------------------------------------------------------------------
def camera_head(sd: SD, tokens_list: List[Tensor], num_iterations: int = 4, p: str = "camera_head.",
                trunk_depth: int = 4, num_heads: int = 16) -> List[Tensor]:
    tok = tokens_list[-1][:, :, 0]
    tok = layer_norm(tok, sd[p + "token_norm.weight"], sd[p + "token_norm.bias"], 1e-5)
    B, S, C = tok.shape
    pred = None
    outs = []
    for _ in range(num_iterations):
        if pred is None:
            inp = F.linear(sd[p + "empty_pose_tokens"].expand(B, S, -1), sd[p + "embed_pose.weight"], sd[p + "embed_pose.bias"])
        else:
            inp = F.linear(pred, sd[p + "embed_pose.weight"], sd[p + "embed_pose.bias"])
        mod = F.linear(F.silu(inp), sd[p + "poseLN_modulation.1.weight"], sd[p + "poseLN_modulation.1.bias"])
        shift, scale, gate = mod.chunk(3, dim=-1)
        x = gate * (layer_norm(tok, None, None, 1e-6) * (1 + scale) + shift)
        x = x + tok
        for i in range(trunk_depth):
            x = block(sd, f"{p}trunk.{i}.", x, num_heads)
        x = layer_norm(x, sd[p + "trunk_norm.weight"], sd[p + "trunk_norm.bias"], 1e-5)
        delta = mlp(sd, p + "pose_branch.", x, False)
        pred = delta if pred is None else pred + delta
        # activate_pose: trans linear, quat linear, fl relu
        outs.append(torch.cat([pred[..., :7], F.relu(pred[..., 7:])], dim=-1))
    return outs


# ----------------------------------------------------------------------------
# DPT head (VGGT heads/dpt_head.py + heads/utils.py, ext)
# ----------------------------------------------------------------------------
def make_sincos_pos_embed(embed_dim: int, pos: Tensor, omega_0: float = 100) -> Tensor:
    omega = torch.arange(embed_dim // 2, dtype=torch.double)
    omega /= embed_dim / 2.0
    omega = 1.0 / omega_0 ** omega
    out = torch.einsum("m,d->md", pos.reshape(-1), omega)
    return torch.cat([torch.sin(out), torch.cos(out)], dim=1).float()


def create_uv_grid(width: int, height: int, aspect_ratio: float, dtype=torch.float32) -> Tensor:
    diag = (aspect_ratio ** 2 + 1.0) ** 0.5
    span_x = aspect_ratio / diag
    span_y = 1.0 / diag
    lx = -span_x * (width - 1) / width
    rx = span_x * (width - 1) / width
    ty = -span_y * (height - 1) / height
    by = span_y * (height - 1) / height
    xs = torch.linspace(lx, rx, steps=width, dtype=dtype)
    ys = torch.linspace(ty, by, steps=height, dtype=dtype)
    uu, vv = torch.meshgrid(xs, ys, indexing="xy")
    return torch.stack((uu, vv), dim=-1)


def dpt_pos_embed(C: int, h: int, w: int, W: int, H: int, ratio: float = 0.1) -> Tensor:
    """DPTHead._apply_pos_embed table, (C, h, w)."""
    grid = create_uv_grid(w, h, aspect_ratio=W / H)
    pf = grid.reshape(-1, 2)
    emb = torch.cat([make_sincos_pos_embed(C // 2, pf[:, 0]), make_sincos_pos_embed(C // 2, pf[:, 1])], dim=-1)
    return (emb.view(h, w, C) * ratio).permute(2, 0, 1)


def _conv(sd: SD, p: str, x: Tensor, stride: int = 1, padding: int = 0) -> Tensor:
    return F.conv2d(x, sd[p + "weight"], sd.get(p + "bias"), stride=stride, padding=padding)


def _rcu(sd: SD, p: str, x: Tensor) -> Tensor:
    """ResidualConvUnit with in-place ReLU activation: the skip sees relu(x)
    (SPEC_ASSUMPTIONS.md A9)."""
    xr = F.relu(x)
    out = _conv(sd, p + "conv1.", xr, padding=1)
    out = _conv(sd, p + "conv2.", F.relu(out), padding=1)
    return out + xr


def _fusion(sd: SD, p: str, x0: Tensor, x1: Optional[Tensor], size=None) -> Tensor:
    out = x0
    if x1 is not None:
        out = out + _rcu(sd, p + "resConfUnit1.", x1)
    out = _rcu(sd, p + "resConfUnit2.", out)
    if size is None:
        out = F.interpolate(out, scale_factor=2, mode="bilinear", align_corners=True)
    else:
        out = F.interpolate(out, size=size, mode="bilinear", align_corners=True)
    return _conv(sd, p + "out_conv.", out)


def dpt_head(sd: SD, p: str, tokens_list: List[Tensor], images: Tensor, patch_start_idx: int,
             activation: str, conf_activation: str = "expp1", frames_chunk_size: int = 8, pos_embed: bool = True,
             stages: Optional[dict] = None) -> Tuple[Tensor, Tensor]:
    """DPTHead.forward (ext).  Frame chunking (frames_chunk_size) does not
    change the arithmetic; all frames are processed at once here.
    ``stages``: filled with the NCHW sub-stage outputs the third-party pin
    (tests/golden/dpt_hf.npz) checks -- reassemble{i}, rn{i}, fused{j}
    (j = 0 is refinenet4) and head_pre (before the activations)."""
    st = stages if stages is not None else {}
    B, S, _, H, W = images.shape
    ps = 14
    ph, pw = H // ps, W // ps
    outs = []
    resize = ["resize_layers.0.", "resize_layers.1.", None, "resize_layers.3."]
    for li in range(4):
        x = tokens_list[li][:, :, patch_start_idx:]
        x = x.reshape(B * S, -1, x.shape[-1])
        x = layer_norm(x, sd[p + "norm.weight"], sd[p + "norm.bias"], 1e-5)
        x = x.permute(0, 2, 1).reshape(B * S, x.shape[-1], ph, pw)
        x = _conv(sd, f"{p}projects.{li}.", x)
        if pos_embed:
            x = x + dpt_pos_embed(x.shape[1], ph, pw, W, H)
        if li == 0:
            x = F.conv_transpose2d(x, sd[p + "resize_layers.0.weight"], sd[p + "resize_layers.0.bias"], stride=4)
        elif li == 1:
            x = F.conv_transpose2d(x, sd[p + "resize_layers.1.weight"], sd[p + "resize_layers.1.bias"], stride=2)
        elif li == 3:
            x = _conv(sd, p + "resize_layers.3.", x, stride=2, padding=1)
        st[f"reassemble{li}"] = x
        outs.append(x)
    ls = [_conv(sd, p + f"scratch.layer{i + 1}_rn.", outs[i], padding=1) for i in range(4)]
    for i in range(4):
        st[f"rn{i}"] = ls[i]
    l1, l2, l3, l4 = ls
    out = st["fused0"] = _fusion(sd, p + "scratch.refinenet4.", l4, None, size=l3.shape[2:])
    out = st["fused1"] = _fusion(sd, p + "scratch.refinenet3.", out, l3, size=l2.shape[2:])
    out = st["fused2"] = _fusion(sd, p + "scratch.refinenet2.", out, l2, size=l1.shape[2:])
    out = st["fused3"] = _fusion(sd, p + "scratch.refinenet1.", out, l1)
    out = _conv(sd, p + "scratch.output_conv1.", out, padding=1)
    out = F.interpolate(out, size=(ph * ps, pw * ps), mode="bilinear", align_corners=True)
    if pos_embed:
        out = out + dpt_pos_embed(out.shape[1], out.shape[2], out.shape[3], W, H)
    out = F.relu(_conv(sd, p + "scratch.output_conv2.0.", out, padding=1))
    out = st["head_pre"] = _conv(sd, p + "scratch.output_conv2.2.", out)
    fmap = out.permute(0, 2, 3, 1)
    xyz, conf = fmap[..., :-1], fmap[..., -1]
    if activation == "exp":
        pts = torch.exp(xyz)
    elif activation == "inv_log":
        pts = torch.sign(xyz) * torch.expm1(torch.abs(xyz))
    else:
        raise ValueError(activation)
    conf = 1 + conf.exp() if conf_activation == "expp1" else conf.exp()
    return pts.view(B, S, *pts.shape[1:]), conf.view(B, S, *conf.shape[1:])


# ----------------------------------------------------------------------------
# alignment head (aligned_vggt/heads/alignment_head.py) + gated update
# ----------------------------------------------------------------------------
def gated_update(sd: SD, p: str, memory: Tensor, update: Tensor) -> Tensor:
    """aligned_vggt/layers/gated_update.py:43-79."""
    B, N, D = memory.shape
    scale = update.norm(dim=-1, keepdim=True)
    upd = update.expand_as(memory)
    mean_scaled = memory.mean(dim=1, keepdim=True).expand_as(memory) * scale
    mem_scaled = memory * scale
    inp = torch.cat([upd, mem_scaled, mean_scaled], dim=-1)
    deltas = []
    for i in range(N):
        h = F.gelu(F.linear(inp[:, i], sd[f"{p}delta_mlps.{i}.0.weight"], sd[f"{p}delta_mlps.{i}.0.bias"]))
        deltas.append(F.linear(h, sd[f"{p}delta_mlps.{i}.2.weight"], sd[f"{p}delta_mlps.{i}.2.bias"]))
    diff = torch.stack(deltas, dim=1) - memory
    g_in = torch.cat([diff, mem_scaled], dim=-1).detach()  # gated_update.py:69: the gate sees no gradient path
    g = F.linear(F.gelu(F.linear(g_in, sd[p + "gate_mlp.0.weight"], sd[p + "gate_mlp.0.bias"])),
                 sd[p + "gate_mlp.2.weight"], sd[p + "gate_mlp.2.bias"])
    g = torch.sigmoid(g)
    orth = diff - (diff * memory).sum(-1, keepdim=True) * memory
    d = F.normalize(orth, dim=-1)
    return F.normalize(memory + g * d, dim=-1)


def decode_alignments(sd: SD, p: str, frame_tok: Tensor, num_memory_tokens: int, memory: Optional[Tensor],
                      num_heads: int = 8, depth_decoder: int = 2) -> Tuple[Tensor, Tensor, Optional[Tensor]]:
    """alignment_head.py:427-540 (eval mode: no frame dropout), fp32."""
    B, S, _ = frame_tok.shape
    seq = torch.arange(1, S)
    pos_frame = (seq.view(1, S - 1).expand(B, -1), torch.zeros(1, dtype=seq.dtype).view(1, 1).expand(B, -1))
    if num_memory_tokens > 0:
        cross = torch.arange(0, S + num_memory_tokens)
        cross[-num_memory_tokens:] += S
    else:
        cross = torch.arange(0, S)
    pos_cross = (torch.zeros(1, dtype=cross.dtype).view(1, 1).expand(B, -1), cross.view(1, -1).expand(B, -1))
    tok = F.linear(frame_tok, sd[p + "project_dec.weight"], sd[p + "project_dec.bias"])
    C = tok.shape[-1]
    tok = layer_norm(tok, sd[p + "dec_norm.weight"], sd[p + "dec_norm.bias"], 1e-5)
    directional = None
    if num_memory_tokens > 0:
        norm_t = tok.norm(dim=-1).mean(dim=-1, keepdim=True).unsqueeze(1)
        if memory is None:
            mem = sd[p + "memory_token"].expand(B, *sd[p + "memory_token"].shape[1:])
            fi = F.linear(tok[:, 0], sd[p + "frame_proj.weight"], sd[p + "frame_proj.bias"]).view(B, -1, C)
            fdir = fi / fi.norm(dim=-1, keepdim=True).clamp_min(1e-6)
            a = torch.sigmoid(sd[p + "alpha"])
            directional = (1 - a) * mem + a * fdir
            eff = mem * norm_t
        else:
            directional = memory
            eff = memory * norm_t
        cross_tok = torch.cat([tok, eff], dim=1)
    else:
        cross_tok = tok
    first = tok[:, :1]
    for i in range(depth_decoder):
        first = cross_attention_block(sd, f"{p}chunk_cross_blocks.{i}.", first, cross_tok, num_heads, pos_cross, False)
    new_mem = None
    if num_memory_tokens > 0:
        new_mem = gated_update(sd, p + "gated_update.", directional, first)
    chunk_tok = layer_norm(first, sd[p + "chunk_norm.weight"], sd[p + "chunk_norm.bias"], 1e-5)
    ft = tok[:, 1:]
    for i in range(depth_decoder):
        ft = cross_attention_block(sd, f"{p}frame_cross_blocks.{i}.", ft, chunk_tok, num_heads, pos_frame, False)
    ft = layer_norm(ft, sd[p + "frame_norm.weight"], sd[p + "frame_norm.bias"], 1e-5)
    frame_se3 = mlp(sd, p + "frame_se3_decoder.", ft, False)
    chunk_sim3 = mlp(sd, p + "chunk_sim3_decoder.", chunk_tok, False).clone()
    chunk_sim3[:, :, -1] = torch.exp(chunk_sim3[:, :, -1])
    return chunk_sim3, frame_se3, new_mem


def alignment_head(sd: SD, tokens: Tensor, image_size, next_num_overlap: int, overlap_tokens: Optional[Tensor],
                   memory_tokens: Optional[Tensor], num_memory_tokens: int = 8, temporal_attention: bool = True,
                   bf16: bool = False, p: str = "alignment_head.", depth_aa: int = 4, num_heads: int = 8,
                   patch_size: int = 14):
    """AlignmentHead.forward, alignment_head.py:224-345 (eval mode)."""
    H, W = image_size
    tokens = linear(tokens, sd[p + "project_in.weight"], sd[p + "project_in.bias"], bf16)
    B, S, P, C = tokens.shape
    tokens = layer_norm(tokens, sd[p + "token_norm.weight"], sd[p + "token_norm.bias"], 1e-5)
    T = overlap_tokens.shape[1] if overlap_tokens is not None else None
    al = slice_expand_and_flatten(sd[p + "per_frame_alignment_token"], B, S)
    tokens = torch.cat([al, tokens], dim=2)
    _, _, P, C = tokens.shape
    if not temporal_attention:
        raise NotImplementedError("temporal_attention=False (global variant) is not in any BASELINE config")
    seq = torch.arange(S)
    if overlap_tokens is not None:
        att = seq + (S - (T - 1))
        cross = torch.cat([seq[:1], seq[-(T - 1):]])
        pos_t = (att.view(1, S).expand(B * P, -1), cross.view(1, T).expand(B * P, -1))
    else:
        pos_t = (seq.view(1, S).expand(B * P, -1), seq.view(1, S).expand(B * P, -1))
    pos2d = position_grid(B * S, H // patch_size, W // patch_size, 6)
    for i in range(depth_aa):
        tokens = block(sd, f"{p}frame_blocks.{i}.", tokens.reshape(B * S, P, C), num_heads, pos2d, "2d", True, bf16=bf16)
        # alignment_head.py:372-380: a raw .view (not a permute) of (B,S,P,C) as (B*P,S,C)
        x = tokens.reshape(B * P, S, C)
        # overlap tokens are detached (alignment_head.py:262): no gradient into the previous chunk
        y = overlap_tokens.detach().reshape(B * P, T, C) if overlap_tokens is not None else x
        tokens = cross_attention_block(sd, f"{p}temporal_blocks.{i}.", x, y, num_heads, pos_t, bf16)
    tokens = tokens.reshape(B, S, P, C)
    chunk_sim3, frame_se3, mem = decode_alignments(sd, p, tokens[..., 0, :].float(), num_memory_tokens, memory_tokens)
    new_ov = torch.cat([tokens[:, :1], tokens[:, -next_num_overlap:]], dim=1).contiguous()
    return chunk_sim3, frame_se3, mem, new_ov


# ----------------------------------------------------------------------------
# FeatureAlignedVGGT.forward composition (featureAligned_vggt.py:48-225)
# ----------------------------------------------------------------------------
def merge_results(first, second, num_overlap: int = 0, dim: int = 1):
    """featureAligned_vggt.py:227-254."""
    if num_overlap > 0:
        second = second[:, num_overlap:]
    return torch.cat((first, second), dim=dim)


def compose_poses(chunk_sim3: Tensor, frame_se3: Tensor, cam_pose_enc: Tensor, ctx_pose_enc: Optional[Tensor],
                  gt_first: Optional[Tensor], overlap: int, hw) -> Tuple[Tensor, Tensor]:
    """featureAligned_vggt.py:96-143 and the point transform of :187-196:
    -> (aligned pose encoding (B,S,9), point transform (B,4,4)).
    ctx_pose_enc = context["pose_enc"][-1] (None: first chunk); gt_first =
    gt_poses[:, 0] (chunk_gt mode) or None."""
    H, W = hw
    B = cam_pose_enc.shape[0]
    chunk_se3 = pose_encoding_to_extri(chunk_sim3)
    chunk_scale = chunk_sim3[..., -1]
    pf = pose_encoding_to_extri(frame_se3)
    pf = torch.matmul(pf, chunk_se3)
    pf = torch.cat([chunk_se3, pf], dim=1)
    extr, intr = pose_encoding_to_extri_intri(cam_pose_enc, (H, W))
    extr = F.pad(extr, (0, 0, 0, 1, 0, 0, 0, 0))
    extr[:, :, 3, 3] = 1.0
    ident = closed_form_inverse_se3(extr[:, 0])
    pt_ident = extr[:, 0].clone()
    extr = extr @ ident.view(B, 1, 4, 4)
    extr[:, :, :3, 3] *= chunk_scale.view(B, 1, 1)
    if ctx_pose_enc is not None:
        if gt_first is not None:
            mean_t = gt_first.reshape(B, 1, 4, 4).to(extr)
        else:
            ctx_o = pose_encoding_to_extri(ctx_pose_enc[:, -overlap:])
            inv_o = closed_form_inverse_se3(extr[:, :overlap].reshape(B * overlap, 4, 4)).reshape(B, overlap, 4, 4)
            ct = inv_o @ ctx_o
            if overlap > 1:
                mean_t = pose_encoding_to_extri(average_pose_encodings(extri_to_pose_encoding(ct)))
            else:
                mean_t = ct
    else:
        mean_t = torch.eye(4, dtype=cam_pose_enc.dtype).view(1, 1, 4, 4).expand(B, -1, -1, -1)
    pf = torch.matmul(pf, mean_t)
    aligned = torch.matmul(extr, pf)
    aligned_enc = extri_intri_to_pose_encoding(aligned, intr, (H, W))
    if ctx_pose_enc is not None:
        tr = closed_form_inverse_se3(pf[:, 0]) @ pt_ident
    else:
        tr = pt_ident
    return aligned_enc, tr


def feature_aligned_encode(sd: SD, images: Tensor, enable_camera=True, enable_depth=True, enable_point=False,
                           bf16: bool = False, agg_kwargs: Optional[dict] = None) -> dict:
    """The context-free half of FeatureAlignedVGGT.forward: aggregator
    (featureAligned_vggt.py:78-82), camera head (:106), depth head (:166-168),
    point head (:183-185) -- raw outputs before any Sim(3) scaling."""
    toks, psi = aggregator(sd, images, bf16=bf16, **(agg_kwargs or {}))
    enc = {"tokens": toks, "patch_start_idx": psi}
    if enable_camera:
        enc["cam_pose_enc"] = camera_head(sd, toks)[-1]
    if enable_depth:
        enc["depth"], enc["depth_conf"] = dpt_head(sd, "depth_head.", toks, images, psi, "exp")
    if enable_point:
        enc["points"], enc["points_conf"] = dpt_head(sd, "point_head.", toks, images, psi, "inv_log")
    return enc


def feature_aligned_forward(sd: SD, images: Tensor, num_overlap: int, context: Optional[dict] = None,
                            gt_poses: Optional[Tensor] = None, enable_camera=True, enable_depth=True,
                            enable_point=False, num_memory_tokens: int = 8, bf16: bool = False,
                            training: bool = False, agg_kwargs: Optional[dict] = None) -> dict:
    """FeatureAlignedVGGT.forward, featureAligned_vggt.py:48-225."""
    enc = feature_aligned_encode(sd, images, enable_camera, enable_depth, enable_point, bf16, agg_kwargs)
    return feature_aligned_compose(sd, enc, images, num_overlap, context, gt_poses,
                                   num_memory_tokens=num_memory_tokens, bf16=bf16, training=training)


def feature_aligned_compose(sd: SD, enc: dict, images: Tensor, num_overlap: int, context: Optional[dict] = None,
                            gt_poses: Optional[Tensor] = None, num_memory_tokens: int = 8, bf16: bool = False,
                            training: bool = False) -> dict:
    """featureAligned_vggt.py:84-225 on given encoder outputs ``enc``
    (feature_aligned_encode): alignment head, Sim(3)/SE(3) composition,
    Markley mean over the overlap, scale / point transforms, context lists."""
    B, S, _, H, W = images.shape
    pred = {}
    toks = enc["tokens"]
    enable_camera = "cam_pose_enc" in enc
    ctx_ov = ctx_mem = None
    if context is not None:
        ctx_ov = context["overlap_tokens"]
        if num_memory_tokens > 0:
            ctx_mem = context["memory_tokens"][-1]
    overlap = num_overlap if S > num_overlap else S - 1
    chunk_sim3, frame_se3, mem, ov_tok = alignment_head(sd, toks[-1], (H, W), overlap, ctx_ov, ctx_mem,
                                                        num_memory_tokens=num_memory_tokens, bf16=bf16)
    chunk_scale = chunk_sim3[..., -1]
    if enable_camera:
        ctx_pe = context["pose_enc"][-1] if context is not None else None
        aligned_enc, tr = compose_poses(chunk_sim3, frame_se3, enc["cam_pose_enc"], ctx_pe,
                                        gt_poses[:, 0] if (context is not None and gt_poses is not None) else None,
                                        overlap, (H, W))
        pred["overlap_tokens"] = ov_tok
        if context is None:
            pred["pose_enc"] = [aligned_enc]
            pred["chunk_sim3_alignment_enc"] = chunk_sim3
            pred["frame_se3_alignment_enc"] = frame_se3
            if num_memory_tokens > 0:
                pred["memory_tokens"] = [mem]
        else:
            context.setdefault("pose_enc", []).append(aligned_enc)
            pred["pose_enc"] = context["pose_enc"]
            pred["chunk_sim3_alignment_enc"] = merge_results(context["chunk_sim3_alignment_enc"], chunk_sim3)
            pred["frame_se3_alignment_enc"] = merge_results(context["frame_se3_alignment_enc"], frame_se3)
            if num_memory_tokens > 0:
                context.setdefault("memory_tokens", []).append(mem)
                pred["memory_tokens"] = context["memory_tokens"]
    if "depth" in enc:
        depth, conf = enc["depth"], enc["depth_conf"]
        depth = depth * chunk_scale.view(B, 1, 1, 1, 1)
        if context is None:
            pred["depth"], pred["depth_conf"] = [depth], [conf]
        else:
            context.setdefault("depth", []).append(depth)
            pred["depth"] = context["depth"]
            context.setdefault("depth_conf", []).append(conf)
            pred["depth_conf"] = context["depth_conf"]
    if "points" in enc:
        pts, pconf = enc["points"], enc["points_conf"]
        if enable_camera:
            pts = pts * chunk_scale.view(B, 1, 1, 1, 1)
            ph = torch.cat([pts, torch.ones_like(pts[..., :1])], dim=-1).view(B, -1, 4)
            pts = (ph @ tr.transpose(-1, -2))[..., :3].view(B, S, H, W, 3)
        if context is None:
            pred["world_points"], pred["world_points_conf"] = [pts], [pconf]
        else:
            context.setdefault("world_points", []).append(pts)
            pred["world_points"] = context["world_points"]
            context.setdefault("world_points_conf", []).append(pconf)
            pred["world_points_conf"] = context["world_points_conf"]
    if not training:
        if context is None:
            pred["images"] = [images]
        else:
            context.setdefault("images", []).append(images)
            pred["images"] = context["images"]
    return pred


# ----------------------------------------------------------------------------
# chunking (aligned_vggt/utils/data.py:155-225)
# ----------------------------------------------------------------------------
def generate_chunks(num_frames: int, seq_width: int, overlap: int) -> List[List[int]]:
    """data.py:178-190, mode 'chunk_overlap'."""
    idx = []
    if num_frames < seq_width:
        return [list(range(num_frames))]
    for i in range(0, num_frames - seq_width + 1, seq_width - overlap):
        idx.append(list(range(i, i + seq_width)))
    if len(idx) * (seq_width - overlap) < num_frames - overlap:
        idx.append(list(range(len(idx) * (seq_width - overlap), num_frames)))
    return idx
