"""ctypes binding of the gfx950 C-ABI library ``libvggt_mi355x.so``
(include/vggt_mi355x.h) plus thin torch-tensor wrappers.

The product path has no CPU or eager-PyTorch fallback: if the library is not
built, or a tensor is not on a HIP device, these wrappers raise.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("VGGT_MI355X_LIB", os.path.join(_PKG_ROOT, "lib", "libvggt_mi355x.so"))
HEADER_PATH = os.path.join(os.path.dirname(_PKG_ROOT), "include", "vggt_mi355x.h")

VGGT_OK, VGGT_ERR_SHAPE, VGGT_ERR_ALIGN, VGGT_ERR_HIP, VGGT_ERR_UNSUPPORTED = 0, -1, -2, -3, -4
DTYPE_F32, DTYPE_BF16 = 0, 1
EPI_BF16, EPI_GELU_BF16, EPI_RESID_F32, EPI_F32 = 0, 1, 2, 3
ROPE_NONE, ROPE_2D, ROPE_1D = 0, 1, 2

_ERR = {VGGT_ERR_SHAPE: "unsupported or inconsistent shape", VGGT_ERR_ALIGN: "misaligned pointer or leading dimension",
        VGGT_ERR_HIP: "HIP launch/runtime error", VGGT_ERR_UNSUPPORTED: "unsupported mode or dtype"}

_vp, _i, _i64, _f = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float
_SIGS = {
    "vggt_gemm_bf16": [_vp, _i64, _vp, _i64, _vp, _i, _i, _i, _i, _vp, _i64, _vp, _vp, _i64, _vp],
    "vggt_layernorm": [_vp, _i, _i64, _vp, _vp, _f, _i, _i, _vp, _i, _i64, _vp],
    "vggt_headnorm_rope": [_vp, _i64, _i, _i, _i, _i, _vp, _vp, _f, _i, _vp, _i, _vp, _vp, _i, _vp],
    "vggt_attention_fwd": [_vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _i, _i, _i, _i, _i, _f,
                           _vp],
    "vggt_patch_im2col": [_vp, _i, _i, _i, _i, ctypes.POINTER(_f), ctypes.POINTER(_f), _vp, _i, _vp],
    "vggt_dino_assemble": [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp],
    "vggt_special_tokens": [_vp, _i64, _i, _i, _i, _i, _i, _vp, _vp],
    "vggt_copy_rows_f32": [_vp, _i64, _vp, _i64, _i, _i, _vp],
}

_lib = None

# Optional timing hook: callable(tag, thunk) wrapping tagged launches (bench.py
# records HIP events around them on the launching stream).
EVENT_HOOK = None


def lib() -> ctypes.CDLL:
    """Load the C-ABI library once; raise loudly if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libvggt_mi355x.so not found at {LIB_PATH}: build it with "
                               f"`make -C large-scale-vit-slam_amd/csrc` (or __graft_entry__.build()); "
                               f"there is no CPU fallback for the HIP hot path")
        L = ctypes.CDLL(LIB_PATH)
        for name, argt in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = argt
            fn.restype = ctypes.c_int
        L.vggt_version.restype = ctypes.c_char_p
        _lib = L
    return _lib


def version() -> str:
    return lib().vggt_version().decode()


def _check(rc: int, name: str) -> None:
    if rc != VGGT_OK:
        raise RuntimeError(f"{name}: {_ERR.get(rc, 'error')} (code {rc})")


def _dev(t: torch.Tensor, name: str) -> None:
    if t.device.type != "cuda":
        raise RuntimeError(f"{name}: tensor on {t.device}; the MI355X hot path runs on HIP devices only")


def _p(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream() -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ld(t: torch.Tensor) -> int:
    if t.dim() != 2 or t.stride(1) != 1:
        raise RuntimeError("expected a 2-D row-major (unit inner stride) view")
    return t.stride(0)


# ---------------------------------------------------------------- wrappers
def gemm_bf16(a: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, out: torch.Tensor, epi: int,
              gamma: Optional[torch.Tensor] = None, out2: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[M,N] = epi(a[M,K] . w[N,K]^T + bias)  (bf16 operands)."""
    _dev(a, "gemm_bf16")
    M, K = a.shape
    N = w.shape[0]
    assert a.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.shape[1] == K
    assert out.shape[0] == M and out.shape[1] == N
    rc = lib().vggt_gemm_bf16(_p(a), _ld(a), _p(w), _ld(w), _p(bias), M, N, K, epi, _p(out), _ld(out), _p(gamma),
                              _p(out2), _ld(out2) if out2 is not None else 0, _stream())
    _check(rc, "vggt_gemm_bf16")
    return out


def layernorm(x: torch.Tensor, w: Optional[torch.Tensor], b: Optional[torch.Tensor], eps: float,
              out: torch.Tensor) -> torch.Tensor:
    _dev(x, "layernorm")
    M, C = x.shape
    assert out.shape[0] == M and out.shape[1] == C
    rc = lib().vggt_layernorm(_p(x), DTYPE_BF16 if x.dtype == torch.bfloat16 else DTYPE_F32, _ld(x), _p(w), _p(b),
                              float(eps), M, C, _p(out), DTYPE_BF16 if out.dtype == torch.bfloat16 else DTYPE_F32,
                              _ld(out), _stream())
    _check(rc, "vggt_layernorm")
    return out


def headnorm_rope(buf: torch.Tensor, col_off: int, H: int, D: int, w: Optional[torch.Tensor],
                  b: Optional[torch.Tensor], eps: float, mode: int = ROPE_NONE, pos: Optional[torch.Tensor] = None,
                  period: int = 1, cos: Optional[torch.Tensor] = None, sin: Optional[torch.Tensor] = None) -> None:
    _dev(buf, "headnorm_rope")
    M = buf.shape[0]
    tab = cos.shape[0] if cos is not None else 0
    rc = lib().vggt_headnorm_rope(_p(buf), _ld(buf), col_off, M, H, D, _p(w), _p(b), float(eps), mode, _p(pos),
                                  period, _p(cos), _p(sin), tab, _stream())
    _check(rc, "vggt_headnorm_rope")


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, o: torch.Tensor, batch: int, heads: int, nq: int,
              nk: int, D: int, q_bstride: int, k_bstride: int, o_bstride: int, scale: Optional[float] = None,
              tag: Optional[str] = None) -> None:
    """q/k/v/o are 2-D row views whose column 0 is head 0's first element."""
    _dev(q, "attention")
    sc = D ** -0.5 if scale is None else scale
    L = lib()

    def call():
        return L.vggt_attention_fwd(_p(q), _ld(q), q_bstride, _p(k), _ld(k), k_bstride, _p(v), _ld(v), k_bstride, _p(o),
                                    _ld(o), o_bstride, batch, heads, nq, nk, D, float(sc), _stream())

    rc = EVENT_HOOK(tag, call) if (EVENT_HOOK is not None and tag is not None) else call()
    _check(rc, "vggt_attention_fwd")


def patch_im2col(images: torch.Tensor, patch: int, mean, std, out: torch.Tensor) -> None:
    _dev(images, "patch_im2col")
    F_, _, H, W = images.shape
    m = (ctypes.c_float * 3)(*mean)
    s = (ctypes.c_float * 3)(*std)
    rc = lib().vggt_patch_im2col(_p(images), F_, H, W, patch, m, s, _p(out), out.shape[1], _stream())
    _check(rc, "vggt_patch_im2col")


def dino_assemble(patch: torch.Tensor, cls: torch.Tensor, reg: torch.Tensor, pos: torch.Tensor, F_: int, hw: int,
                  nreg: int, C: int, x: torch.Tensor) -> None:
    _dev(patch, "dino_assemble")
    rc = lib().vggt_dino_assemble(_p(patch), _p(cls), _p(reg), _p(pos), F_, hw, nreg, C, _p(x), _stream())
    _check(rc, "vggt_dino_assemble")


def special_tokens(x: torch.Tensor, F_: int, S: int, P: int, tok: torch.Tensor) -> None:
    _dev(x, "special_tokens")
    n, C = tok.shape[1], tok.shape[2]
    rc = lib().vggt_special_tokens(_p(x), _ld(x), F_, S, P, n, C, _p(tok), _stream())
    _check(rc, "vggt_special_tokens")


def copy_rows_f32(src: torch.Tensor, dst: torch.Tensor) -> None:
    _dev(src, "copy_rows_f32")
    rc = lib().vggt_copy_rows_f32(_p(src), _ld(src), _p(dst), _ld(dst), src.shape[0], src.shape[1], _stream())
    _check(rc, "vggt_copy_rows_f32")
