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

from .runtime import scratch_table

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
    "vggt_tune": [_i, _i],
    "vggt_set_stream_config": [_vp, _i, _i],
    "vggt_mfma_probe": [_vp, _vp, _vp, _i, _i, _vp],
    "vggt_attention_stamps": [_vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _vp, _i, _i, _i, _i,
                              _f, _vp],
    "vggt_gemm_bf16": [_vp, _i64, _vp, _i64, _vp, _i, _i, _i, _i, _vp, _i64, _vp, _vp, _i64, _vp],
    "vggt_gemm_qkv": [_vp, _i64, _vp, _i64, _vp, _i, _i, _i, _i, _vp, _i64, _vp, _vp, _vp, _vp, _f, _i, _vp, _i, _vp,
                      _vp, _i, _vp],
    "vggt_gemm_headnorm": [_vp, _i64, _vp, _i64, _vp, _i, _i, _i, _i, _i, _vp, _i64, _vp, _vp, _f, _i, _vp, _i, _vp,
                           _vp, _i, _vp],
    "vggt_linear_f32_grouped": [_vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _i, _i, _i, _i, _i, _i, _vp, _i64, _i64,
                                _vp],
    "vggt_gated_update_prep": [_vp, _vp, _i, _i, _i, _vp, _vp, _vp],
    "vggt_gated_update_diff": [_vp, _vp, _i, _i, _vp, _vp],
    "vggt_gated_update_tail": [_vp, _vp, _vp, _i, _i, _vp, _vp],
    "vggt_layernorm": [_vp, _i, _i64, _vp, _vp, _f, _i, _i, _vp, _i, _i64, _vp],
    "vggt_resid_add_layernorm": [_vp, _i64, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _f, _i, _i, _vp, _i64, _vp],
    "vggt_headnorm_rope": [_vp, _i64, _i, _i, _i, _i, _vp, _vp, _f, _i, _vp, _i, _vp, _vp, _i, _vp],
    "vggt_attention_fwd": [_vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _i, _i, _i, _i, _i, _f,
                           _vp],
    "vggt_patch_im2col": [_vp, _i, _i, _i, _i, ctypes.POINTER(_f), ctypes.POINTER(_f), _vp, _i, _vp],
    "vggt_dino_assemble": [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp],
    "vggt_special_tokens": [_vp, _i64, _i, _i, _i, _i, _i, _vp, _vp],
    "vggt_copy_rows_f32": [_vp, _i64, _vp, _i64, _i, _i, _vp],
    "vggt_qknorm_rope": [_vp, _i64, _i, _i, _i, _vp, _vp, _vp, _vp, _f, _i, _vp, _i, _vp, _vp, _i, _vp],
    "vggt_layernorm_grouped": [_vp, _i, _i64, _vp, _vp, _f, _i, _i, _vp, _i, _i64, _i, _i, _i, _i, _i, _vp],
    "vggt_linear_f32": [_vp, _i64, _vp, _i64, _vp, _i, _i, _i, _i, _i, _vp, _i64, _vp, _vp],
    "vggt_linear_f32_ws": [_vp, _i64, _vp, _i64, _vp, _i, _i, _i, _i, _i, _vp, _i64, _vp, _vp, ctypes.c_size_t, _vp],
    "vggt_attention_small": [_vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _vp, _i64, _i64, _i, _i, _i, _i, _i, _i, _f,
                             _vp],
    "vggt_headnorm_rope_f32": [_vp, _i64, _i, _i, _i, _i, _vp, _vp, _f, _i, _vp, _i, _vp, _vp, _i, _vp],
    "vggt_cast_f32_bf16": [_vp, _i64, _vp, _i64, _i, _i, _vp],
    "vggt_conv2d_f32": [_vp, _i64, _i, _i, _i, _i, _vp, _vp, _i, _i, _i, _i, _i, _vp, _i64, _i, _i, _vp, _i64, _i, _vp,
                        _i64, _vp, _i, _vp],
    "vggt_conv2d_bf16x3": [_vp, _i64, _i, _i, _i, _i, _vp, _vp, _vp, _i, _i, _i, _i, _i, _vp, _i64, _i, _i, _vp, _i64,
                           _i, _vp, _i64, _vp, _i, _vp],
    "vggt_split_bf16x2": [_vp, _i64, _vp, _vp, _vp],
    "vggt_conv2d_bf16x3_pre": [_vp, _vp, _i64, _i, _i, _i, _i, _vp, _vp, _vp, _i, _i, _i, _i, _i, _vp, _i64, _i, _vp,
                               _i64, _i, _vp, _i64, _vp, _i, _vp, _vp, _i64, _i, _vp],
    "vggt_upsample_bilinear_split": [_vp, _i, _i, _i, _i, _vp, _i, _i, _vp, _vp, _vp, _i, _vp],
    "vggt_upsample_bilinear_split_sep": [_vp, _i, _i, _i, _i, _vp, _i, _i, _vp, _vp, _vp, _i, _vp],
    "vggt_conv2d_upsample_bf16x3": [_vp, _i, _i, _i, _i, _vp, _i, _i, _vp, _vp, _vp, _i, _i, _vp, _i64, _vp, _vp,
                                    _i64, _i, _vp],
    "vggt_split_act_bf16x2": [_vp, _i64, _i64, _i, _i, _vp, _vp, _vp],
    "vggt_upsample_bilinear_f32": [_vp, _i, _i, _i, _i, _vp, _i, _i, _vp, _vp],
    "vggt_dpt_activate": [_vp, _i64, _i64, _i, _i, _i, _vp, _vp, _vp, _vp],
    "vggt_irls_sim3": [_vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _i, _i64, _f, _f, _i, _f, _vp, _vp, _vp, _vp,
                       ctypes.c_size_t, _vp],
    "vggt_sim3_points": [_vp, _i64, _i, _i64, _vp, _vp, _vp, _i64, _vp],
    "vggt_scale_f32": [_vp, _i64, _i, _i64, _vp, _vp],
    "vggt_pose_compose": [_vp, _vp, _vp, _vp, _i, _vp, _i, _i, _i, _i, _i, _vp, _vp, _vp],
    # training (backward) entry points
    "vggt_attention_fwd_lse": [_vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _vp, _i, _i, _i,
                               _i, _i, _f, _vp],
    "vggt_attention_bwd": [_vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _vp, _vp, _i64, _i64, _vp, _vp, _vp, _i64,
                           _vp, _vp, _i64, _i, _i, _i, _i, _i, _f, _vp],
    "vggt_attention_small_bwd": [_vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _vp,
                                 _vp, _i64, _i64, _i, _i, _i, _i, _i, _i, _f, _vp],
    "vggt_layernorm_bwd": [_vp, _i, _i64, _vp, _f, _vp, _i, _i64, _vp, _i, _i64, _i, _i, _i, _i, _i, _i, _i, _i, _vp,
                           _vp, _vp, ctypes.c_size_t, _vp],
    "vggt_headnorm_rope_bwd": [_vp, _i64, _vp, _i64, _i, _i, _i, _i, _i, _vp, _vp, _f, _i, _vp, _i, _vp, _vp, _i, _vp,
                               _vp, _vp, _vp, _vp, ctypes.c_size_t, _vp],
    "vggt_colsum": [_vp, _i, _i64, _i, _i, _vp, _i, _vp, ctypes.c_size_t, _vp],
    "vggt_layerscale_bwd": [_vp, _i64, _vp, _i, _i64, _vp, _vp, _i, _i64, _i, _i, _vp, _vp, _vp, ctypes.c_size_t,
                            _vp],
    "vggt_gelu_fwd": [_vp, _i, _i64, _vp, _i, _i64, _i, _i, _vp],
    "vggt_gelu_bwd": [_vp, _i, _i64, _vp, _i, _i64, _vp, _i, _i64, _i, _i, _vp, _vp, ctypes.c_size_t, _vp],
    "vggt_resid_scale_add": [_vp, _i64, _vp, _i, _i64, _vp, _i, _i, _vp],
    "vggt_gemm_bf16_gelu_pre": [_vp, _i64, _vp, _i64, _vp, _i, _i, _i, _vp, _i64, _vp, _i64, _vp],
    "vggt_resid_scale_add_from": [_vp, _i64, _vp, _i64, _vp, _i, _i64, _vp, _i, _i, _vp],
    "vggt_qknorm_rope_out": [_vp, _i64, _vp, _i64, _i, _i, _i, _vp, _vp, _vp, _vp, _f, _i, _vp, _i, _vp, _vp, _i, _vp],
    "vggt_headnorm_rope_out": [_vp, _i64, _vp, _i64, _i, _i, _i, _vp, _vp, _f, _i, _vp, _i, _vp, _vp, _i, _vp],
    "vggt_transpose_b16": [_vp, _i64, _i, _i, _vp, _i64, _i, _vp],
    "vggt_wgrad_f32": [_vp, _i64, _vp, _i64, _i, _i, _i, _vp, _i64, _i, _vp],
    "vggt_wgrad_bias_f32": [_vp, _i64, _vp, _i64, _i, _i, _i, _vp, _i64, _vp, _i, _vp],
    "vggt_wgrad_bf16": [_vp, _i64, _vp, _i64, _i, _i, _i, _vp, _i64, _i, _vp, ctypes.c_size_t, _vp],
    "vggt_batch_dot_f32": [_vp, _vp, _i64, _i, _i64, _vp, _vp, ctypes.c_size_t, _vp],
}
_WS_FNS = {"vggt_colred_workspace_bytes": [_i, _i], "vggt_layernorm_bwd_workspace_bytes": [_i, _i],
           "vggt_headnorm_rope_bwd_workspace_bytes": [_i, _i], "vggt_batch_dot_workspace_bytes": [_i, _i64],
           "vggt_wgrad_bf16_workspace_bytes": [_i, _i, _i]}

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
        L.vggt_irls_workspace_bytes.argtypes = [_i]
        L.vggt_irls_workspace_bytes.restype = ctypes.c_size_t
        for name, argt in _WS_FNS.items():
            fn = getattr(L, name)
            fn.argtypes = argt
            fn.restype = ctypes.c_size_t
        _lib = L
    return _lib


def version() -> str:
    return lib().vggt_version().decode()


TUNE_GEMM_TILE = 1
TUNE_ATTN_WAVES = 2
TUNE_ATTN_VARIANT = 3
TUNE_CONV_PF2 = 4
TUNE_ATTN16 = 5
TUNE_LINEAR_ONE_LAUNCH = 6
TUNE_LINEAR_SPLIT_K = 7
TUNE_LINEAR_WK = 8
TUNE_GEMM_BALANCE = 10


def tune(knob: int, value: int) -> int:
    """vggt_tune: set a process-wide kernel-variant knob, return the previous value."""
    rc = lib().vggt_tune(knob, value)
    if rc == VGGT_ERR_UNSUPPORTED:
        raise ValueError(f"vggt_tune: unsupported knob/value ({knob}, {value})")
    return rc


STREAM_SHORT_WORKGROUPS = 1


def set_stream_config(stream: int, cus: int, flags: int = 0) -> int:
    """vggt_set_stream_config on a raw stream handle: the CUs its launches may use (a CU-masked
    stream; 0 = the device's) and STREAM_* flags.  Returns the previous cus | flags << 16;
    cus = flags = 0 forgets the stream."""
    rc = lib().vggt_set_stream_config(ctypes.c_void_p(stream), cus, flags)
    if rc < 0:
        raise ValueError(f"vggt_set_stream_config: rejected ({rc})")
    return rc


def mfma_probe(iters: int = 200_000, random: bool = True, seconds: float = 2.0, device=None) -> dict:
    """Sustained bf16 MFMA rate and in-kernel clock (vggt_mfma_probe): one
    workgroup of 4 waves per CU, back-to-back launches for ``seconds`` (the
    clock the chip holds under load), the last launch timed by HIP events and
    stamped with s_memtime / s_memrealtime; returns TF/s, the clock (median over
    workgroups) and the FLOP per cycle per CU that implies."""
    import statistics
    device = torch.device(device or "cuda")
    ncu = torch.cuda.get_device_properties(device).multi_processor_count
    g = torch.Generator(device="cpu").manual_seed(0)
    n = ncu * 256 * 16
    ops = (torch.randn(n, generator=g) if random else torch.zeros(n)).to(torch.bfloat16).to(device)
    stamps = torch.zeros(ncu * 4, dtype=torch.int64, device=device)
    sink = torch.empty(ncu * 256, dtype=torch.float32, device=device)
    st = ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
    launch = lambda: _check(lib().vggt_mfma_probe(_p(stamps), _p(sink), _p(ops), ncu, iters, st),  # noqa: E731
                            "vggt_mfma_probe")
    import time
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end:
        launch()
        torch.cuda.synchronize(device)
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    launch()
    b.record()
    b.synchronize()
    ms = a.elapsed_time(b)
    sp = stamps.view(ncu, 4).cpu().tolist()
    clocks = [(t1 - t0) / (r1 - r0) * 100e6 for t0, t1, r0, r1 in sp if r1 > r0]
    clk = statistics.median(clocks)
    flop = ncu * 4 * iters * 8 * 32768.0
    return {"tflops": round(flop / (ms * 1e-3) / 1e12, 1), "clock_ghz": round(clk / 1e9, 3),
            "flop_per_cycle_per_cu": round(flop / ncu / (ms * 1e-3 * clk), 1), "ms": round(ms, 3), "cus": ncu,
            "operands": "random bf16" if random else "zeros"}


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


def gemm_bf16_gelu_pre(a: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, out: torch.Tensor,
                       pre: torch.Tensor) -> torch.Tensor:
    """out = GELU(a . w^T + bias) and pre = a . w^T + bias, both bf16 (one pass)."""
    _dev(a, "gemm_bf16_gelu_pre")
    M, K = a.shape
    N_ = w.shape[0]
    assert a.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.shape[1] == K
    assert out.shape[0] == M and out.shape[1] == N_ and pre.shape[0] == M and pre.shape[1] == N_
    assert out.dtype == torch.bfloat16 and pre.dtype == torch.bfloat16
    rc = lib().vggt_gemm_bf16_gelu_pre(_p(a), _ld(a), _p(w), _ld(w), _p(bias), M, N_, K, _p(out), _ld(out), _p(pre),
                                       _ld(pre), _stream())
    _check(rc, "vggt_gemm_bf16_gelu_pre")
    return out


def gemm_qkv(a: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, out: torch.Tensor, H: int, D: int, qw=None, qb=None,
             kw=None, kb=None, eps: float = 0.0, mode: int = ROPE_NONE, pos=None, period: int = 1, cos=None,
             sin=None) -> torch.Tensor:
    """Fused qkv projection + q/k LayerNorm + RoPE (vggt_gemm_qkv)."""
    _dev(a, "gemm_qkv")
    M, K = a.shape
    assert a.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.shape == (3 * H * D, K)
    assert out.shape[0] == M and out.shape[1] == 3 * H * D
    tab = cos.shape[0] if cos is not None else 0
    rc = lib().vggt_gemm_qkv(_p(a), _ld(a), _p(w), _ld(w), _p(bias), M, H, D, K, _p(out), _ld(out), _p(qw), _p(qb),
                             _p(kw), _p(kb), float(eps), mode, _p(pos), period, _p(cos), _p(sin), tab, _stream())
    _check(rc, "vggt_gemm_qkv")
    return out


def gemm_headnorm(a: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, out: torch.Tensor, H: int, D: int, nw=None,
                  nb=None, eps: float = 0.0, mode: int = ROPE_NONE, pos=None, period: int = 1, cos=None,
                  sin=None) -> torch.Tensor:
    """q (N = H*D) or packed kv (N = 2*H*D) projection with the per-head norm +
    RoPE of the first H*D columns in the epilogue (vggt_gemm_headnorm)."""
    _dev(a, "gemm_headnorm")
    M, K = a.shape
    N_ = w.shape[0]
    assert a.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.shape[1] == K and N_ in (H * D, 2 * H * D)
    assert out.shape[0] == M and out.shape[1] == N_ and out.dtype == torch.bfloat16
    tab = cos.shape[0] if cos is not None else 0
    rc = lib().vggt_gemm_headnorm(_p(a), _ld(a), _p(w), _ld(w), _p(bias), M, N_, H, D, K, _p(out), _ld(out), _p(nw),
                                  _p(nb), float(eps), mode, _p(pos), period, _p(cos), _p(sin), tab, _stream())
    _check(rc, "vggt_gemm_headnorm")
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


def resid_add_layernorm(x: torch.Tensor, y: torch.Tensor, gamma: torch.Tensor, out2: Optional[torch.Tensor],
                        w: Optional[torch.Tensor], b: Optional[torch.Tensor], eps: float,
                        xn: Optional[torch.Tensor]) -> None:
    """x += gamma * y (fp32 residual, bf16 branch output; the GEMM EPI_RESID_F32
    arithmetic), mirrored into out2 if given, then xn = LayerNorm(x) in bf16 if
    xn is given (one HBM pass instead of the epilogue RMW + a LayerNorm)."""
    _dev(x, "resid_add_layernorm")
    M, C = x.shape
    assert x.dtype == torch.float32 and y.dtype == torch.bfloat16 and y.shape[0] == M and y.shape[1] == C
    assert xn is None or (xn.dtype == torch.bfloat16 and xn.shape[0] == M and xn.shape[1] == C)
    rc = lib().vggt_resid_add_layernorm(_p(x), _ld(x), _p(y), _ld(y), _p(gamma), _p(out2),
                                        _ld(out2) if out2 is not None else 0, _p(w), _p(b), float(eps), M, C, _p(xn),
                                        _ld(xn) if xn is not None else 0, _stream())
    _check(rc, "vggt_resid_add_layernorm")


def headnorm_rope(buf: torch.Tensor, col_off: int, H: int, D: int, w: Optional[torch.Tensor],
                  b: Optional[torch.Tensor], eps: float, mode: int = ROPE_NONE, pos: Optional[torch.Tensor] = None,
                  period: int = 1, cos: Optional[torch.Tensor] = None, sin: Optional[torch.Tensor] = None) -> None:
    _dev(buf, "headnorm_rope")
    M = buf.shape[0]
    tab = cos.shape[0] if cos is not None else 0
    rc = lib().vggt_headnorm_rope(_p(buf), _ld(buf), col_off, M, H, D, _p(w), _p(b), float(eps), mode, _p(pos),
                                  period, _p(cos), _p(sin), tab, _stream())
    _check(rc, "vggt_headnorm_rope")


def qknorm_rope(qkv: torch.Tensor, H: int, D: int, qw, qb, kw, kb, eps: float, mode: int = ROPE_NONE, pos=None,
                period: int = 1, cos=None, sin=None) -> None:
    _dev(qkv, "qknorm_rope")
    tab = cos.shape[0] if cos is not None else 0
    rc = lib().vggt_qknorm_rope(_p(qkv), _ld(qkv), qkv.shape[0], H, D, _p(qw), _p(qb), _p(kw), _p(kb), float(eps), mode,
                                _p(pos), period, _p(cos), _p(sin), tab, _stream())
    _check(rc, "vggt_qknorm_rope")


def qknorm_rope_out(src: torch.Tensor, dst: torch.Tensor, H: int, D: int, qw, qb, kw, kb, eps: float,
                    mode: int = ROPE_NONE, pos=None, period: int = 1, cos=None, sin=None) -> None:
    """dst[:, :2HD] = q/k-norm + RoPE of src[:, :2HD] (src untouched)."""
    _dev(src, "qknorm_rope_out")
    assert src.dtype == torch.bfloat16 and dst.dtype == torch.bfloat16 and dst.shape[0] == src.shape[0]
    assert src.shape[1] >= 2 * H * D and dst.shape[1] >= 2 * H * D
    tab = cos.shape[0] if cos is not None else 0
    rc = lib().vggt_qknorm_rope_out(_p(src), _ld(src), _p(dst), _ld(dst), src.shape[0], H, D, _p(qw), _p(qb), _p(kw),
                                    _p(kb), float(eps), mode, _p(pos), period, _p(cos), _p(sin), tab, _stream())
    _check(rc, "vggt_qknorm_rope_out")


def headnorm_rope_out(src: torch.Tensor, dst: torch.Tensor, H: int, D: int, w, b, eps: float, mode: int = ROPE_NONE,
                      pos=None, period: int = 1, cos=None, sin=None) -> None:
    """dst[:, :HD] = per-head norm + RoPE of src[:, :HD] (src untouched)."""
    _dev(src, "headnorm_rope_out")
    assert src.dtype == torch.bfloat16 and dst.dtype == torch.bfloat16 and dst.shape[0] == src.shape[0]
    assert src.shape[1] >= H * D and dst.shape[1] >= H * D
    tab = cos.shape[0] if cos is not None else 0
    rc = lib().vggt_headnorm_rope_out(_p(src), _ld(src), _p(dst), _ld(dst), src.shape[0], H, D, _p(w), _p(b),
                                      float(eps), mode, _p(pos), period, _p(cos), _p(sin), tab, _stream())
    _check(rc, "vggt_headnorm_rope_out")


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


def attention_stamps(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, o: torch.Tensor, batch: int, heads: int,
                     nq: int, nk: int, q_bstride: int, k_bstride: int, o_bstride: int) -> torch.Tensor:
    """Diagnostic (vggt_attention_stamps): the default D = 64 forward with per-wave
    s_memtime cycle sums of its tile segments; returns (nwg * NW, 8) int64."""
    _dev(q, "attention_stamps")
    nw = 8 if nq >= 4096 else 4
    nwg = ((nq + nw * 32 - 1) // (nw * 32)) * heads * batch
    st = torch.zeros(nwg * nw, 8, dtype=torch.int64, device=q.device)
    rc = lib().vggt_attention_stamps(_p(q), _ld(q), q_bstride, _p(k), _ld(k), k_bstride, _p(v), _ld(v), k_bstride,
                                     _p(o), _ld(o), o_bstride, _p(st), batch, heads, nq, nk, float(64 ** -0.5),
                                     _stream())
    _check(rc, "vggt_attention_stamps")
    return st


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


def _dt(t: torch.Tensor) -> int:
    if t.dtype == torch.bfloat16:
        return DTYPE_BF16
    if t.dtype == torch.float32:
        return DTYPE_F32
    raise RuntimeError(f"unsupported dtype {t.dtype}")


def layernorm_grouped(x: torch.Tensor, w, b, eps: float, out: torch.Tensor, M: int, C: int, group: int,
                      x_gstride: int, x_off: int, y_gstride: int, y_off: int) -> None:
    _dev(x, "layernorm_grouped")
    rc = lib().vggt_layernorm_grouped(_p(x), _dt(x), _ld(x), _p(w), _p(b), float(eps), M, C, _p(out), _dt(out),
                                      _ld(out), group, x_gstride, x_off, y_gstride, y_off, _stream())
    _check(rc, "vggt_layernorm_grouped")


def linear_f32(a: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], out: torch.Tensor, epi: int = EPI_F32,
               act_in: int = 0, gamma: Optional[torch.Tensor] = None) -> torch.Tensor:
    _dev(a, "linear_f32")
    M, K = a.shape
    N_ = w.shape[0]
    assert a.dtype == torch.float32 and w.dtype == torch.float32 and w.shape[1] == K and out.shape == (M, N_)
    # split-K scratch for skinny M: the zeroed per-tile counter words, then at most
    # LINEAR_F32_MAX_SPLITS splits of a 64-row-padded [M, N] fp32 slab
    need = LINEAR_F32_WS_COUNTERS + LINEAR_F32_MAX_SPLITS * ((M + 63) // 64) * 64 * N_
    ws = _split_ws(a.device, need) if M <= 256 else None
    rc = lib().vggt_linear_f32_ws(_p(a), _ld(a), _p(w), _ld(w), _p(bias), M, N_, K, act_in, epi, _p(out), _ld(out),
                                  _p(gamma), _p(ws), 0 if ws is None else ws.numel() * 4, _stream())
    _check(rc, "vggt_linear_f32_ws")
    return out


def linear_f32_grouped(a: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], out: torch.Tensor,
                       epi: int = EPI_F32) -> torch.Tensor:
    """out[g] = epi(a[g] . w[g]^T + bias[g]) for g < G: a [G, M, K] (rows may be
    strided), w [G, N, K], bias [G, N], out [G, M, N] fp32 (vggt_linear_f32_grouped)."""
    _dev(a, "linear_f32_grouped")
    G, M, K = a.shape
    N_ = w.shape[1]
    assert w.shape == (G, N_, K) and out.shape == (G, M, N_) and a.dtype == w.dtype == out.dtype == torch.float32
    assert a.stride(2) == 1 and w.stride(2) == 1 and w.stride(1) == K and out.stride(2) == 1
    assert bias is None or (bias.shape == (G, N_) and bias.stride(1) == 1)
    rc = lib().vggt_linear_f32_grouped(_p(a), a.stride(1), a.stride(0), _p(w), w.stride(1), w.stride(0), _p(bias),
                                       bias.stride(0) if bias is not None else 0, M, N_, K, G, 0, epi, _p(out),
                                       out.stride(1), out.stride(0), _stream())
    _check(rc, "vggt_linear_f32_grouped")
    return out


def gated_update_prep(memory: torch.Tensor, update: torch.Tensor, inp: torch.Tensor, g_in: torch.Tensor) -> None:
    _dev(memory, "gated_update_prep")
    B, Nt, D = memory.shape
    assert memory.is_contiguous() and update.is_contiguous() and update.numel() == B * D
    assert inp.is_contiguous() and inp.numel() == B * Nt * 3 * D and g_in.is_contiguous() and g_in.numel() == B * Nt * 2 * D
    _check(lib().vggt_gated_update_prep(_p(memory), _p(update), B, Nt, D, _p(inp), _p(g_in), _stream()),
           "vggt_gated_update_prep")


def gated_update_diff(memory: torch.Tensor, deltas: torch.Tensor, g_in: torch.Tensor) -> None:
    _dev(memory, "gated_update_diff")
    D = memory.shape[-1]
    rows = memory.numel() // D
    assert memory.is_contiguous() and deltas.is_contiguous() and deltas.numel() == rows * D
    assert g_in.is_contiguous() and g_in.numel() == rows * 2 * D
    _check(lib().vggt_gated_update_diff(_p(memory), _p(deltas), rows, D, _p(g_in), _stream()), "vggt_gated_update_diff")


def gated_update_tail(memory: torch.Tensor, deltas: torch.Tensor, logit: torch.Tensor, out: torch.Tensor) -> None:
    _dev(memory, "gated_update_tail")
    D = memory.shape[-1]
    rows = memory.numel() // D
    assert memory.is_contiguous() and deltas.is_contiguous() and logit.is_contiguous() and logit.numel() == rows
    assert out.is_contiguous() and out.numel() == rows * D
    _check(lib().vggt_gated_update_tail(_p(memory), _p(deltas), _p(logit), rows, D, _p(out), _stream()),
           "vggt_gated_update_tail")


_SPLIT_WS = {}


def _stream_key(device) -> tuple:
    """(device, current stream id): scratch is reused in stream order only, so
    work queued on two streams at once (the ring aligns chunk i on a side
    stream while the compute stream encodes, dist/pipeline.py) never shares a
    slab -- and a grown slab's old storage is released on the one stream that
    used it (the caching allocator's reuse is ordered on that stream)."""
    device = torch.device(device)
    if device.type != "cuda":
        return (device, 0)
    if device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    return (device, torch.cuda.current_stream(device).stream_id)


LINEAR_F32_WS_COUNTERS = 1024  # include/vggt_mi355x.h VGGT_LINEAR_F32_WS_COUNTERS
LINEAR_F32_MAX_SPLITS = 32  # VGGT_LINEAR_F32_MAX_SPLITS


def _split_ws(device, n_floats: int) -> torch.Tensor:
    """Grow-only per-(device, stream) scratch for split-K partial sums; zero-filled
    when (re)allocated (vggt_linear_f32_ws's tile counters at its start must start at
    zero, and every call leaves them zero)."""
    key = _stream_key(device)
    table = scratch_table(_SPLIT_WS, "split_k")
    t = table.get(key)
    if t is None or t.numel() < n_floats:
        t = torch.zeros(n_floats, device=key[0], dtype=torch.float32)
        table[key] = t
    return t


ATTN_SMALL_EXACT = 0x100  # include/vggt_mi355x.h VGGT_ATTN_SMALL_EXACT


def attention_small(q, k, v, o, batch: int, heads: int, nq: int, nk: int, D: int, q_bstride: int, k_bstride: int,
                    o_bstride: int, scale: Optional[float] = None, exact: bool = False) -> None:
    """exact: the fp32 LDS form for bf16 windows too (the training forward, which its
    backward recomputes in fp32); else <= 16 x 16 bf16 windows run on the matrix cores."""
    _dev(q, "attention_small")
    sc = D ** -0.5 if scale is None else scale
    rc = lib().vggt_attention_small(_p(q), _ld(q), q_bstride, _p(k), _ld(k), k_bstride, _p(v), _ld(v), _p(o), _ld(o),
                                    o_bstride, _dt(q) | (ATTN_SMALL_EXACT if exact else 0), batch, heads, nq, nk, D,
                                    float(sc), _stream())
    _check(rc, "vggt_attention_small")


def headnorm_rope_any(buf: torch.Tensor, col_off: int, H: int, D: int, w, b, eps: float, mode: int = ROPE_NONE,
                      pos=None, period: int = 1, cos=None, sin=None) -> None:
    """Dispatch on dtype: bf16 -> vectorised kernel (D in {64,128}); f32 -> generic kernel."""
    if buf.dtype == torch.bfloat16:
        return headnorm_rope(buf, col_off, H, D, w, b, eps, mode, pos, period, cos, sin)
    _dev(buf, "headnorm_rope_f32")
    tab = cos.shape[0] if cos is not None else 0
    rc = lib().vggt_headnorm_rope_f32(_p(buf), _ld(buf), col_off, buf.shape[0], H, D, _p(w), _p(b), float(eps), mode,
                                      _p(pos), period, _p(cos), _p(sin), tab, _stream())
    _check(rc, "vggt_headnorm_rope_f32")


def cast_f32_bf16(x: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    _dev(x, "cast_f32_bf16")
    rc = lib().vggt_cast_f32_bf16(_p(x), _ld(x), _p(out), _ld(out), x.shape[0], x.shape[1], _stream())
    _check(rc, "vggt_cast_f32_bf16")
    return out


def conv2d_f32(x: torch.Tensor, nimg: int, hi: int, wi: int, ci: int, w: torch.Tensor, bias, co: int, kh: int, kw: int,
               stride: int, pad: int, y: torch.Tensor, relu_in: bool = False, relu_out: bool = False,
               res1: Optional[torch.Tensor] = None, res1_relu: bool = False, res2: Optional[torch.Tensor] = None,
               pos: Optional[torch.Tensor] = None, shuffle: int = 0) -> torch.Tensor:
    """x, y, res*: 2-D [pixels, channels] row views (NHWC flattened)."""
    _dev(x, "conv2d_f32")
    rc = lib().vggt_conv2d_f32(_p(x), _ld(x), nimg, hi, wi, ci, _p(w), _p(bias), co, kh, kw, stride, pad, _p(y), _ld(y),
                               int(relu_in), int(relu_out), _p(res1), _ld(res1) if res1 is not None else 0,
                               int(res1_relu), _p(res2), _ld(res2) if res2 is not None else 0, _p(pos), shuffle,
                               _stream())
    _check(rc, "vggt_conv2d_f32")
    return y


def conv2d_bf16x3(x: torch.Tensor, nimg: int, hi: int, wi: int, ci: int, w_hi: torch.Tensor, w_lo: torch.Tensor, bias,
                  co: int, kh: int, kw: int, stride: int, pad: int, y: torch.Tensor, relu_in: bool = False,
                  relu_out: bool = False, res1: Optional[torch.Tensor] = None, res1_relu: bool = False,
                  res2: Optional[torch.Tensor] = None, pos: Optional[torch.Tensor] = None, shuffle: int = 0):
    """vggt_conv2d_f32 on the bf16 matrix path with split (hi + lo) operands."""
    _dev(x, "conv2d_bf16x3")
    rc = lib().vggt_conv2d_bf16x3(_p(x), _ld(x), nimg, hi, wi, ci, _p(w_hi), _p(w_lo), _p(bias), co, kh, kw, stride,
                                  pad, _p(y), _ld(y), int(relu_in), int(relu_out), _p(res1),
                                  _ld(res1) if res1 is not None else 0, int(res1_relu), _p(res2),
                                  _ld(res2) if res2 is not None else 0, _p(pos), shuffle, _stream())
    _check(rc, "vggt_conv2d_bf16x3")
    return y


def conv2d_bf16x3_pre(x_hi: torch.Tensor, x_lo: torch.Tensor, nimg: int, hi: int, wi: int, ci: int,
                      w_hi: torch.Tensor, w_lo: torch.Tensor, bias, co: int, kh: int, kw: int, stride: int, pad: int,
                      y: torch.Tensor, relu_out: bool = False, res1: Optional[torch.Tensor] = None,
                      res1_relu: bool = False, res2: Optional[torch.Tensor] = None, pos: Optional[torch.Tensor] = None,
                      shuffle: int = 0, y_split=None, split_relu: bool = False):
    """conv2d_bf16x3 on an activation pre-split by split_act_bf16x2 (LDS-DMA gather).
    y (f32) and/or y_split = (hi, lo) bf16 (the next conv's split input) are written."""
    _dev(x_hi, "conv2d_bf16x3_pre")
    yh, yl = y_split if y_split is not None else (None, None)
    rc = lib().vggt_conv2d_bf16x3_pre(_p(x_hi), _p(x_lo), _ld(x_hi), nimg, hi, wi, ci, _p(w_hi), _p(w_lo), _p(bias), co,
                                      kh, kw, stride, pad, _p(y), _ld(y) if y is not None else 0, int(relu_out),
                                      _p(res1), _ld(res1) if res1 is not None else 0, int(res1_relu), _p(res2),
                                      _ld(res2) if res2 is not None else 0, _p(pos), shuffle, _p(yh), _p(yl),
                                      _ld(yh) if yh is not None else 0, int(split_relu), _stream())
    _check(rc, "vggt_conv2d_bf16x3_pre")
    return y


def upsample_bilinear_split(x: torch.Tensor, nimg: int, hi: int, wi: int, C: int, y, ho: int, wo: int,
                            pos: Optional[torch.Tensor] = None, y_split=None, split_relu: bool = False):
    """upsample_bilinear_f32 writing y (may be None) and/or the split halves of relu?(y)."""
    _dev(x, "upsample_bilinear_split")
    yh, yl = y_split if y_split is not None else (None, None)
    rc = lib().vggt_upsample_bilinear_split(_p(x), nimg, hi, wi, C, _p(y), ho, wo, _p(pos), _p(yh), _p(yl),
                                            int(split_relu), _stream())
    _check(rc, "vggt_upsample_bilinear_split")


def upsample_bilinear_split_sep(x: torch.Tensor, nimg: int, hi: int, wi: int, C: int, y, ho: int, wo: int,
                                pos_sep: torch.Tensor, y_split=None, split_relu: bool = False):
    """upsample_bilinear_split with the separable positional table [wo + ho, C/2]."""
    _dev(x, "upsample_bilinear_split_sep")
    yh, yl = y_split if y_split is not None else (None, None)
    assert pos_sep.shape == (wo + ho, C // 2) and pos_sep.is_contiguous()
    rc = lib().vggt_upsample_bilinear_split_sep(_p(x), nimg, hi, wi, C, _p(y), ho, wo, _p(pos_sep), _p(yh), _p(yl),
                                                int(split_relu), _stream())
    _check(rc, "vggt_upsample_bilinear_split_sep")


def conv2d_upsample_bf16x3(x: torch.Tensor, nimg: int, hi: int, wi: int, C: int, pos_sep: Optional[torch.Tensor],
                           ho: int, wo: int, w_hi: torch.Tensor, w_lo: torch.Tensor, bias, co: int,
                           y: Optional[torch.Tensor], relu_out: bool = False, y_split=None, split_relu: bool = False):
    """3x3 conv (pad 1) of the bilinear resize (align_corners) of x [nimg*hi*wi, C] to (ho, wo)
    plus the separable positional table, on split-bf16 operands, without the resized map."""
    _dev(x, "conv2d_upsample_bf16x3")
    yh, yl = y_split if y_split is not None else (None, None)
    rc = lib().vggt_conv2d_upsample_bf16x3(_p(x), nimg, hi, wi, C, _p(pos_sep), ho, wo, _p(w_hi), _p(w_lo), _p(bias),
                                           co, int(relu_out), _p(y), _ld(y) if y is not None else 0, _p(yh), _p(yl),
                                           _ld(yh) if yh is not None else 0, int(split_relu), _stream())
    _check(rc, "vggt_conv2d_upsample_bf16x3")


def split_act_bf16x2(x: torch.Tensor, relu: bool = False, out=None):
    """(hi, lo) bf16 [rows, cols] maps of relu?(x) for a 2-D f32 row view x."""
    _dev(x, "split_act_bf16x2")
    rows, cols = x.shape
    if out is None:
        out = (torch.empty(rows, cols, dtype=torch.bfloat16, device=x.device),
               torch.empty(rows, cols, dtype=torch.bfloat16, device=x.device))
    hi, lo = out
    _check(lib().vggt_split_act_bf16x2(_p(x), _ld(x), rows, cols, int(relu), _p(hi), _p(lo), _stream()),
           "vggt_split_act_bf16x2")
    return hi, lo


def split_bf16x2(x: torch.Tensor):
    """(hi, lo) bf16 tensors with x = hi + lo + O(2^-16 |x|)."""
    _dev(x, "split_bf16x2")
    x = x.contiguous().float()
    hi = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
    lo = torch.empty_like(hi)
    _check(lib().vggt_split_bf16x2(_p(x), x.numel(), _p(hi), _p(lo), _stream()), "vggt_split_bf16x2")
    return hi, lo


def upsample_bilinear_f32(x: torch.Tensor, nimg: int, hi: int, wi: int, C: int, y: torch.Tensor, ho: int, wo: int,
                          pos: Optional[torch.Tensor] = None) -> torch.Tensor:
    _dev(x, "upsample_bilinear_f32")
    rc = lib().vggt_upsample_bilinear_f32(_p(x), nimg, hi, wi, C, _p(y), ho, wo, _p(pos), _stream())
    _check(rc, "vggt_upsample_bilinear_f32")
    return y


def dpt_activate(x: torch.Tensor, npix: int, ppi: int, ncl: int, act: int, scale, pts: torch.Tensor,
                 conf: torch.Tensor) -> None:
    _dev(x, "dpt_activate")
    rc = lib().vggt_dpt_activate(_p(x), _ld(x), npix, ppi, ncl, act, _p(scale), _p(pts), _p(conf), _stream())
    _check(rc, "vggt_dpt_activate")


def _bstride(t: torch.Tensor, per_batch: int) -> int:
    """Batch stride (elements) of a tensor whose first dim is the batch and
    whose per-batch block of ``per_batch`` elements is contiguous."""
    if t.shape[0] > 1:
        return t.stride(0)
    return per_batch


def irls_sim3(src: torch.Tensor, dst: torch.Tensor, conf_src: torch.Tensor, conf_dst: torch.Tensor,
              conf_threshold_factor: float = 0.5, delta: float = 0.1, max_iters: int = 20, tol: float = 1e-9):
    """Batched irls_sim3_umeyama (pointAligned_wrapped_vggt.py:225-305) on the
    GPU.  src/dst: (B, ..., 3) fp32, conf_*: (B, ...) fp32 with the same point
    count; every per-batch block contiguous.  Returns device tensors R (B,3,3),
    t (B,3), s (B,) without synchronising the host."""
    _dev(src, "irls_sim3")
    B = src.shape[0]
    n = src[0].numel() // 3
    for t_, per in ((src, 3 * n), (dst, 3 * n), (conf_src, n)) + (((conf_dst, n),) if conf_dst is not None else ()):
        assert t_.dtype == torch.float32 and t_.shape[0] == B and t_[0].numel() == per and t_[0].is_contiguous(), \
            "irls_sim3: (B, ..., 3) / (B, ...) fp32 inputs with contiguous per-batch blocks"
    L = lib()
    ws_bytes = int(L.vggt_irls_workspace_bytes(B))
    ws = torch.empty((ws_bytes + 15) // 16 * 16, dtype=torch.uint8, device=src.device)
    R = torch.empty(B, 3, 3, device=src.device)
    t = torch.empty(B, 3, device=src.device)
    s = torch.empty(B, device=src.device)
    rc = L.vggt_irls_sim3(_p(src), _bstride(src, 3 * n), _p(dst), _bstride(dst, 3 * n), _p(conf_src),
                          _bstride(conf_src, n), _p(conf_dst), _bstride(conf_dst, n) if conf_dst is not None else 0, B, n, float(conf_threshold_factor),
                          float(delta), int(max_iters), float(tol), _p(R), _p(t), _p(s), _p(ws), ws.numel(), _stream())
    _check(rc, "vggt_irls_sim3")
    return R, t, s


def sim3_points(pts: torch.Tensor, T: torch.Tensor, scale: Optional[torch.Tensor], out: Optional[torch.Tensor] = None):
    """out = T[:3,:3] (scale * pts) + T[:3,3] per batch element; pts (B, ..., 3)
    fp32 with contiguous per-batch blocks, T (B,4,4), scale (B,) or None."""
    _dev(pts, "sim3_points")
    B = pts.shape[0]
    n = pts[0].numel() // 3
    assert pts.dtype == torch.float32 and pts[0].is_contiguous()
    T = T.to(device=pts.device, dtype=torch.float32).contiguous()
    if scale is not None:
        scale = scale.to(device=pts.device, dtype=torch.float32).reshape(B).contiguous()
    if out is None:
        out = torch.empty_like(pts)
    rc = lib().vggt_sim3_points(_p(pts), _bstride(pts, 3 * n), B, n, _p(T), _p(scale), _p(out), _bstride(out, 3 * n),
                                _stream())
    _check(rc, "vggt_sim3_points")
    return out


def pose_compose(chunk_sim3: torch.Tensor, frame_se3: torch.Tensor, cam_pose_enc: torch.Tensor,
                 ctx_pose_enc: Optional[torch.Tensor], gt_first: Optional[torch.Tensor], overlap: int,
                 image_hw, want_point_transform: bool = True):
    """featureAligned_vggt.py:96-143 (+ the point transform of :187-196) in one
    launch -> (aligned_pose_enc (B,S,9), point_transform (B,4,4) or None)."""
    _dev(cam_pose_enc, "pose_compose")
    dev = cam_pose_enc.device
    B, S = cam_pose_enc.shape[:2]
    f32 = lambda t: t.to(device=dev, dtype=torch.float32).contiguous() if t is not None else None  # noqa: E731
    cs, fs, cam = f32(chunk_sim3.reshape(B, 8)), f32(frame_se3.reshape(B, S - 1, 7)), f32(cam_pose_enc)
    ctx = f32(ctx_pose_enc)
    gt = f32(gt_first.reshape(B, 4, 4)) if gt_first is not None else None
    out = torch.empty(B, S, 9, device=dev)
    pt = torch.empty(B, 4, 4, device=dev) if want_point_transform else None
    H, W = int(image_hw[0]), int(image_hw[1])
    rc = lib().vggt_pose_compose(_p(cs), _p(fs), _p(cam), _p(ctx), ctx.shape[1] if ctx is not None else 0, _p(gt),
                                 B, S, int(overlap), H, W, _p(out), _p(pt), _stream())
    _check(rc, "vggt_pose_compose")
    return out, pt


def scale_(x: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
    """x[b] *= scale[b] in place (fp32, contiguous per-batch blocks)."""
    _dev(x, "scale_f32")
    B = x.shape[0]
    n = x[0].numel()
    assert x.dtype == torch.float32 and x[0].is_contiguous()
    scale = scale.to(device=x.device, dtype=torch.float32).reshape(B).contiguous()
    rc = lib().vggt_scale_f32(_p(x), _bstride(x, n), B, n, _p(scale), _stream())
    _check(rc, "vggt_scale_f32")
    return x


# ---------------------------------------------------------------- training (backward) wrappers
_TRAIN_WS = {}


def _train_ws(device, nbytes: int) -> torch.Tensor:
    """Grow-only per-(device, stream) scratch for the deterministic reduction
    partials (stream-ordered reuse: every user consumes it before the next
    launch on the same stream; see _stream_key)."""
    key = _stream_key(device)
    table = scratch_table(_TRAIN_WS, "train")
    t = table.get(key)
    if t is None or t.numel() * 4 < nbytes:
        t = torch.empty((nbytes + 3) // 4 + 64, device=key[0], dtype=torch.float32)
        table[key] = t
    return t


def attention_fwd_lse(q, k, v, o, lse: torch.Tensor, batch: int, heads: int, nq: int, nk: int, D: int,
                      q_bstride: int, k_bstride: int, o_bstride: int, scale: Optional[float] = None) -> None:
    _dev(q, "attention_fwd_lse")
    assert lse.dtype == torch.float32 and lse.numel() >= batch * heads * nq
    sc = D ** -0.5 if scale is None else scale
    rc = lib().vggt_attention_fwd_lse(_p(q), _ld(q), q_bstride, _p(k), _ld(k), k_bstride, _p(v), _ld(v), k_bstride,
                                      _p(o), _ld(o), o_bstride, _p(lse), batch, heads, nq, nk, D, float(sc), _stream())
    _check(rc, "vggt_attention_fwd_lse")


def attention_bwd(q, k, v, o, do, lse, dq, dk, dv, batch: int, heads: int, nq: int, nk: int, D: int, q_bstride: int,
                  k_bstride: int, o_bstride: int, scale: Optional[float] = None) -> None:
    """q/k/v/o/do/dq/dk/dv: 2-D bf16 row views; dk and dv share one leading dimension."""
    _dev(q, "attention_bwd")
    assert _ld(dk) == _ld(dv)
    sc = D ** -0.5 if scale is None else scale
    delta = _train_ws(q.device, 4 * batch * heads * nq)
    rc = lib().vggt_attention_bwd(_p(q), _ld(q), q_bstride, _p(k), _ld(k), k_bstride, _p(v), _ld(v), _p(o), _p(do),
                                  _ld(o), o_bstride, _p(lse), _p(delta), _p(dq), _ld(dq), _p(dk), _p(dv), _ld(dk),
                                  batch, heads, nq, nk, D, float(sc), _stream())
    _check(rc, "vggt_attention_bwd")


def attention_small_bwd(q, k, v, do, dq, dk, dv, batch: int, heads: int, nq: int, nk: int, D: int, q_bstride: int,
                        k_bstride: int, o_bstride: int, dq_bstride: int, dkv_bstride: int,
                        scale: Optional[float] = None) -> None:
    _dev(q, "attention_small_bwd")
    assert _ld(dk) == _ld(dv) and _ld(do) is not None
    sc = D ** -0.5 if scale is None else scale
    rc = lib().vggt_attention_small_bwd(_p(q), _ld(q), q_bstride, _p(k), _ld(k), k_bstride, _p(v), _ld(v), _p(do),
                                        _ld(do), o_bstride, _p(dq), _ld(dq), dq_bstride, _p(dk), _p(dv), _ld(dk),
                                        dkv_bstride, _dt(q), batch, heads, nq, nk, D, float(sc), _stream())
    _check(rc, "vggt_attention_small_bwd")


def layernorm_bwd(x, w, eps: float, dy, dx, accumulate: bool, dw=None, db=None, M: Optional[int] = None,
                  group: Optional[int] = None, x_gstride: int = 0, x_off: int = 0, y_gstride: int = 0,
                  y_off: int = 0, params_write: bool = False) -> None:
    """dx (+)= LayerNorm backward; dw/db (+)= parameter gradients (written
    instead with params_write).  Identity row map unless group/strides are
    given (vggt_layernorm_grouped's)."""
    _dev(x, "layernorm_bwd")
    M = x.shape[0] if M is None else M
    C = x.shape[1]
    L = lib()
    nb = int(L.vggt_layernorm_bwd_workspace_bytes(M, C))
    ws = _train_ws(x.device, nb)
    g = (M if M > 0 else 1) if group is None else group
    rc = L.vggt_layernorm_bwd(_p(x), _dt(x), _ld(x), _p(w), float(eps), _p(dy), _dt(dy), _ld(dy), _p(dx), _dt(dx),
                              _ld(dx), int(accumulate) | (2 if params_write else 0), M, C, g, x_gstride, x_off, y_gstride,
                              y_off, _p(dw), _p(db),
                              _p(ws), ws.numel() * 4, _stream())
    _check(rc, "vggt_layernorm_bwd")


def headnorm_rope_bwd(pre, grad, H: int, hsplit: int, D: int, w0, w1, eps: float, mode: int, pos, period: int, cos,
                      sin, dw0=None, db0=None, dw1=None, db1=None) -> None:
    """In place grad := d(pre) for per-head LayerNorm + RoPE (pre / grad: 2-D row
    views whose column 0 is head 0)."""
    _dev(pre, "headnorm_rope_bwd")
    M = pre.shape[0]
    L = lib()
    ws = _train_ws(pre.device, int(L.vggt_headnorm_rope_bwd_workspace_bytes(M, D)))
    tab = cos.shape[0] if cos is not None else 0
    rc = L.vggt_headnorm_rope_bwd(_p(pre), _ld(pre), _p(grad), _ld(grad), _dt(pre), M, H, hsplit, D, _p(w0), _p(w1),
                                  float(eps), mode, _p(pos), period, _p(cos), _p(sin), tab, _p(dw0), _p(db0), _p(dw1),
                                  _p(db1), _p(ws), ws.numel() * 4, _stream())
    _check(rc, "vggt_headnorm_rope_bwd")


def colsum(x, out, accumulate: bool = True) -> None:
    _dev(x, "colsum")
    M, N_ = x.shape
    L = lib()
    ws = _train_ws(x.device, int(L.vggt_colred_workspace_bytes(M, N_)))
    _check(L.vggt_colsum(_p(x), _dt(x), _ld(x), M, N_, _p(out), int(accumulate), _p(ws), ws.numel() * 4, _stream()),
           "vggt_colsum")


def layerscale_bwd(dout, branch, gamma, dbranch, dgamma=None, dbias=None) -> None:
    _dev(dout, "layerscale_bwd")
    M, N_ = dout.shape
    L = lib()
    ws = _train_ws(dout.device, int(L.vggt_colred_workspace_bytes(M, N_)))
    rc = L.vggt_layerscale_bwd(_p(dout), _ld(dout), _p(branch), _dt(branch), _ld(branch), _p(gamma), _p(dbranch),
                               _dt(dbranch), _ld(dbranch), M, N_, _p(dgamma), _p(dbias), _p(ws), ws.numel() * 4,
                               _stream())
    _check(rc, "vggt_layerscale_bwd")


def gelu_fwd(x, y) -> None:
    _dev(x, "gelu_fwd")
    M, N_ = x.shape
    _check(lib().vggt_gelu_fwd(_p(x), _dt(x), _ld(x), _p(y), _dt(y), _ld(y), M, N_, _stream()), "vggt_gelu_fwd")


def gelu_bwd(dh, pre, dpre, dbias=None) -> None:
    _dev(dh, "gelu_bwd")
    M, N_ = dh.shape
    L = lib()
    ws = _train_ws(dh.device, int(L.vggt_colred_workspace_bytes(M, N_)))
    rc = L.vggt_gelu_bwd(_p(dh), _dt(dh), _ld(dh), _p(pre), _dt(pre), _ld(pre), _p(dpre), _dt(dpre), _ld(dpre), M, N_,
                         _p(dbias), _p(ws), ws.numel() * 4, _stream())
    _check(rc, "vggt_gelu_bwd")


def resid_scale_add(x, branch, gamma) -> None:
    _dev(x, "resid_scale_add")
    M, N_ = x.shape
    rc = lib().vggt_resid_scale_add(_p(x), _ld(x), _p(branch), _dt(branch), _ld(branch), _p(gamma), M, N_, _stream())
    _check(rc, "vggt_resid_scale_add")


def resid_scale_add_from(out, x, branch, gamma) -> None:
    """out = x + gamma * branch (fp32 out / x; out may be x)."""
    _dev(x, "resid_scale_add_from")
    M, N_ = x.shape
    assert out.shape == x.shape and out.dtype == torch.float32 and x.dtype == torch.float32
    rc = lib().vggt_resid_scale_add_from(_p(out), _ld(out), _p(x), _ld(x), _p(branch), _dt(branch), _ld(branch),
                                         _p(gamma), M, N_, _stream())
    _check(rc, "vggt_resid_scale_add_from")


def transpose_b16(src, dst, rows_pad: int) -> None:
    """dst[c, r] = src[r, c]; dst columns [rows, rows_pad) zero."""
    _dev(src, "transpose_b16")
    rows, cols = src.shape
    assert src.element_size() == 2 and dst.element_size() == 2 and dst.shape[0] >= cols and dst.shape[1] >= rows_pad
    rc = lib().vggt_transpose_b16(_p(src), _ld(src), rows, cols, _p(dst), _ld(dst), rows_pad, _stream())
    _check(rc, "vggt_transpose_b16")


def wgrad_bf16(dy, x, dw, accumulate: bool = False) -> None:
    """dw[N, K] (+)= bf16-rounded dy[M, N]^T x[M, K] (bf16 row views, split-K MFMA)."""
    _dev(dy, "wgrad_bf16")
    M, N_ = dy.shape
    K = x.shape[1]
    assert x.shape[0] == M and dw.shape == (N_, K) and dw.dtype == torch.float32
    L = lib()
    ws = _train_ws(dy.device, int(L.vggt_wgrad_bf16_workspace_bytes(M, N_, K)))
    rc = L.vggt_wgrad_bf16(_p(dy), _ld(dy), _p(x), _ld(x), M, N_, K, _p(dw), _ld(dw), int(accumulate), _p(ws),
                           ws.numel() * 4, _stream())
    _check(rc, "vggt_wgrad_bf16")


def wgrad_f32(dy, x, dw, accumulate: bool = True) -> None:
    _dev(dy, "wgrad_f32")
    M, N_ = dy.shape
    K = x.shape[1]
    assert x.shape[0] == M and dw.shape == (N_, K)
    rc = lib().vggt_wgrad_f32(_p(dy), _ld(dy), _p(x), _ld(x), M, N_, K, _p(dw), _ld(dw), int(accumulate), _stream())
    _check(rc, "vggt_wgrad_f32")


def wgrad_bias_f32(dy, x, dw, db, accumulate: bool = False) -> None:
    """dw (+)= dy^T x and db (+)= column sums of dy in one launch (fp32)."""
    _dev(dy, "wgrad_bias_f32")
    M, N_ = dy.shape
    K = x.shape[1]
    assert x.shape[0] == M and dw.shape == (N_, K) and db.shape == (N_,) and db.is_contiguous()
    rc = lib().vggt_wgrad_bias_f32(_p(dy), _ld(dy), _p(x), _ld(x), M, N_, K, _p(dw), _ld(dw), _p(db),
                                   int(accumulate), _stream())
    _check(rc, "vggt_wgrad_bias_f32")


def batch_dot_f32(a, c, out) -> None:
    """out[b] = sum(a[b] * c[b]) (fp32, contiguous per-batch blocks)."""
    _dev(a, "batch_dot_f32")
    B = a.shape[0]
    n = a[0].numel()
    L = lib()
    ws = _train_ws(a.device, int(L.vggt_batch_dot_workspace_bytes(B, n)))
    rc = L.vggt_batch_dot_f32(_p(a), _p(c), _bstride(a, n), B, n, _p(out), _p(ws), ws.numel() * 4, _stream())
    _check(rc, "vggt_batch_dot_f32")
