"""CPU-side checks of the C-ABI boundary: the built library loads and exports
every function declared in include/*.h (no compute calls without a GPU)."""
import ctypes
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"\b(vggt_[a-z0-9_]+)\s*\(", src))
    return names


def test_header_declares_entry_points():
    names = _declared()
    assert {"vggt_gemm_bf16", "vggt_attention_fwd", "vggt_layernorm", "vggt_headnorm_rope"} <= names


def test_library_exports_every_declared_symbol():
    from aligned_vggt import _native
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("library not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_native.LIB_PATH)
    missing = [n for n in sorted(_declared()) if not hasattr(lib, n)]
    assert not missing, missing
    assert _native.version().startswith("vggt_mi355x")
    # every binding signature refers to a declared symbol
    assert set(_native._SIGS) <= _declared()


def test_product_refuses_cpu_tensors():
    import torch
    from aligned_vggt import _native
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("library not built")
    a = torch.zeros(128, 64, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="HIP devices only"):
        _native.gemm_bf16(a, a, torch.zeros(128), torch.zeros(128, 128, dtype=torch.bfloat16), 0)


def test_tune_knobs_range_and_restore():
    """vggt_tune (a host-side switch, no GPU call) returns the previous value and rejects
    values outside each knob's documented range (include/vggt_mi355x.h)."""
    from aligned_vggt import _native as N
    if not os.path.exists(N.LIB_PATH):
        pytest.skip("library not built")
    lib = N.lib()
    assert lib.vggt_tune(6, 5) < 0  # the retired GEMM DMA-placement knob
    for knob, good, bad in ((N.TUNE_ATTN16, (0, 1, 2), (3, -1)),
                            (N.TUNE_ATTN_WAVES, (2, 4, 8), (3, 16)),
                            (N.TUNE_LINEAR_SPLIT_K, (128, 64, 32, 16, 4096), (8, 48, 8192)),
                            (N.TUNE_LINEAR_WK, (0, 64, 128, 4096), (32, 96, 8192, -1)),
                            (N.TUNE_GEMM_BALANCE, (0, 1), (2, -1))):
        first = lib.vggt_tune(knob, good[0])
        assert first >= 0
        prev = good[0]
        for v in good[1:]:
            assert lib.vggt_tune(knob, v) == prev
            prev = v
        for v in bad:
            assert lib.vggt_tune(knob, v) < 0
            assert lib.vggt_tune(knob, prev) == prev  # a rejected value changed nothing
        lib.vggt_tune(knob, first)
    # the defaults the round-3 measurements chose, unless the environment overrides them
    if "VGGT_ATTN16" not in os.environ:
        p = lib.vggt_tune(N.TUNE_ATTN16, 2)
        assert p == 2


def test_stream_config_registry():
    """vggt_set_stream_config (host-side table, no GPU call): returns the previous
    setting (cus | flags << 16), cus = flags = 0 forgets the stream, a null stream,
    a negative count or an unknown flag is rejected."""
    from aligned_vggt import _native as N
    if not os.path.exists(N.LIB_PATH):
        pytest.skip("library not built")
    fake = 0x1234560  # never dereferenced: the table only compares handles
    assert N.set_stream_config(fake, 240) == 0
    assert N.set_stream_config(fake, 224, N.STREAM_SHORT_WORKGROUPS) == 240
    assert N.set_stream_config(fake, 0, N.STREAM_SHORT_WORKGROUPS) == 224 | 1 << 16
    assert N.set_stream_config(fake, 0, 0) == 1 << 16
    assert N.set_stream_config(fake, 0, 0) == 0
    for bad in ((0, 8, 0), (fake, -1, 0), (fake, 0, 2)):
        with pytest.raises(ValueError):
            N.set_stream_config(*bad)
