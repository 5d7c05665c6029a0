"""GPU parity of the HIP aggregator against the CPU oracle (bf16-mixed
emulation tier), through the C ABI."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import vggt_oracle as O  # noqa: E402


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.fixture(scope="module")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda")


def _run(cuda, depth, dino_depth, B, S, H, W, keep):
    from aligned_vggt.backbone.aggregator import Aggregator
    from aligned_vggt.utils.synthetic import synthetic_init_, synthetic_images
    agg = Aggregator(depth=depth, dino_depth=dino_depth)
    synthetic_init_(agg, seed=3)
    sd = {"aggregator." + k: v for k, v in agg.state_dict().items()}
    img = synthetic_images(B, S, H, W)
    ref, psi = O.aggregator(sd, img, bf16=True, keep=keep, depth=depth, dino_depth=dino_depth)
    ref32, _ = O.aggregator(sd, img, bf16=False, keep=keep, depth=depth, dino_depth=dino_depth)
    agg = agg.to(cuda)
    outs, psi2 = agg(img.to(cuda), keep_layers=keep)
    torch.cuda.synchronize()
    assert psi2 == psi == 5
    return [o.cpu() for o in outs], ref, ref32


def test_aggregator_small_depth(cuda):
    outs, ref, ref32 = _run(cuda, depth=3, dino_depth=2, B=1, S=3, H=56, W=70, keep=(0, 2))
    for o, r, r32 in zip(outs, ref, ref32):
        assert o.shape == r.shape
        assert torch.isfinite(o).all()
        e, e32 = _rel(o, r), _rel(r32, r)
        assert e < 2e-2, (e, e32)


def test_aggregator_full_depth_two_frames(cuda):
    """Full 24+24 layer aggregator on a 2-frame 112x112 chunk (layers 4,11,17,23)."""
    outs, ref, ref32 = _run(cuda, depth=24, dino_depth=24, B=1, S=2, H=112, W=112, keep=(4, 11, 17, 23))
    for o, r in zip(outs, ref):
        assert torch.isfinite(o).all()
        assert _rel(o, r) < 3e-2, _rel(o, r)


def test_aggregator_batch2(cuda):
    outs, ref, _ = _run(cuda, depth=2, dino_depth=1, B=2, S=2, H=42, W=56, keep=(1,))
    assert _rel(outs[0], ref[0]) < 2e-2


def test_aggregator_fused_add_ln_matches_epilogue_path(cuda, monkeypatch):
    """fc2 as plain GEMM + fused residual-add / next-norm1 pass (default) vs the
    fp32 read-modify-write epilogue + separate LayerNorm: same arithmetic, so
    the kept-layer outputs agree to fp32 accumulation-order noise."""
    from aligned_vggt.backbone import layers as L
    from aligned_vggt.backbone.aggregator import Aggregator
    from aligned_vggt.utils.synthetic import synthetic_init_, synthetic_images
    agg = Aggregator(depth=4, dino_depth=3)
    synthetic_init_(agg, seed=5)
    agg = agg.to(cuda)
    img = synthetic_images(1, 3, 112, 126).to(cuda)
    monkeypatch.setattr(L, "_FUSED_ADD_LN", True)
    a, _ = agg(img, keep_layers=(0, 3))
    a = [t.clone() for t in a]
    monkeypatch.setattr(L, "_FUSED_ADD_LN", False)
    b, _ = agg(img, keep_layers=(0, 3))
    torch.cuda.synchronize()
    for u, v in zip(a, b):
        assert _rel(u, v) < 2e-3, _rel(u, v)
