"""GPU parity of the point-map Sim(3) alignment kernels (vggt_irls_sim3,
vggt_sim3_points, vggt_scale_f32) and of the point-aligned VGGT model
(BASELINE config 1 family) against the reference's own outputs
(tests/golden/irls_sim3*.npz) and the CPU oracle."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import alignment_oracle as AO  # noqa: E402
from oracle import vggt_oracle as O  # noqa: E402


@pytest.fixture(scope="module")
def N():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from aligned_vggt import _native
    _native.lib()
    return _native


def _rel(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def test_irls_matches_reference_fixture(N, golden):
    from aligned_vggt.models.pointAligned_wrapped_vggt import irls_sim3_umeyama
    g = golden("irls_sim3")
    r, t, s = irls_sim3_umeyama(*(torch.from_numpy(g[k]).cuda() for k in ("src", "dst", "conf_src", "conf_dst")))
    assert _rel(r, g["r"]) < 1e-5 and _rel(t, g["t"]) < 1e-5 and abs(float(s) / float(g["s"]) - 1) < 1e-5


def test_irls_batched_matches_reference_fixture(N, golden):
    """Three problems (5% gross outliers, a sub-threshold confidence band) in
    ONE batched call."""
    g = golden("irls_sim3_batch")
    src = torch.stack([torch.from_numpy(g[f"src{b}"]) for b in range(3)]).cuda()
    dst = torch.stack([torch.from_numpy(g[f"dst{b}"]) for b in range(3)]).cuda()
    cs = torch.stack([torch.from_numpy(g[f"cs{b}"]) for b in range(3)]).cuda()
    cd = torch.stack([torch.from_numpy(g[f"cd{b}"]) for b in range(3)]).cuda()
    R, t, s = N.irls_sim3(src, dst, cs, cd)
    for b in range(3):
        assert _rel(R[b], g[f"r{b}"]) < 1e-5, b
        assert _rel(t[b], g[f"t{b}"]) < 1e-4, b
        assert abs(float(s[b]) / float(g[f"s{b}"]) - 1) < 1e-5, b


@pytest.mark.parametrize("npts_hw", [(2, 37, 50), (4, 130, 130)])
def test_irls_vs_oracle_large(N, npts_hw):
    nf, h, w = npts_hw
    gen = torch.Generator().manual_seed(nf * h)
    src = torch.randn(nf, h, w, 3, generator=gen) * 3 + torch.tensor([0.0, 0.0, 8.0])
    ang = 0.25
    R0 = torch.tensor([[np.cos(ang), 0, np.sin(ang)], [0, 1, 0], [-np.sin(ang), 0, np.cos(ang)]], dtype=torch.float32)
    dst = 1.3 * src @ R0.T + torch.tensor([0.5, -1.0, 2.0]) + 0.01 * torch.randn(src.shape, generator=gen)
    bad = torch.rand(src.shape[:-1], generator=gen) < 0.1
    dst[bad] += 4 * torch.randn(int(bad.sum()), 3, generator=gen)
    cs = 1 + 3 * torch.rand(src.shape[:-1], generator=gen)
    cd = 1 + 3 * torch.rand(src.shape[:-1], generator=gen)
    r_ref, t_ref, s_ref = AO.irls_sim3_umeyama(src, dst, cs, cd)
    R, t, s = N.irls_sim3(src[None].cuda(), dst[None].cuda(), cs[None].cuda(), cd[None].cuda())
    assert _rel(R[0], r_ref) < 1e-4 and _rel(t[0], t_ref) < 1e-4 and abs(float(s[0]) / float(s_ref) - 1) < 1e-4


def test_weighted_umeyama_direct(N):
    from aligned_vggt.models.pointAligned_wrapped_vggt import weighted_umeyama_sim3
    gen = torch.Generator().manual_seed(4)
    src = torch.randn(5000, 3, generator=gen)
    dst = 0.7 * src.flip(-1) + 1.0 + 0.01 * torch.randn(5000, 3, generator=gen)  # reflection-free permutation+scale
    w = torch.rand(5000, generator=gen)
    r_ref, t_ref, s_ref = AO.weighted_umeyama_sim3(src, dst, w)
    r, t, s = weighted_umeyama_sim3(src.cuda(), dst.cuda(), w.cuda())
    # the oracle (like the reference) reduces and decomposes in fp32; the kernel in fp64
    assert _rel(r, r_ref) < 1e-4 and _rel(t, t_ref) < 1e-4 and abs(float(s) / float(s_ref) - 1) < 1e-4
    r64, t64, s64 = AO.weighted_umeyama_sim3(src.double(), dst.double(), w.double())
    assert _rel(r, r64) < 2e-6 and _rel(t, t64) < 2e-6 and abs(float(s) / float(s64) - 1) < 2e-6


def test_sim3_points_and_scale(N, golden):
    g = golden("alignment_utils")
    pm = torch.from_numpy(g["pm"]).cuda()
    out = N.sim3_points(pm, torch.from_numpy(g["T"]).cuda(), torch.from_numpy(g["sc"]).cuda())
    np.testing.assert_allclose(out.cpu().numpy(), g["pm_out"], rtol=1e-5, atol=1e-5)
    x = torch.randn(3, 5, 7, 1, device="cuda")
    sc = torch.tensor([2.0, -0.5, 3.0], device="cuda")
    ref = x * sc.view(3, 1, 1, 1)
    N.scale_(x, sc)
    torch.testing.assert_close(x, ref)


@pytest.fixture(scope="module")
def point_model():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from aligned_vggt.models.pointAligned_wrapped_vggt import VGGT
    from aligned_vggt.utils.synthetic import condition_pose_outputs_, synthetic_init_
    m = VGGT(enable_track=False)
    synthetic_init_(m, seed=5)
    condition_pose_outputs_(m)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    return m.cuda().eval(), sd


def test_point_aligned_state_dict_names(point_model):
    m, sd = point_model
    for k in ("aggregator.camera_token", "point_head.scratch.output_conv2.2.weight", "depth_head.projects.0.weight",
              "camera_head.trunk.0.attn.qkv.weight"):
        assert k in sd, k


def test_point_aligned_two_chunks_vs_oracle(point_model):
    """Config-1 family: two overlapping chunks; the second is aligned to the
    first by the GPU IRLS.  HIP (bf16 aggregator) vs the oracle's bf16
    emulation, with the oracle's own bf16-vs-fp32 spread as the yardstick."""
    m, sd = point_model
    from aligned_vggt.utils.synthetic import synthetic_images
    S, ov, H, W = 3, 1, 42, 56
    imgs = synthetic_images(1, 2 * S - ov, H, W, seed=8)
    chunks = O.generate_chunks(imgs.shape[1], S, ov)
    ref = ref32 = got = None
    for ids in chunks:
        x = imgs[:, ids]
        ref = AO.point_aligned_forward(sd, x, ov, ref, bf16=True)
        ref32 = AO.point_aligned_forward(sd, x, ov, ref32, bf16=False)
        got = m(x.cuda(), ov, got)
    torch.cuda.synchronize()
    for k in ("world_points", "depth", "pose_enc"):
        for a, b, c in zip(got[k], ref[k], ref32[k]):
            e_hip, e_ref = _rel(a, b), _rel(c, b)
            print(k, e_hip, e_ref)
            assert e_hip < max(3e-2, 1.5 * e_ref), (k, e_hip, e_ref)


# configs[0] bars: ~2-3x the MI355X measurement (round 4: points 3.0e-4, confidences 3e-6,
# depth 5.7e-4 on the aligned chunk -- the Sim(3) scale from the IRLS, whose reductions run
# in fp64 on the GPU but in fp32 over 1.07 M points in the reference / oracle -- and 3.7e-6
# on the first); the camera-head pose encodings of the random-init model amplify bf16 token
# rounding (measured 2.0e-2 vs the oracle's own bf16-vs-fp32 spread of 1.7-1.9e-2) and keep
# the spread-relative bar
CONFIG0_BARS = {"world_points": 1e-3, "world_points_conf": 1e-4, "depth": 2e-3, "depth_conf": 1e-4}


def test_point_aligned_config0_full_size_two_chunks(N):
    """BASELINE configs[0] at its size: 8-frame 518 x 518 chunks through the
    point-aligned VGGT (pointAligned_wrapped_vggt.py:34-157), reduced depth
    (4 frame/global blocks, 1 DINOv2 block; the DPT heads read all four), plus
    a second chunk overlapping by 4 frames, so the GPU IRLS (:219-305) fits a
    Sim(3) between full-size point maps (4 x 518^2 = 1.07 M points) and the
    point maps / poses / depths are re-expressed through it.  HIP vs the
    oracle's bf16-mixed emulation; the oracle's own fp32-vs-bf16 spread is
    printed beside every error."""
    import os
    from aligned_vggt.backbone.aggregator import Aggregator
    from aligned_vggt.models.pointAligned_wrapped_vggt import VGGT
    from aligned_vggt.utils.synthetic import condition_pose_outputs_, synthetic_images, synthetic_init_
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    m = VGGT(enable_track=False)
    m.aggregator = Aggregator(depth=4, dino_depth=1)
    m.intermediate_layer_indices = [0, 1, 2, 3]
    synthetic_init_(m, seed=11)
    condition_pose_outputs_(m)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.cuda().eval()
    S, ov, H, W = 8, 4, 518, 518
    imgs = synthetic_images(1, 2 * S - ov, H, W, seed=1234)
    chunks = O.generate_chunks(imgs.shape[1], S, ov)
    assert [len(c) for c in chunks] == [8, 8]
    agg_kw = {"keep": (0, 1, 2, 3), "depth": 4, "dino_depth": 1}
    ref = ref32 = got = None
    for ids in chunks:
        x = imgs[:, ids]
        with torch.no_grad():
            ref = AO.point_aligned_forward(sd, x, ov, ref, bf16=True, agg_kwargs=agg_kw)
            ref32 = AO.point_aligned_forward(sd, x, ov, ref32, bf16=False, agg_kwargs=agg_kw)
        got = m(x.cuda(), ov, got)
    torch.cuda.synchronize()
    assert got["world_points"][-1].shape == (1, 8, 518, 518, 3)
    assert got["depth"][-1].shape == (1, 8, 518, 518, 1)
    worst = {}
    for k in ("world_points", "world_points_conf", "depth", "depth_conf", "pose_enc"):
        for c, (a, b, r32) in enumerate(zip(got[k], ref[k], ref32[k])):
            assert torch.isfinite(a).all(), k
            e_hip, e_ref = _rel(a, b), _rel(r32, b)
            print(f"configs[0] chunk {c} {k}: hip vs bf16 oracle {e_hip:.3e}, oracle fp32 vs bf16 {e_ref:.3e}")
            worst[k] = max(worst.get(k, 0.0), e_hip)
            assert e_hip < CONFIG0_BARS.get(k, max(3e-2, 1.5 * e_ref)), (k, c, e_hip, e_ref)
    print("configs[0] worst rel-L2:", worst)
