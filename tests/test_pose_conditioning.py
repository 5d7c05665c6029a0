"""Why the composed pose translations carry percent-level errors in every
bf16-tier parity test ("pose_T back under ~1e-2 once T
is conditioned, or the error budget showing why not").

The camera head reads ONE token per frame, the camera token of the last kept
layer (VGGT camera_head.py; featureAligned_vggt.py:106), whose residual
stream starts from a 1e-6-scale learned token: bf16 rounding of the blocks'
outputs is large against its own norm, so its bf16-vs-fp32 error is about
twice the kept layer's average.  The random-init head (4 refinement
iterations x 4 trunk blocks, its output fed back through embed_pose)
multiplies that by 2-4 in the translations, and featureAligned_vggt.py:96-143
then re-centres every chunk on its first frame.  With the translation bias of
``condition_pose_outputs_(translation=...)`` |T| is ~1 (no longer near zero),
and the error is still ~2.5e-2 in the reference's OWN numerics (bf16-mixed vs
fp32), measured here on the CPU oracle alone -- the floor every HIP pose bar
inherits.  Parity unpinned in the VGGT-internal part (SPEC_ASSUMPTIONS.md);
the re-centring is the reference's own code (pinned by tests/golden)."""
import torch

from oracle import vggt_oracle as O


def _recentred_T(enc, hw):
    extr, _ = O.pose_encoding_to_extri_intri(enc, hw)
    extr = torch.nn.functional.pad(extr, (0, 0, 0, 1))
    extr[..., 3, 3] = 1.0
    return (extr @ O.closed_form_inverse_se3(extr[:, 0]).unsqueeze(1))[:, 1:, :3, 3]


def _rel(a, b):
    return ((a - b).norm() / b.norm()).item()


def test_camera_head_translation_condition_number(monkeypatch):
    from aligned_vggt.backbone.aggregator import Aggregator
    from aligned_vggt.models import featureAligned_vggt as FAmod
    from aligned_vggt.models.featureAligned_vggt import FeatureAlignedVGGT
    from aligned_vggt.utils.synthetic import condition_pose_outputs_, synthetic_images, synthetic_init_
    torch.set_num_threads(max(1, min(8, torch.get_num_threads())))
    monkeypatch.setattr(FAmod, "Aggregator", lambda **kw: Aggregator(depth=4, dino_depth=1, **kw))
    m = FeatureAlignedVGGT(enable_point=False, enable_depth=False, enable_track=False, num_memory_tokens=8)
    synthetic_init_(m, seed=17)  # the model of test_gpu_fullsize.py::test_vkitti_sequence_ate_rpe_parity
    condition_pose_outputs_(m, translation=0.25)
    sd = {k: v.detach() for k, v in m.state_dict().items() if k.startswith(("aggregator.", "camera_head."))}
    del m
    S, H, W = 8, 154, 518
    hw = (H, W)
    imgs = synthetic_images(1, S, H, W, seed=41)
    kw = {"keep": (3,), "depth": 4, "dino_depth": 1}
    with torch.no_grad():
        tb, _ = O.aggregator(sd, imgs, bf16=True, **kw)
        tf, _ = O.aggregator(sd, imgs, bf16=False, **kw)
        tok_err = _rel(tb[-1][:, :, 0], tf[-1][:, :, 0])  # the camera tokens the head reads
        all_err = _rel(tb[-1], tf[-1])  # every token of the kept layer
        enc_b, enc_f = O.camera_head(sd, tb)[-1], O.camera_head(sd, tf)[-1]
        T_b, T_f = _recentred_T(enc_b, hw), _recentred_T(enc_f, hw)
        raw_T = _rel(enc_f[..., :3], enc_b[..., :3])
        rec_T = _rel(T_f, T_b)
        quat = _rel(enc_f[..., 3:7], enc_b[..., 3:7])
        # the same map under isotropic noise of the bf16 token error's size (4 draws)
        g = torch.Generator().manual_seed(0)
        amp = []
        for _ in range(4):
            t = [x.clone() for x in tb]
            c = t[-1][:, :, 0]
            n = torch.randn(c.shape, generator=g)
            t[-1][:, :, 0] = c + n * (tok_err * c.norm() / n.norm())
            amp.append(_rel(_recentred_T(O.camera_head(sd, t)[-1], hw), T_b) / tok_err)
    print(f"kept-layer bf16-vs-fp32 error {all_err:.2e}; camera-token error {tok_err:.2e} -> raw T {raw_T:.2e}, "
          f"re-centred T {rec_T:.2e}, quat {quat:.2e}; re-centred T amplification under same-size noise: "
          + ", ".join(f"{a:.1f}" for a in amp) + f"; |T| raw {enc_b[..., :3].norm(dim=-1).mean():.3f}, "
          f"re-centred {T_b.norm(dim=-1).mean():.3f}")
    # measured (8 frames of 154 x 518): kept layer 4.0e-3 on average, but the camera
    # token -- whose residual stream starts from a 1e-6-scale learned token, so bf16
    # rounding of the layers' outputs is large against its own norm -- 8.2e-3; the
    # re-centred translations 2.5e-2 (3.1x the camera-token error; 2.4-4.4x under
    # isotropic noise of that size), quaternions 1.1e-2.  So bf16-mixed autocast itself
    # puts the composed translations at percent level, and a 1e-2 bar on pose_T would
    # fail the reference's own bf16 run against its fp32 one.
    assert tok_err > 1.5 * all_err, (tok_err, all_err)
    assert rec_T > 1e-2 and rec_T > 2 * tok_err and min(amp) > 1.5, (rec_T, tok_err, amp)
