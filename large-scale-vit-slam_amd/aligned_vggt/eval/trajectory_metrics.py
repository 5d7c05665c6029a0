"""ATE / RPE (eval/trajectory_metrics.py:11-77 and :134-223 of the
reference), restated without the ``torchmetrics`` dependency, which is absent
from this image.

Same public surface: ``update(preds, target)`` with (N, 4, 4) camera-to-world
poses, ``compute()`` -> dict with the reference's keys, ``detailed`` flag and
RPE ``delta``; plus ``reset()`` and ``sync(group)``, the latter standing in for
torchmetrics' ``dist_reduce_fx="cat"`` (all ranks' error lists concatenated in
rank order).  Pinned by tests/golden/trajectory_metrics.npz, produced by the
reference's own update/compute bodies.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..utils.geometry import closed_form_inverse_se3
from ..utils.pose_enc import pose_encoding_to_extri_intri


def _cat_across_ranks(t: torch.Tensor, group=None) -> torch.Tensor:
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return t
    W = dist.get_world_size(group)
    n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
    ns = [torch.zeros_like(n) for _ in range(W)]
    dist.all_gather(ns, n, group=group)
    m = int(max(x.item() for x in ns))
    pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    outs = [torch.zeros_like(pad) for _ in range(W)]
    dist.all_gather(outs, pad, group=group)
    return torch.cat([o[: int(k.item())] for o, k in zip(outs, ns)], 0)


class AbsoluteTrajectoryError:
    """RMSE of camera-centre differences (trajectory_metrics.py:11-77)."""

    def __init__(self, detailed: bool = False, **kwargs):
        self.detailed = detailed
        self.reset()

    def reset(self) -> None:
        self.errors = torch.tensor([], dtype=torch.float32)
        self.per_dim_errors = torch.tensor([], dtype=torch.float32)

    def update(self, preds: torch.Tensor, target: torch.Tensor) -> None:
        assert preds.shape == target.shape, "Preds and targets must have the same shape"
        assert preds.shape[-2:] == (4, 4), "Poses must be 4x4 matrices"
        err = preds[:, :3, 3] - target[:, :3, 3]
        trans = torch.linalg.norm(err, dim=1)
        self.errors = torch.cat([self.errors, trans.detach().to(self.errors.device)])
        self.per_dim_errors = torch.cat([self.per_dim_errors, err.detach().to(self.per_dim_errors.device)])

    def sync(self, group=None) -> None:
        self.errors = _cat_across_ranks(self.errors, group)
        self.per_dim_errors = _cat_across_ranks(self.per_dim_errors.reshape(-1, 3), group)

    def compute(self) -> dict:
        e, pd = self.errors, self.per_dim_errors
        rmse = torch.sqrt(torch.mean(e ** 2)).item()
        if not self.detailed:
            return {"ate_rmse": rmse}
        return {"ate_rmse": rmse, "ate_mean": torch.mean(e).item(), "ate_median": torch.median(e).item(),
                "ate_std": torch.std(e).item(), "ate_min": torch.min(e).item(), "ate_max": torch.max(e).item(),
                "ate_rmse_per_dim": torch.sqrt(torch.mean(pd ** 2, dim=0)).tolist()}

    __call__ = update


class RelativePoseError:
    """Translational / rotational RPE over frame pairs (i, i+delta)
    (trajectory_metrics.py:134-223); rotation error acos((tr R - 1)/2) in
    degrees in ``compute``."""

    def __init__(self, delta: int = 1, detailed: bool = False, **kwargs):
        self.delta = delta
        self.detailed = detailed
        self.reset()

    def reset(self) -> None:
        self.trans_errors = torch.tensor([], dtype=torch.float32)
        self.rot_errors = torch.tensor([], dtype=torch.float32)

    def update(self, preds: torch.Tensor, target: torch.Tensor) -> None:
        assert preds.shape == target.shape, "Preds and targets must have the same shape"
        assert preds.shape[-2:] == (4, 4), "Poses must be 4x4 matrices"
        if preds.shape[0] <= self.delta:
            return
        d = self.delta
        pred_rel = torch.linalg.inv(preds[:-d]) @ preds[d:]
        gt_rel = torch.linalg.inv(target[:-d]) @ target[d:]
        err = torch.linalg.inv(gt_rel) @ pred_rel
        trans = torch.linalg.norm(err[:, :3, 3], dim=1)
        tr = torch.sum(torch.diagonal(err[:, :3, :3], dim1=-2, dim2=-1), dim=1)
        rot = torch.acos(torch.clamp((tr - 1) / 2, -1.0, 1.0))
        self.trans_errors = torch.cat([self.trans_errors, trans.detach().to(self.trans_errors.device)])
        self.rot_errors = torch.cat([self.rot_errors, rot.detach().to(self.rot_errors.device)])

    def sync(self, group=None) -> None:
        self.trans_errors = _cat_across_ranks(self.trans_errors, group)
        self.rot_errors = _cat_across_ranks(self.rot_errors, group)

    def compute(self) -> dict:
        t, r = self.trans_errors, self.rot_errors
        have = len(t) > 0

        def f(fn, x, deg=False):
            if not have:
                return 0.0
            v = fn(x)
            return (torch.rad2deg(v) if deg else v).item()
        out = {"rpe_trans_rmse": f(lambda x: torch.sqrt(torch.mean(x ** 2)), t),
               "rpe_rot_rmse": f(lambda x: torch.sqrt(torch.mean(x ** 2)), r, True)}
        if not self.detailed:
            return out
        for name, fn in (("mean", torch.mean), ("median", torch.median), ("std", torch.std), ("min", torch.min),
                         ("max", torch.max)):
            out[f"rpe_trans_{name}"] = f(fn, t)
            out[f"rpe_rot_{name}"] = f(fn, r, True)
        return {k: out[k] for k in ("rpe_trans_rmse", "rpe_trans_mean", "rpe_trans_median", "rpe_trans_std",
                                    "rpe_trans_min", "rpe_trans_max", "rpe_rot_rmse", "rpe_rot_mean",
                                    "rpe_rot_median", "rpe_rot_std", "rpe_rot_min", "rpe_rot_max")}

    __call__ = update


def poses_c2w_from_predictions(pose_enc: torch.Tensor, extrinsics: torch.Tensor, image_hw,
                               device: Optional[torch.device] = None):
    """The pose half of training_metrics.py:233-260 (prepare_data_for_metrics):
    pose encodings (B,S,9) and GT w2c extrinsics (B,S,3,4) -> 4x4 c2w (B,S,4,4)."""
    B, S = extrinsics.shape[:2]
    pred_extr, _ = pose_encoding_to_extri_intri(pose_enc.float(), image_size_hw=image_hw)
    pred = closed_form_inverse_se3(pred_extr.reshape(B * S, 3, 4)).reshape(B, S, 4, 4)
    gt = closed_form_inverse_se3(extrinsics.float().reshape(B * S, 3, 4)).reshape(B, S, 4, 4)
    if device is not None:
        pred, gt = pred.to(device), gt.to(device)
    return pred, gt
