"""CPU parity of the evaluation / GT-alignment utilities against fixtures
produced by the reference's own code (tests/golden/gen_golden.py):
ATE / RPE (eval/trajectory_metrics.py), Umeyama / LSE scale / Sim(3)
application (aligned_vggt/utils/alignment.py) and the GT scale alignments."""
import numpy as np
import pytest
import torch

from aligned_vggt.eval import AbsoluteTrajectoryError, RelativePoseError
from aligned_vggt.utils import alignment as A


def test_ate_matches_reference(golden):
    g = golden("trajectory_metrics")
    pred, gt = torch.from_numpy(g["pred"]), torch.from_numpy(g["gt"])
    for det in (0, 1):
        m = AbsoluteTrajectoryError(detailed=bool(det))
        m.update(pred[:25], gt[:25])
        m.update(pred[25:], gt[25:])
        out = m.compute()
        keys = [k[len(f"ate_{det}_"):] for k in g if k.startswith(f"ate_{det}_")]
        assert sorted(out) == sorted(keys)
        for k in keys:
            np.testing.assert_allclose(np.asarray(out[k]), g[f"ate_{det}_{k}"], rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("delta", [1, 3])
def test_rpe_matches_reference(golden, delta):
    g = golden("trajectory_metrics")
    pred, gt = torch.from_numpy(g["pred"]), torch.from_numpy(g["gt"])
    m = RelativePoseError(delta=delta, detailed=True)
    m.update(pred, gt)
    m.update(pred[:2], gt[:2])
    out = m.compute()
    keys = [k[len(f"rpe_{delta}_"):] for k in g if k.startswith(f"rpe_{delta}_")]
    assert list(out) == keys  # same key order as the reference dict
    for k in keys:
        np.testing.assert_allclose(out[k], g[f"rpe_{delta}_{k}"], rtol=2e-5, atol=1e-6)


def test_ate_rpe_known_answers():
    N = 10
    gt = torch.eye(4).repeat(N, 1, 1)
    gt[:, 0, 3] = torch.arange(N, dtype=torch.float32)
    pred = gt.clone()
    pred[:, 1, 3] += 0.5  # constant offset: ATE = 0.5, RPE = 0
    a = AbsoluteTrajectoryError()
    a.update(pred, gt)
    assert abs(a.compute()["ate_rmse"] - 0.5) < 1e-6
    r = RelativePoseError()
    r.update(pred, gt)
    out = r.compute()
    assert out["rpe_trans_rmse"] < 1e-6 and out["rpe_rot_rmse"] < 1e-2
    empty = RelativePoseError(delta=20)
    empty.update(pred, gt)
    assert empty.compute() == {"rpe_trans_rmse": 0.0, "rpe_rot_rmse": 0.0}


def test_umeyama_scale_sim3_match_reference(golden):
    g = golden("alignment_utils")
    r, t, c = A.umeyama(g["x"], g["y"])
    np.testing.assert_allclose(r, g["r"], atol=1e-10)
    np.testing.assert_allclose(t, g["t"], atol=1e-10)
    np.testing.assert_allclose(c, g["c"], rtol=1e-12)
    np.testing.assert_allclose(A.scale_lse_solver(g["x"].reshape(-1), g["y"].reshape(-1)), g["s"], rtol=1e-12)
    pm = A.apply_sim3_alignment_on_point_maps(torch.from_numpy(g["pm"]), torch.from_numpy(g["T"]),
                                              torch.from_numpy(g["sc"]))
    np.testing.assert_allclose(pm.numpy(), g["pm_out"], rtol=1e-6, atol=1e-6)
    c2w = A.apply_sim3_alignment_on_c2w(torch.from_numpy(g["poses"]).clone(), torch.from_numpy(g["T"]),
                                        torch.from_numpy(g["sc"]))
    np.testing.assert_allclose(c2w.numpy(), g["c2w_out"], rtol=1e-6, atol=1e-6)


def test_horn_agrees_with_umeyama(golden):
    g = golden("alignment_utils")
    r, t, s = A.methodOfHorn(g["x"], g["y"])
    r2, t2, c2 = A.umeyama(g["x"], g["y"])
    np.testing.assert_allclose(r, r2, atol=1e-6)
    assert abs(float(s) - c2) < 1e-3


def _preds(g):
    return {k[3:]: torch.from_numpy(g[k]).clone() for k in g if k.startswith("in_")}


@pytest.mark.parametrize("name", ["scale_poses", "scale_poses_w3", "frame_scale", "depth_scale", "chunk_scale"])
def test_gt_scale_alignments_match_reference(golden, name):
    g = golden("scale_alignment")
    extr = torch.from_numpy(g["extr"])
    p = _preds(g)
    if name == "scale_poses":
        A.scale_alignment_from_poses(p, {"extrinsics": extr})
    elif name == "scale_poses_w3":
        A.scale_alignment_from_poses(p, {"extrinsics": extr}, 3)
    elif name == "frame_scale":
        A.per_frame_scale_alignment_from_poses(p, {"extrinsics": extr})
    elif name == "depth_scale":
        A.scale_align_from_depths(p, {"depths": torch.from_numpy(g["depths"])[..., None],
                                      "point_masks": torch.from_numpy(g["mask"])})
    else:
        ch = {k: [v[:, :3].clone(), v[:, 3:].clone()] for k, v in p.items()}
        A.per_chunk_scale_alignment_from_poses(ch, {"extrinsics": [extr[:, :3], extr[:, 3:]]})
        p = {k: torch.cat(v, 1) for k, v in ch.items() if k != "alignment_scales_per_chunk"}
        p["alignment_scales"] = torch.stack(ch["alignment_scales_per_chunk"])
    for k in ("pose_enc", "depth", "world_points"):
        np.testing.assert_allclose(p[k].numpy(), g[f"{name}_{k}"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(np.asarray(p["alignment_scales"], dtype=np.float64), g[f"{name}_scales"], rtol=1e-6)


def _sync_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(3)
        pred = torch.eye(4).repeat(12, 1, 1)
        pred[:, :3, 3] = torch.randn(12, 3, generator=g)
        gt = torch.eye(4).repeat(12, 1, 1)
        lo, hi = (0, 7) if rank == 0 else (7, 12)  # ragged shards
        ate, rpe = AbsoluteTrajectoryError(), RelativePoseError()
        ate.update(pred[lo:hi], gt[lo:hi])
        rpe.update(pred[lo:hi], gt[lo:hi])
        ate.sync()
        rpe.sync()
        if rank == 0:
            q.put({**ate.compute(), **rpe.compute()})
    finally:
        dist.destroy_process_group()


def test_metric_sync_across_ranks():
    """sync() = torchmetrics' dist_reduce_fx='cat': the two ragged shards
    reduce to the metric over the concatenated error lists."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_sync_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = q.get(timeout=120)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    g = torch.Generator().manual_seed(3)
    pred = torch.eye(4).repeat(12, 1, 1)
    pred[:, :3, 3] = torch.randn(12, 3, generator=g)
    gt = torch.eye(4).repeat(12, 1, 1)
    ate, rpe = AbsoluteTrajectoryError(), RelativePoseError()
    ate.update(pred, gt)
    rpe.update(pred[:7], gt[:7])
    rpe.update(pred[7:], gt[7:])
    ref = {**ate.compute(), **rpe.compute()}
    for k in ref:
        assert abs(got[k] - ref[k]) < 1e-6, (k, got, ref)
