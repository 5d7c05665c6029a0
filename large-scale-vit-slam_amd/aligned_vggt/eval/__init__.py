"""Trajectory evaluation (eval/trajectory_metrics.py of the reference) without torchmetrics."""
from .trajectory_metrics import AbsoluteTrajectoryError, RelativePoseError, poses_c2w_from_predictions  # noqa: F401
