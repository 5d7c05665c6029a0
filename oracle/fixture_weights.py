"""Deterministic fixture weights and inputs -- TEST INFRASTRUCTURE ONLY.

The golden fixtures of the reference-authored alignment path
(tests/golden/ref_*.npz, written by tests/golden/gen_golden.py from the
reference's own AlignmentHead / CrossAttentionBlock / FeatureAlignedVGGT) do
not store their weights or inputs: the 1024-wide alignment head alone has
~60M parameters.  Both the generator (which loads them into the reference's
modules) and the tests (oracle state dicts, the HIP model) regenerate them
from the rule below: numpy PCG64 streams seeded by (seed, crc32(name)), stable
across machines and numpy / torch versions.

The rule is chosen for sensitivity, not to mimic a trained model: LayerScale
gammas of ~0.1 (the reference init is 0.01, which would hide the blocks behind
the residual), unit-scale alignment tokens (reference init 1e-6), linear
weights of std 0.7/sqrt(fan_in), and the Sim(3)/SE(3) decoders biased towards
the identity quaternion so the rotations they emit are well conditioned.
"""
from __future__ import annotations

import zlib
from typing import Dict, Iterable, Mapping, Tuple

import numpy as np
import torch


def _rng(seed: int, name: str) -> np.random.Generator:
    return np.random.default_rng([int(seed) & 0x7FFFFFFF, zlib.crc32(name.encode())])


def fixture_value(name: str, shape: Tuple[int, ...], seed: int) -> np.ndarray:
    """The fixture value of parameter ``name`` (float32, ``shape``)."""
    g = _rng(seed, name)
    shape = tuple(int(s) for s in shape)
    parts = name.split(".")
    leaf = parts[-1]
    owner = parts[-2] if len(parts) > 1 else ""
    r = g.standard_normal(shape)
    if leaf == "gamma":  # LayerScale
        v = 0.1 * (1.0 + 0.2 * r)
    elif leaf == "per_frame_alignment_token":
        v = 0.5 * r
    elif leaf == "memory_token":  # (1, N, D): orthonormal rows (alignment_head.py:211-214)
        n, d = shape[-2], shape[-1]
        q, _ = np.linalg.qr(g.standard_normal((d, n)))
        v = (q.T / np.linalg.norm(q.T, axis=-1, keepdims=True)).reshape(shape)
    elif leaf == "alpha":
        v = np.full(shape, 0.3)
    elif len(shape) == 1 and "norm" in owner and leaf == "weight":
        v = 1.0 + 0.1 * r
    elif len(shape) == 1 and "norm" in owner and leaf == "bias":
        v = 0.05 * r
    elif len(shape) == 1:  # linear biases
        v = 0.02 * r
        if name.endswith(("chunk_sim3_decoder.fc2.bias", "frame_se3_decoder.fc2.bias")):
            v[6] = 1.0  # quaternion w (scalar-last): rotations near the identity
    elif len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        v = (0.7 / np.sqrt(fan_in)) * r
    else:  # 0-d
        v = 0.1 * r
    return np.asarray(v, dtype=np.float32)


def fixture_state_dict(named_shapes: Iterable[Tuple[str, Tuple[int, ...]]], seed: int) -> Dict[str, torch.Tensor]:
    return {n: torch.from_numpy(fixture_value(n, s, seed)) for n, s in named_shapes}


@torch.no_grad()
def load_fixture_weights_(module: torch.nn.Module, seed: int, prefix: str = "") -> torch.nn.Module:
    """Overwrite every parameter of ``module`` with its fixture value; the
    value is keyed by ``prefix + name`` so a sub-module gets the same numbers as
    inside its parent tree."""
    for n, p in module.named_parameters():
        p.copy_(torch.from_numpy(fixture_value(prefix + n, tuple(p.shape), seed)).to(p.device, p.dtype))
    return module


def fixture_tensor(tag: str, shape: Tuple[int, ...], seed: int, kind: str = "normal") -> torch.Tensor:
    """Deterministic fixture inputs: ``normal`` N(0,1), ``uniform`` [0,1),
    ``positive`` in [0.5, 2)."""
    g = _rng(seed, "input:" + tag)
    if kind == "normal":
        v = g.standard_normal(tuple(shape))
    elif kind == "uniform":
        v = g.random(tuple(shape))
    elif kind == "positive":
        v = 0.5 + 1.5 * g.random(tuple(shape))
    else:
        raise ValueError(kind)
    return torch.from_numpy(np.asarray(v, dtype=np.float32))


def fixture_pose_enc(tag: str, B: int, S: int, seed: int) -> torch.Tensor:
    """Well-conditioned camera pose encodings (B, S, 9) = [T(3), quat xyzw (4)
    near the identity, FoV h/w ~1 rad] -- the stub camera head's output."""
    g = _rng(seed, "pose:" + tag)
    t = g.standard_normal((B, S, 3)) * 0.5
    q = g.standard_normal((B, S, 4)) * 0.1
    q[..., 3] += 1.0
    q /= np.linalg.norm(q, axis=-1, keepdims=True)
    fov = 0.9 + 0.2 * g.random((B, S, 2))
    return torch.from_numpy(np.concatenate([t, q, fov], -1).astype(np.float32))


# ----------------------------------------------------------------------------
# case tables of the reference alignment-path fixtures (tests/golden/ref_*.npz)
# ----------------------------------------------------------------------------
FIX_SEED = 2024
FIX_HW = (42, 56)  # 3 x 4 patches: P = 5 + 12 = 17 aggregator tokens per frame

# (case, head, B, S, next_num_overlap, previous case feeding overlap / memory);
# head m8 = 8 memory tokens, m0 = none
ALIGN_CASES = [("a1", "m8", 1, 3, 1, None), ("a2", "m8", 1, 3, 1, "a1"), ("a3", "m8", 1, 2, 1, "a2"),
               ("b1", "m8", 2, 5, 2, None), ("b2", "m8", 2, 5, 2, "b1"),
               ("c1", "m0", 1, 5, 2, None), ("c2", "m0", 1, 5, 2, "c1")]

# (run, frames N, chunk width, overlap, with gt_poses)
FA_RUNS = [("ov2", 12, 5, 2, False), ("ov1", 8, 3, 1, False), ("gt", 8, 4, 2, True)]


# training-gradient fixture (tests/golden/ref_train_grads.npz): two chunks of S
# frames through the alignment head with memory, next overlap ov
TRAIN_CASE = {"S": 4, "ov": 2}


def train_inputs():
    """(chunk 1, chunk 2) layer-23 tokens (1, S, P, 2048) of the gradient fixture."""
    P = fix_tokens_per_frame()
    S = TRAIN_CASE["S"]
    return tuple(fixture_tensor(f"tr.tok{i}", (1, S, P, 2048), FIX_SEED) for i in (1, 2))


def train_loss(o1, o2):
    """The gradient fixture's loss: a fixed linear functional of both chunks'
    (chunk_sim3, frame_se3, memory, new_overlap_tokens) outputs (on o1's device)."""
    (cs1, fs1, m1, _), (cs2, fs2, m2, nov2) = o1, o2
    S, ov = TRAIN_CASE["S"], TRAIN_CASE["ov"]
    P = fix_tokens_per_frame()
    dev = cs1.device
    w = {k: fixture_tensor("tr.w" + k, shp, FIX_SEED).to(dev) for k, shp in
         (("cs", (1, 1, 8)), ("fs", (1, S - 1, 7)), ("mem", (1, 8, 512)), ("ov", (1, ov + 1, P + 1, 1024)))}
    return ((cs1.float() * w["cs"]).sum() + (fs1.float() * w["fs"]).sum() + (cs2.float() * w["cs"]).sum()
            + 2 * (fs2.float() * w["fs"]).sum() + (m2.float() * w["mem"]).sum() + 1e-2 * (nov2.float() * w["ov"]).sum())


GRAD_FULL_MAX = 8192  # parameters up to this size are stored whole
GRAD_SAMPLES = 512


def grad_indices(name: str, numel: int) -> np.ndarray:
    """Fixed sampled flat indices of a large parameter's gradient."""
    return np.sort(_rng(FIX_SEED, "gradidx:" + name).choice(numel, GRAD_SAMPLES, replace=False))


def grad_sample(name: str, grad: torch.Tensor) -> Dict[str, np.ndarray]:
    """What the fixture keeps of one parameter gradient: ``full`` (small ones)
    or ``idx`` / ``val`` sampled entries plus the whole gradient's ``norm``."""
    g = grad.detach().float().reshape(-1).cpu()
    out = {"norm": np.array(float(g.double().norm()), dtype=np.float64)}  # fp64: an fp32 norm over 4 M entries is off by ~1e-4
    if g.numel() <= GRAD_FULL_MAX:
        out["full"] = g.numpy().copy()
    else:
        idx = grad_indices(name, g.numel())
        out["val"] = g[torch.from_numpy(idx)].numpy().copy()
    return out


def _rel_l2(a, b) -> float:
    a, b = torch.as_tensor(a).double(), torch.as_tensor(b).double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


ZERO_GRAD = 1e-5  # every non-degenerate gradient of the fixture has norm > 1e-3


def grad_errors(g, prec: str, grads) -> Dict[str, float]:
    """Per-parameter rel-L2 of ``grads`` (name -> full gradient) against the
    fixture's stored entries (the whole gradient or its sampled indices) and
    the relative error of the gradient norm."""
    errs = {}
    for key in g:
        if not (key.startswith(prec + ".") and key.endswith(".norm")):
            continue
        name = key[len(prec) + 1:-len(".norm")]
        gr = grads[name].detach().double().reshape(-1).cpu()
        if float(g[key]) < ZERO_GRAD:
            # mathematically zero: q / k / norm1 of the decoder's frame-cross blocks attend
            # to ONE key (softmax == 1), so only rounding noise of order 1e-8 is stored
            errs[name] = 0.0 if float(gr.norm()) < ZERO_GRAD else 1.0
            continue
        if f"{prec}.{name}.full" in g:
            e = _rel_l2(gr, g[f"{prec}.{name}.full"])
        else:
            e = _rel_l2(gr[torch.from_numpy(grad_indices(name, gr.numel()))], g[f"{prec}.{name}.val"])
        en = abs(float(gr.norm()) / max(float(g[key]), 1e-30) - 1.0)
        errs[name] = max(e, en)
    return errs


def fix_tokens_per_frame() -> int:
    H, W = FIX_HW
    return 5 + (H // 14) * (W // 14)


def fa_feed(run: str, i: int, S: int) -> dict:
    """Stub encoder outputs for chunk i of a composition run: 4 kept token
    layers, camera pose encodings, depth / points and their confidences."""
    H, W = FIX_HW
    P = fix_tokens_per_frame()
    k = f"fa.{run}.{i}."
    return {
        "tokens": [fixture_tensor(k + f"tok{l}", (1, S, P, 2048), FIX_SEED) for l in range(4)],
        "pose_enc": fixture_pose_enc(k + "cam", 1, S, FIX_SEED),
        "depth": fixture_tensor(k + "depth", (1, S, H, W, 1), FIX_SEED, "positive"),
        "depth_conf": 1.0 + fixture_tensor(k + "dconf", (1, S, H, W), FIX_SEED, "positive"),
        "points": fixture_tensor(k + "pts", (1, S, H, W, 3), FIX_SEED),
        "points_conf": 1.0 + fixture_tensor(k + "pconf", (1, S, H, W), FIX_SEED, "positive"),
    }


def fa_gt_poses(run: str, i: int, S: int) -> torch.Tensor:
    """(1, S, 4, 4) ground-truth w2c poses of the chunk_gt composition run."""
    from . import vggt_oracle as O
    return O.pose_encoding_to_extri(fixture_pose_enc(f"fa.{run}.{i}.gt", 1, S, FIX_SEED)[..., :7])


def fa_images(run: str, N: int) -> torch.Tensor:
    H, W = FIX_HW
    return fixture_tensor(f"fa.{run}.images", (1, N, 3, H, W), FIX_SEED, "uniform")


def state_dict_shapes(sd: Mapping[str, torch.Tensor]):
    return [(k, tuple(v.shape)) for k, v in sd.items()]
