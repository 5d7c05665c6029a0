"""Which sources a committed measurement was taken on.

Counter files under profiles/ (HBM traffic of the global attention, MFMA
utilisation of the aggregator step) are written on the GPU box, where the
tree has no .git.  They record ``source_fingerprint()`` -- a SHA-256 over the
HIP sources and the host modules that choose the aggregator's launches -- and
the git HEAD passed in as VGGT_GIT_HEAD; bench.py reports a committed counter
only while the fingerprint still matches the tree it runs from."""
from __future__ import annotations

import glob
import hashlib
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
_CSRC = os.path.join(os.path.dirname(_PKG), "csrc")


def aggregator_sources() -> list:
    files = sorted(glob.glob(os.path.join(_CSRC, "*")))
    files += [os.path.join(_PKG, f) for f in ("_native.py", "runtime.py")]
    files += sorted(glob.glob(os.path.join(_PKG, "backbone", "*.py")))
    return [f for f in files if os.path.isfile(f)]


def source_fingerprint() -> str:
    h = hashlib.sha256()
    for f in aggregator_sources():
        h.update(os.path.relpath(f, os.path.dirname(_PKG)).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def stamp() -> dict:
    """Provenance fields for a measurement file written now."""
    return {"source_fingerprint": source_fingerprint(), "git_head": os.environ.get("VGGT_GIT_HEAD")}
