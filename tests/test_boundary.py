"""The drop-in boundary against the reference's own module tree (SURVEY.md
§8b): parameter names / shapes of the alignment head, ``set_config``
(featureAligned_vggt.py:34-46), and the checkpoint load of run_model.py:388-394
(``model.``-prefixed Lightning state dict, prefix stripped, strict load).
The reference tree's names and shapes come from running the reference's own
AlignmentHead / FeatureAlignedVGGT (tests/golden/ref_*.json, gen_golden.py).
Construction on the meta device: no weights are materialised.  CPU only."""
import json
import os
from types import SimpleNamespace

import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def _shapes(module):
    return [[k, list(v.shape)] for k, v in module.state_dict().items()]


def test_alignment_head_tree_equals_reference():
    from aligned_vggt.heads.alignment_head import AlignmentHead
    ref = _json("ref_alignment_keys.json")
    for tag, nm in (("m8", 8), ("m0", 0)):
        with torch.device("meta"):
            h = AlignmentHead(in_dim=2048, patch_size=14, num_memory_tokens=nm, temporal_attention=True)
        got = _shapes(h)
        assert sorted(got) == sorted(ref[tag]), (tag, set(map(tuple, map(str, got))) ^ set(map(str, ref[tag])))
        # registration order too (state-dict iteration order = the reference's)
        assert [k for k, _ in got] == [k for k, _ in ref[tag]]


def test_set_config_matches_reference():
    """set_config rebuilds the alignment head from cfg and drops the disabled
    heads, exactly as the reference's (same resulting key set / shapes)."""
    from aligned_vggt.models.featureAligned_vggt import FeatureAlignedVGGT
    info = _json("ref_set_config.json")
    with torch.device("meta"):
        m = FeatureAlignedVGGT(enable_track=False)
    old = m.alignment_head
    m.set_config(SimpleNamespace(**info["cfg"]))
    assert m.alignment_head is not old  # re-created (fresh weights), as featureAligned_vggt.py:46
    assert m.enable_memory == info["enable_memory"]
    assert [n for n in ("camera_head", "point_head", "depth_head", "track_head") if getattr(m, n) is None] == \
        info["heads_none"]
    got = [[k, s] for k, s in _shapes(m) if k.startswith("alignment_head.")]
    assert got == info["keys"]  # the reference's stub encoders hold no parameters: alignment_head.* only
    assert not hasattr(m.alignment_head, "memory_token") and not hasattr(m.alignment_head, "gated_update")


def test_lightning_checkpoint_strict_load():
    """run_model.py:388-394: the Lightning checkpoint's state dict carries the
    LitModel's ``model.`` prefix; it is stripped with k.split('.', 1)[1] and
    loaded strictly.  Every key round-trips and nothing is missing."""
    from aligned_vggt.models.featureAligned_vggt import FeatureAlignedVGGT
    with torch.device("meta"):
        src = FeatureAlignedVGGT(enable_track=False)
        dst = FeatureAlignedVGGT(enable_track=False)
    ckpt = {"state_dict": {"model." + k: v for k, v in src.state_dict().items()}}
    sd = ckpt["state_dict"] if "state_dict" in ckpt else ckpt
    sd = {k.split(".", 1)[1]: v for k, v in sd.items()}
    res = dst.load_state_dict(sd, strict=True)
    assert not res.missing_keys and not res.unexpected_keys
    # the reference's freeze globs (test_featureAlignedVGGT_vkitti.yaml:80-83) select
    # exactly the encoder trees; the alignment head is what remains trainable
    names = [k for k, _ in src.named_parameters()]
    frozen = [k for k in names if any(g in k for g in ("aggregator", "camera_head", "depth_head"))]
    trainable = set(names) - set(frozen) - {k for k in names if k.startswith("point_head.")}
    assert trainable and all(k.startswith("alignment_head.") for k in trainable)
