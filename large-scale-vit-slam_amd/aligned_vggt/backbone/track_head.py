"""TrackHead placeholder.

The reference constructs VGGT's TrackHead when ``enable_track=True``
(featureAligned_vggt.py:30) but never calls it in any forward, and every
reference config disables it (test_featureAlignedVGGT_vkitti.yaml:103).  This
module exists so checkpoints that carry ``track_head.*`` keys (e.g. VGGT-1B)
load: it adopts whatever tensors the state dict holds under its prefix as
buffers.  It has no forward (OUT OF SCOPE).
"""
from __future__ import annotations

import torch
import torch.nn as nn


class TrackHead(nn.Module):
    def __init__(self, dim_in: int = 2048, patch_size: int = 14, **kwargs):
        super().__init__()
        self.dim_in = dim_in
        self.patch_size = patch_size

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        for k in list(state_dict.keys()):
            if k.startswith(prefix):
                name = k[len(prefix):].replace(".", "__")
                self.register_buffer(name, state_dict[k].detach().clone(), persistent=True)

    def forward(self, *args, **kwargs):
        raise NotImplementedError("TrackHead is not on the reference's feature-aligned path (never called)")
