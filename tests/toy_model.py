"""A small deterministic stand-in for FeatureAlignedVGGT with the same
encode_chunk / align_chunk / forward protocol and context semantics (CPU
arithmetic, real dependence on the previous chunk's overlap tokens, memory and
poses).  Used by the gloo multi-process pipeline tests and by
``bench.py --workload selftest`` (the CPU check of the multi-rank launcher)."""
import torch

from aligned_vggt.models.featureAligned_vggt import merge_results

P1, C, NMEM, DEC = 7, 16, 3, 8


class ToyAlignModel:
    """Same protocol as FeatureAlignedVGGT (encode_chunk / align_chunk /
    forward + reference context semantics), tiny CPU arithmetic with a real
    dependence on the previous chunk's overlap tokens, memory and poses."""

    point_head = None

    def encode_chunk(self, images, dense=True):
        B, S = images.shape[:2]
        f = images.mean(dim=(2, 3, 4))  # (B, S)
        tok = f[:, :, None, None] * torch.arange(1, P1 * C + 1, dtype=torch.float32).view(1, 1, P1, C) / 100
        enc = {"images": images, "tok": tok}
        return self.encode_dense(enc) if dense else enc

    def encode_dense(self, enc):
        images = enc["images"]
        enc["depth"] = images[:, :, :1].permute(0, 1, 3, 4, 2) * 2
        enc["depth_conf"] = images[:, :, 1] + 1
        return enc

    def ship_spec(self, B, S, H, W):
        return {"tok": (B, S, P1, C)}

    def ship_payload(self, enc):
        return {"tok": enc["tok"]}

    def enc_from_ship(self, t, B, S, H, W):
        return {"images": torch.zeros(1).expand(B, S, 3, H, W), "tok": t["tok"]}

    def scale_dense(self, enc, sim3):
        B = enc["depth"].shape[0]
        return {"depth": enc["depth"] * sim3[..., -1].view(B, 1, 1, 1, 1), "depth_conf": enc["depth_conf"]}

    def align_chunk(self, enc, num_overlap, context=None):
        tok = enc["tok"].clone()
        B, S = tok.shape[:2]
        ov = num_overlap if S > num_overlap else S - 1
        if context is not None:
            prev = context["overlap_tokens"]
            tok = tok + prev.mean(dim=1, keepdim=True) * 0.5
            mem = context["memory_tokens"][-1] * 0.9 + tok.mean() * 0.1
            base = context["pose_enc"][-1][:, -ov:].mean(dim=1, keepdim=True)
        else:
            mem = torch.ones(B, NMEM, DEC)
            base = torch.zeros(B, 1, 9)
        pose = base + tok.mean(dim=(2, 3))[..., None] * torch.arange(9, dtype=torch.float32)
        sim3 = tok.mean(dim=(1, 2, 3))[:, None, None].expand(B, 1, 8).clone()
        fse3 = tok[:, 1:].mean(dim=(2, 3))[..., None].expand(B, S - 1, 7).clone()
        scale = sim3[..., -1]
        dense = "depth" in enc  # else the pipeline scales it after encode_dense (scale_dense)
        depth = enc["depth"] * scale.view(B, 1, 1, 1, 1) if dense else None
        pred = {"overlap_tokens": torch.cat([tok[:, :1], tok[:, -ov:]], 1).contiguous()}
        if context is None:
            pred.update(pose_enc=[pose], chunk_sim3_alignment_enc=sim3, frame_se3_alignment_enc=fse3,
                        memory_tokens=[mem])
            if dense:
                pred.update(depth=[depth], depth_conf=[enc["depth_conf"]])
        else:
            context.setdefault("pose_enc", []).append(pose)
            pred["pose_enc"] = context["pose_enc"]
            pred["chunk_sim3_alignment_enc"] = merge_results(context["chunk_sim3_alignment_enc"], sim3)
            pred["frame_se3_alignment_enc"] = merge_results(context["frame_se3_alignment_enc"], fse3)
            context.setdefault("memory_tokens", []).append(mem)
            pred["memory_tokens"] = context["memory_tokens"]
            for k, v in ((("depth", depth), ("depth_conf", enc["depth_conf"])) if dense else ()):
                context.setdefault(k, []).append(v)
                pred[k] = context[k]
        return pred

    def __call__(self, images, num_overlap, context=None, gt_poses=None):
        return self.align_chunk(self.encode_chunk(images), num_overlap, context)
