"""Drop-in ``LossModule`` (synth_sod/src/synth_sod/model_training/loss.py:236-275).

Accepts the reference's Hydra criterion list (``config/loss/focal_iou.yaml`` /
``bce_iou_ssim.yaml``: dicts with name / weight / target_key / output_key / loss._target_) and
runs the whole multi-mask loss — sigmoid, soft-IoU selection, argmax best mask, focal / BCE /
IoU / SSIM components with the decayed all-mask term and the aux MSE — as fused HIP kernels
(``s3od_mask_loss_fwd/bwd``; SSIM = separable 11x11 Gaussian filters over LDS tiles).  ``forward(outputs, targets, epoch) -> (loss, parts)`` with the
same part names as the reference (each reduced by ``.mean()``).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .autograd import mask_loss

_KIND = {
    "FocalLoss": "focal", "IoULoss": "iou", "BCELoss": "bce", "MSELoss": "mse", "SSIMLoss": "ssim", "DiceLoss": "dice",
}


def _kind(loss_cfg):
    t = loss_cfg["_target_"] if isinstance(loss_cfg, dict) else type(loss_cfg).__name__
    return _KIND.get(t.rsplit(".", 1)[-1], t)


class LossComponent:
    def __init__(self, name, weight, target_key, output_key, loss, add_sigmoid=True):
        assert weight >= 0.0, "Weight must be non-negative"
        self.name, self.weight, self.target_key, self.output_key = name, float(weight), target_key, output_key
        self.kind = _kind(loss)
        self.add_sigmoid = add_sigmoid

    @classmethod
    def from_dict(cls, c):
        return cls(c["name"], c["weight"], c["target_key"], c["output_key"], c["loss"])


class LossModule(nn.Module):
    def __init__(self, loss_config, full_mask_lambda: float = 0.01, decay_rate: float = 0.2):
        super().__init__()
        self.components = [LossComponent.from_dict(c) for c in loss_config]
        self.full_mask_lambda = float(full_mask_lambda)
        self.decay_rate = float(decay_rate)
        self.mask_components = [c for c in self.components if c.target_key == "masks" and c.output_key == "pred_masks"]
        self.aux_components = [c for c in self.components if c not in self.mask_components]
        w = {"focal": 0.0, "iou": 0.0, "bce": 0.0, "ssim": 0.0, "mse": 0.0}
        for c in self.mask_components:
            if c.kind not in ("focal", "iou", "bce", "ssim"):
                raise NotImplementedError(f"mask criterion {c.kind!r} is not fused on MI355X yet")
            w[c.kind] += c.weight
        for c in self.aux_components:
            if not (c.kind == "mse" and c.target_key == "gt_ious" and c.output_key == "pred_iou"):
                raise NotImplementedError(f"aux criterion {c.name!r}")
            w["mse"] += c.weight
        self.w = w
        self._names = {c.kind: c.name for c in self.components}

    def forward(self, outputs, targets, epoch: int):
        pm = outputs["pred_masks"]
        if pm.size(1) == 1:
            return self._single_mask(pm, outputs["pred_iou"], targets)
        lam = self.full_mask_lambda * math.exp(-self.decay_rate * epoch)
        cfg = {"w_focal": self.w["focal"], "w_iou": self.w["iou"], "w_bce": self.w["bce"], "w_ssim": self.w["ssim"],
               "w_mse": self.w["mse"], "lam": lam}
        loss, packed = mask_loss(pm, outputs["pred_iou"], targets["masks"], cfg)
        B, M = pm.shape[:2]
        parts = {"best_iou": packed[1], "gt_ious": packed[2]}
        for ci, kind in enumerate(("focal", "iou", "bce", "ssim")):
            if kind in self._names:
                n = self._names[kind]
                parts[f"{n}_best"] = packed[4 + 2 * ci]
                parts[f"{n}_full"] = packed[5 + 2 * ci]
        if "mse" in self._names:
            parts[self._names["mse"]] = packed[3]
        self.last_gt_ious = packed[16:16 + B * M].view(B, M)
        self.last_best = packed[16 + B * M:16 + B * M + B]
        return loss, parts


    def _single_mask(self, pm, pred_iou, targets):
        """MaskLossHandler.compute_single_mask_loss (loss.py:166-188; the dinol config, num_outputs=1):
        loss = sum_c w_c * mean(criterion_c(sigmoid(logits), masks)) over the [B,H,W] maps; no best-mask
        selection, no decayed all-mask term and no aux MSE (pred_iou gets no gradient).  This is the fused
        multi-mask kernel at M=1 with lambda=0 and w_mse=0.  Returns parts {criterion name: value}."""
        if self.w["ssim"]:
            # SSIMLoss(reduction='none') on a [B,H,W] map: F.conv2d reads it as unbatched [C=B,H,W] and
            # .mean((1,2,3)) has no dim 3 -- the reference raises here for every batch size
            raise RuntimeError("SSIMLoss on the single-mask [B,H,W] maps fails in the reference (loss.py:176-179, :74-75)")
        cfg = {"w_focal": self.w["focal"], "w_iou": self.w["iou"], "w_bce": self.w["bce"], "w_ssim": 0.0, "w_mse": 0.0,
               "lam": 0.0}
        loss, packed = mask_loss(pm, pred_iou.detach(), targets["masks"], cfg)
        parts = {}
        for ci, kind in enumerate(("focal", "iou", "bce")):
            if kind in self._names:
                parts[self._names[kind]] = packed[4 + 2 * ci]
        self.last_gt_ious = packed[16:16 + pm.shape[0]].view(-1, 1)
        self.last_best = None
        return loss, parts


FOCAL_IOU = [
    {"name": "focal_loss", "target_key": "masks", "output_key": "pred_masks", "weight": 20,
     "loss": {"_target_": "synth_sod.model_training.loss.FocalLoss", "reduction": "none"}},
    {"name": "iou_loss", "target_key": "masks", "output_key": "pred_masks", "weight": 1.0,
     "loss": {"_target_": "synth_sod.model_training.loss.IoULoss", "smooth": 1e-6, "reduction": "none"}},
    {"name": "mse_ious_loss", "target_key": "gt_ious", "output_key": "pred_iou", "weight": 0.05,
     "loss": {"_target_": "torch.nn.MSELoss"}},
]

BCE_IOU_SSIM = [
    {"name": "bce_loss", "target_key": "masks", "output_key": "pred_masks", "weight": 30,
     "loss": {"_target_": "torch.nn.BCELoss", "reduction": "none"}},
    {"name": "iou_loss", "target_key": "masks", "output_key": "pred_masks", "weight": 0.5,
     "loss": {"_target_": "synth_sod.model_training.loss.IoULoss", "smooth": 1e-6, "reduction": "none"}},
    {"name": "ssim_loss", "target_key": "masks", "output_key": "pred_masks", "weight": 10,
     "loss": {"_target_": "synth_sod.model_training.loss.SSIMLoss", "reduction": "none"}},
    {"name": "mse_ious_loss", "target_key": "gt_ious", "output_key": "pred_iou", "weight": 0.05,
     "loss": {"_target_": "torch.nn.MSELoss"}},
]
