"""Training-side predictor — drop-in for ``synth_sod.model_training.predictor.SODPredictor`` /
``PredictionResult`` (``synth_sod/src/synth_sod/model_training/predictor.py:22-41, 330-477``), the
model the evaluation loop (``compute_metrics.py:42-100``, ``train.py:30-55``) scores.

Device path: uint8 upload -> ``s3od_preprocess`` (LongestMaxSize + centred PadIfNeeded(fill 0) +
Normalize) -> DPTSegmentation forward -> ``s3od_sigmoid_unpad_resize`` over all N masks (sigmoid,
``remove_padding`` crop, antialiased bilinear resize to the original size).  Only the final masks
and the N IoU scores come back to the host, as in the reference.

Kept reference behaviour:
  * ``get_pad_info`` (:374-398) truncates ``int(new_w / aspect_ratio)`` and ``remove_padding``
    (:400-406) slices ``[pad:-pad]`` of the model output, which for an ``image_size`` that is not a
    multiple of 16 (the default 840) is 16*floor(S/16) pixels wide — the crop is applied to that
    output exactly as the reference slices it;
  * the letterbox itself follows albumentations 2.0.8 ``LongestMaxSize`` (``round(dim * scale)``)
    and ``PadIfNeeded`` (top/left = floor of half the pad), which can differ from ``get_pad_info``
    by a pixel — also the reference's behaviour.  albumentations / cv2 are not installed here, so
    the resize / normalise bit-parity is unpinned (the cv2 INTER_LINEAR emulation is shared with
    ``BackgroundRemoval``).
Checkpoints load with ``weights_only=True`` only: a Lightning checkpoint's model config must be a
plain dict (``hyper_parameters.config.model``); otherwise the variant is inferred from the weights.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from .checkpoint import model_state_dict, read_checkpoint
from .lightning_module import _get, instantiate
from .model import DPTSegmentation


@dataclass
class PredictionResult:
    binary_mask: np.ndarray
    soft_mask: np.ndarray
    all_masks: Optional[np.ndarray] = None
    all_ious: Optional[np.ndarray] = None

    @property
    def has_multiple_masks(self) -> bool:
        return self.all_masks is not None

    @property
    def num_masks(self) -> int:
        return len(self.all_masks) if self.has_multiple_masks else 1


def _model_from_weights(sd, compute_dtype):
    hidden = sd["encoder.embeddings.patch_embeddings.weight"].shape[0] if "encoder.embeddings.patch_embeddings.weight" in sd \
        else next(v.shape[0] for k, v in sd.items() if k.endswith("patch_embeddings.weight"))
    nm = next((v.shape[0] for k, v in sd.items() if k.endswith("classifier_head.4.weight")), 3)
    enc = "dinov3_large" if hidden == 1024 else "dinov3_base"
    return DPTSegmentation(num_classes=1, num_outputs=nm, encoder_name=enc, features=256, use_bn=True,
                           use_clstoken=False, compute_dtype=compute_dtype, init_seed=None)


class SODPredictor:
    def __init__(self, checkpoint_path, image_size: int = 840, device: str = "cuda", compute_dtype: str = "bf16"):
        if not str(device).startswith("cuda"):
            raise RuntimeError("SODPredictor runs on the MI355X HIP kernels only (device='cuda')")
        self.device = device
        self.image_size = int(image_size)
        self.model = self._load_checkpoint(checkpoint_path, compute_dtype)
        self.model.to(device)
        self.model.eval()

    def _load_checkpoint(self, checkpoint_path, compute_dtype):
        """predictor.py:358-372: Lightning checkpoint -> model from its config, else a saved model."""
        if isinstance(checkpoint_path, torch.nn.Module):
            return checkpoint_path
        ckpt = read_checkpoint(checkpoint_path)
        sd = model_state_dict(ckpt)
        cfg = _get(_get(ckpt.get("hyper_parameters"), "config"), "model") if isinstance(ckpt, dict) else None
        if cfg is not None and _get(cfg, "_target_") is not None:
            model = instantiate(cfg, compute_dtype=compute_dtype, init_seed=None)
        else:
            model = _model_from_weights(sd, compute_dtype)
        model.load_state_dict(sd)
        return model

    def get_pad_info(self, image: np.ndarray) -> dict:
        h, w = image.shape[:2]
        aspect_ratio = w / h
        if aspect_ratio > 1:
            new_w = self.image_size
            new_h = int(new_w / aspect_ratio)
            return {"height_pad": (self.image_size - new_h) // 2, "width_pad": 0, "original_size": (h, w),
                    "resized_size": (new_h, new_w)}
        new_h = self.image_size
        new_w = int(new_h * aspect_ratio)
        return {"height_pad": 0, "width_pad": (self.image_size - new_w) // 2, "original_size": (h, w),
                "resized_size": (new_h, new_w)}

    def letterbox(self, h: int, w: int):
        """albumentations LongestMaxSize(S) + PadIfNeeded(S, S, center): (new_h, new_w, top, left)."""
        S = self.image_size
        scale = S / float(max(h, w))
        nh, nw = (round(h * scale), round(w * scale)) if scale != 1.0 else (h, w)
        return nh, nw, max(0, (S - nh) // 2), max(0, (S - nw) // 2)

    @torch.no_grad()
    def predict(self, image: np.ndarray, threshold: float = 0.5) -> PredictionResult:
        from ._lib import lib, stream
        image = np.require(image, np.uint8, ["C", "W"])
        pad_info = self.get_pad_info(image)
        S = self.image_size
        H0, W0 = image.shape[:2]
        nh, nw, top, left = self.letterbox(H0, W0)
        img = torch.from_numpy(image).to(self.device)
        x = torch.empty((1, 3, S, S), dtype=torch.float32, device=self.device)
        lib()("s3od_preprocess", img, H0, W0, nh, nw, top, left, S, x, stream())
        out = self.model(x)
        logits = out["pred_masks"][0].contiguous()                 # [N, LH, LW]
        NM, LH, LW = logits.shape
        ph, pw = pad_info["height_pad"], pad_info["width_pad"]
        h, w = LH - 2 * ph, LW - 2 * pw                             # masks[:, ph:-ph, pw:-pw]
        tmp = torch.empty((NM, h, W0), dtype=torch.float32, device=self.device)
        masks = torch.empty((NM, H0, W0), dtype=torch.float32, device=self.device)
        lib()("s3od_sigmoid_unpad_resize", logits, NM, LH, LW, ph, pw, h, w, H0, W0, tmp, masks, stream())
        all_masks = masks.cpu().numpy()
        if NM == 1:
            soft = all_masks[0]
            return PredictionResult(binary_mask=(soft > threshold).astype(np.float32), soft_mask=soft)
        ious = torch.sigmoid(out["pred_iou"][0]).cpu().numpy()
        soft = all_masks[int(ious.argmax())]
        return PredictionResult(binary_mask=(soft > threshold).astype(np.float32), soft_mask=soft,
                                all_masks=(all_masks > threshold).astype(np.float32), all_ious=ious)
