"""Drop-in inference API (src/s3od/predictor.py:16-139): ``BackgroundRemoval`` / ``RemovalResult``.

Same names, constructor and ``remove_background(image, threshold=0.5) -> RemovalResult``.
The whole path runs on the GPU: uint8 upload -> letterbox resize (cv2 INTER_LINEAR fixed-point
emulation) + ImageNet normalisation -> DINOv3/DPT forward -> sigmoid -> unpad -> antialiased
bilinear resize back to the original size, all in libs3od_hip.so; only the 3 IoU scores,
the masks and the RGBA composition come back to the host, as in the reference.

Model loading is offline-safe: a local checkpoint path is tried first (``torch.load`` with
``weights_only=True``; ``{"state_dict": ...}``, Lightning ``model.``-prefixed and both
transformers key layouts are accepted), then the Hugging Face cache (``local_files_only``).
``model_id="synthetic"`` builds the deterministic synthetic weights (tests / benchmarks).
Errors: ``ValueError`` when the model cannot be located (predictor.py:59-63).
Reference quirks kept under ``exact_reference_quirks=True`` (the default):
  1. when (image_size - new_h) or (image_size - new_w) is odd and the pad is > 0, the reference
     raises a numpy broadcast ValueError (predictor.py:83-89);
  2. when the pad is 0 but the resized side is < image_size (e.g. 1024x1023), the reference feeds
     the UNPADDED resized image (S x new_w) to the model (predictor.py:89-90: ``padded = resized``),
     whose output is then S x 16*floor(new_w/16) and is resized back from that.
``exact_reference_quirks=False`` pads asymmetrically / to S x S instead.
"""
from __future__ import annotations

from dataclasses import dataclass
from pathlib import Path
from typing import Any, Dict, Optional, Tuple, Union

import numpy as np
import torch
from PIL import Image

from .utils import get_pad_info, remove_padding  # noqa: F401  (re-exported like the reference)
from .model import DPTSegmentation


@dataclass
class RemovalResult:
    predicted_mask: np.ndarray
    all_masks: np.ndarray
    all_ious: np.ndarray
    rgba_image: Image.Image


class BackgroundRemoval:
    DEFAULT_MODEL_ID = "okupyn/s3od"
    DEFAULT_CHECKPOINT_NAME = "s3od.pt"

    def __init__(self, model_id: Optional[str] = None, image_size: int = 1024, device: Optional[str] = None,
                 compute_dtype: str = "bf16", exact_reference_quirks: bool = True):
        if image_size % 16 != 0:
            raise ValueError("image_size must be a multiple of 16")
        self.image_size = image_size
        self.device = device or "cuda"
        if not str(self.device).startswith("cuda"):
            raise RuntimeError("BackgroundRemoval runs on the MI355X HIP kernels only (device='cuda')")
        self.exact_reference_quirks = exact_reference_quirks
        model_id = model_id or self.DEFAULT_MODEL_ID
        self.model = self._load_model(model_id, compute_dtype)
        self.model.to(self.device)
        self.model.eval()
        self.mean = np.array([0.485, 0.456, 0.406])
        self.std = np.array([0.229, 0.224, 0.225])

    @classmethod
    def from_pretrained(cls, model_id: str, **kwargs):
        return cls(model_id=model_id, **kwargs)

    def _load_model(self, model_id: str, compute_dtype: str) -> torch.nn.Module:
        if model_id == "synthetic":
            return DPTSegmentation(compute_dtype=compute_dtype, init_seed=0)
        path = Path(model_id)
        if not path.exists():
            try:
                from huggingface_hub import hf_hub_download
                path = Path(hf_hub_download(repo_id=model_id, filename=self.DEFAULT_CHECKPOINT_NAME, local_files_only=True))
            except Exception as e:
                raise ValueError(f"Could not load model from {model_id}. Ensure model exists on HuggingFace or provide "
                                 f"valid local path. Error: {e}")
        try:
            ckpt = torch.load(str(path), map_location="cpu", weights_only=True)
        except Exception as e:
            raise ValueError(f"Could not load checkpoint {path} with a safe (weights_only) loader: {e}")
        model = DPTSegmentation(num_classes=1, num_outputs=3, encoder_name="dinov3_base", features=256, use_bn=True,
                                use_clstoken=False, compute_dtype=compute_dtype, init_seed=None)
        model.load_state_dict(ckpt["state_dict"] if isinstance(ckpt, dict) and "state_dict" in ckpt else ckpt)
        return model

    # ------------------------------------------------------------------ pre / post
    def _pad_info(self, image: np.ndarray) -> Dict[str, Any]:
        info = get_pad_info(image, self.image_size)
        nh, nw = info["resized_size"]
        S = self.image_size
        if self.exact_reference_quirks and ((info["height_pad"] > 0 and S - nh != 2 * info["height_pad"]) or
                                            (info["width_pad"] > 0 and S - nw != 2 * info["width_pad"])):
            raise ValueError(f"could not broadcast input array from shape ({nh},{nw},3) into the padded canvas "
                             f"(reference predictor.py:83-89 behaviour for odd padding)")
        return info

    def _preprocess(self, image: np.ndarray) -> Tuple[torch.Tensor, Dict[str, Any]]:
        from ._lib import lib, stream
        info = self._pad_info(image)
        S = self.image_size
        nh, nw = info["resized_size"]
        img = torch.from_numpy(np.ascontiguousarray(image, dtype=np.uint8)).to(self.device)
        x = torch.empty((1, 3, S, S), dtype=torch.float32, device=self.device)
        lib()("s3od_preprocess", img, image.shape[0], image.shape[1], nh, nw, info["height_pad"], info["width_pad"], S, x, stream())
        if self.exact_reference_quirks and info["height_pad"] == 0 and info["width_pad"] == 0 and (nh, nw) != (S, S):
            # Quirk 2: `padded = resized` -> the model sees the nh x nw image (it sits at the canvas origin)
            x = x[:, :, :nh, :nw]
        return x, info

    @torch.no_grad()
    def remove_background(self, image: Union[np.ndarray, Image.Image], threshold: float = 0.5) -> RemovalResult:
        from ._lib import lib, stream
        if isinstance(image, Image.Image):
            image_pil = image.convert("RGB")
            image = np.array(image_pil)
        else:
            image_pil = Image.fromarray(image)
        x, pad = self._preprocess(image)
        out = self.model(x)
        H0, W0 = pad["original_size"]
        LH, LW = out["pred_masks"].shape[2], out["pred_masks"].shape[3]
        h, w = LH - 2 * pad["height_pad"], LW - 2 * pad["width_pad"]
        NM = out["pred_masks"].shape[1]
        tmp = torch.empty((NM, h, W0), dtype=torch.float32, device=x.device)
        masks = torch.empty((NM, H0, W0), dtype=torch.float32, device=x.device)
        lib()("s3od_sigmoid_unpad_resize", out["pred_masks"].contiguous(), NM, LH, LW, pad["height_pad"], pad["width_pad"], h, w,
              H0, W0, tmp, masks, stream())
        pred_ious = torch.sigmoid(out["pred_iou"]).squeeze(0).cpu().numpy()   # 3 floats
        all_masks = masks.cpu().numpy()
        best_idx = pred_ious.argmax()
        predicted_mask = all_masks[best_idx]
        alpha = (predicted_mask * 255).astype(np.uint8)
        rgba = np.dstack([image, alpha])
        return RemovalResult(predicted_mask=predicted_mask, all_masks=all_masks, all_ious=pred_ious,
                             rgba_image=Image.fromarray(rgba, mode="RGBA"))

    @torch.no_grad()
    def remove_background_batch(self, images: torch.Tensor) -> Dict[str, torch.Tensor]:
        """Batched device entry (C2/C5 benchmarks): normalised [B,3,S,S] -> sigmoid masks + ious on device."""
        out = self.model(images)
        return {"masks": torch.sigmoid(out["pred_masks"]), "ious": torch.sigmoid(out["pred_iou"])}
