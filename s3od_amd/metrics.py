"""SOD evaluation metrics on the GPU — drop-in for ``synth_sod.model_training.metrics.EvaluationMetrics``
(``synth_sod/src/synth_sod/model_training/metrics.py:213-424``) and the dataset loop that drives it
(``compute_metrics.py:42-100`` ``process_dataset``).

Every per-image number comes from one ``s3od_eval_metrics`` call (``csrc/metrics.hip``): MAE, the
255-threshold MaxF / AvgF curve, the S-measure, the changeable E-measure (mean of its 256-point
curve, which is what ``EMeasure.get_metrics`` reports) and the weighted F-measure with an exact
Euclidean distance transform.  The reference copies every mask to the host for the E-measure and
weighted-F (numpy / scipy); here nothing leaves the device until ``compute_metrics``.

Contract (as the reference's ``process_dataset`` feeds it): ``pred`` a soft mask in [0, 1], ``mask``
a {0, 1} ground truth (``cv2.imread(...) > 128``), both [H, W] (a leading 1-dim is accepted).  Like
the reference, ``step`` binarises ``mask`` in place at 0.5 when it is neither all-0 nor all-1
(``metrics.py:239-240,267-268``).  Numerics: MAE, MaxF, E-measure and weighted F match the
reference to rounding (the distance transform reproduces scipy's nearest-feature choice on ties);
AvgF and the S-measure are computed in float64 where the reference keeps some float32 tensors
(differences ~1e-7 relative; ``tests/test_gpu_metrics.py`` states the bounds).
"""
from __future__ import annotations

import ctypes
import glob
import os
from typing import Dict, Optional

import numpy as np
import torch

from ._lib import lib, stream

KEYS = ("mae", "max_f", "avg_f", "s_score", "em", "wfm")


def _tables():
    thr = torch.linspace(0, 1 - 1e-10, 255, dtype=torch.float32).numpy().copy()     # metrics.py:322
    m = 3.0
    y, x = np.ogrid[-m:m + 1, -m:m + 1]
    h = np.exp(-(x * x + y * y) / (2 * 5.0 * 5.0))                                  # metrics.py:193-205
    h[h < np.finfo(h.dtype).eps * h.max()] = 0
    h = np.ascontiguousarray(h / h.sum(), dtype=np.float64)
    return thr, h


_THR, _K7 = _tables()


def _plane(t, dev):
    """-> contiguous float32 [H, W] on `dev` (a view when already so)."""
    if isinstance(t, np.ndarray):
        t = torch.from_numpy(t)
    t = t.reshape(t.shape[-2], t.shape[-1])
    return t.to(device=dev, dtype=torch.float32).contiguous()


class EvaluationMetrics:
    """metrics.py:213-314 with the same constructor, ``step`` / ``compute_metrics`` / ``reset``."""

    def __init__(self, device="cuda", sm_only: bool = False):
        self.device = device
        self.sm_only = sm_only
        self._dev = torch.device("cuda", torch.cuda.current_device()) if not isinstance(device, torch.device) or \
            device.type != "cuda" else device
        self._out = []                    # device float64 [6] per step
        self._ws = None

    def _workspace(self, H, W):
        need = ctypes.c_long(0)
        lib()("s3od_eval_metrics_ws", H, W, ctypes.addressof(need))
        if self._ws is None or self._ws.numel() < need.value:
            self._ws = torch.empty(need.value, dtype=torch.uint8, device=self._dev)
        return self._ws

    def step(self, pred, mask):
        p = _plane(pred, self._dev)
        g = _plane(mask, self._dev)
        if p.shape != g.shape:
            raise ValueError(f"pred {tuple(p.shape)} and mask {tuple(g.shape)} differ")
        H, W = p.shape
        ws = self._workspace(H, W)
        out = torch.empty(6, dtype=torch.float64, device=self._dev)
        lib()("s3od_eval_metrics", p, g, H, W, _THR.ctypes.data, _K7.ctypes.data, ws, ws.numel(), int(self.sm_only), 1,
              out, stream())
        self._out.append(out)
        # the reference binarises the caller's mask in place (only changes values in the general case)
        shares = isinstance(mask, torch.Tensor) and mask.data_ptr() == g.data_ptr()
        if not shares:
            if isinstance(mask, torch.Tensor):
                mask.copy_(g.view(mask.shape).to(mask.device, mask.dtype))
            elif isinstance(mask, np.ndarray) and mask.flags.writeable:
                np.copyto(mask, g.view(mask.shape).cpu().numpy().astype(mask.dtype))

    @property
    def metrics(self) -> Dict[str, list]:
        """Per-image lists in the reference's layout (metrics.py:217-222), materialised on demand."""
        v = torch.stack(self._out).cpu().numpy() if self._out else np.zeros((0, 6))
        if self.sm_only:
            return {"mae": [], "max_f": [], "avg_f": [], "s_score": list(v[:, 3])}
        return {k: list(v[:, i]) for i, k in enumerate(KEYS[:4])}

    def per_image(self) -> np.ndarray:
        """[n_images, 6] float64: MAE, MaxF, AvgF, Sm, Em (curve mean), wF."""
        return torch.stack(self._out).cpu().numpy() if self._out else np.zeros((0, 6))

    def compute_metrics(self) -> dict:
        v = self.per_image()
        if self.sm_only:
            return {"Sm": np.mean(v[:, 3])}
        return {"MAE": np.mean(v[:, 0]), "MaxF": np.mean(v[:, 1]), "AvgF": np.mean(v[:, 2]), "Sm": np.mean(v[:, 3]),
                "Em": np.mean(v[:, 4]), "wF": np.mean(v[:, 5])}

    def reset(self):
        self._out.clear()


def find_gt_mask_path(image_path: str, data_dir: str) -> Optional[str]:
    """compute_metrics.py:180-195: masks/<stem>{.png,.jpg,.jpeg}, then the images->masks path swap."""
    from pathlib import Path
    stem, suffix = Path(image_path).stem, Path(image_path).suffix
    for ext in (".png", ".jpg", ".jpeg"):
        p = os.path.join(data_dir, "masks", stem + ext)
        if os.path.exists(p):
            return p
    for ext in (".png", ".jpg", ".jpeg"):
        p = image_path.replace("/images/", "/masks/").replace(suffix, ext)
        if os.path.exists(p):
            return p
    return None


def read_gray_u8(path):
    """``cv2.imread(path, cv2.IMREAD_GRAYSCALE)`` restated on PIL: 16-bit masks are scaled to 8 bits
    (>> 8, as cv2 does; PIL's convert("L") would clip them) and colour masks use cv2's BT.601
    fixed-point weights ((4899 R + 9617 G + 1868 B + 8192) >> 14).  Remaining gap (unpinned, cv2 is
    absent): JPEG masks, which libjpeg converts to grey inside the decoder."""
    from PIL import Image
    im = Image.open(path)
    if im.mode in ("I;16", "I;16B", "I;16L", "I"):
        a = np.asarray(im).astype(np.int64)
        return np.clip(a >> 8, 0, 255).astype(np.uint8)
    if im.mode in ("L", "1"):
        return np.asarray(im.convert("L"))
    a = np.asarray(im.convert("RGB")).astype(np.int64)
    return ((4899 * a[..., 0] + 9617 * a[..., 1] + 1868 * a[..., 2] + 8192) >> 14).astype(np.uint8)


def process_dataset(data_dir: str, predictor, compute_best_metrics: bool = False):
    """compute_metrics.py:42-100: predict every ``images/*`` file, score it against ``masks/``.

    ``predictor.predict(rgb_uint8)`` must return an object with ``soft_mask`` (and, for
    ``compute_best_metrics``, ``has_multiple_masks`` / ``num_masks`` / ``all_masks``), as
    ``SODPredictor`` (``s3od_amd.predictor.SODPredictor``) does.  Image decoding uses PIL (cv2 is
    not part of this stack); ``> 128`` thresholding of the grey mask as the reference."""
    from PIL import Image
    images = glob.glob(f"{data_dir}/images/*")
    counter = EvaluationMetrics(device="cuda")
    best = EvaluationMetrics(device="cuda") if compute_best_metrics else None
    for image_path in images:
        image = np.asarray(Image.open(image_path).convert("RGB"))
        result = predictor.predict(image)
        gt_path = find_gt_mask_path(image_path, data_dir)
        if not gt_path:
            print(f"Warning: GT mask not found for {image_path}")
            continue
        gt_mask = (read_gray_u8(gt_path) > 128).astype(np.float32)
        gt_t = torch.from_numpy(gt_mask).cuda()
        soft = torch.as_tensor(result.soft_mask)
        counter.step(soft, gt_t.clone())
        if compute_best_metrics:
            chosen = soft
            if getattr(result, "has_multiple_masks", False):
                best_iou, chosen = -1.0, None
                g = gt_mask > 0.5
                for i in range(result.num_masks):
                    m = np.asarray(result.all_masks[i]) > 0.5
                    union = np.logical_or(m, g).sum()
                    iou = np.logical_and(m, g).sum() / union if union > 0 else 1.0
                    if iou > best_iou:
                        best_iou, chosen = iou, torch.as_tensor(result.all_masks[i])
                if chosen is None:
                    chosen = soft
            best.step(chosen, gt_t.clone())
    pred_metrics = counter.compute_metrics()
    if compute_best_metrics:
        return {"pred_metrics": pred_metrics, "best_metrics": best.compute_metrics()}
    return pred_metrics
