"""Letterbox geometry (src/s3od/utils.py:6-37), same signatures and semantics."""
from __future__ import annotations

from typing import Any, Dict

import numpy as np


def get_pad_info(image: np.ndarray, image_size: int = 1024) -> Dict[str, Any]:
    h, w = image.shape[:2]
    aspect_ratio = w / h
    if aspect_ratio > 1:
        new_w = image_size
        new_h = int(new_w / aspect_ratio)
        return {"height_pad": (image_size - new_h) // 2, "width_pad": 0, "original_size": (h, w), "resized_size": (new_h, new_w)}
    new_h = image_size
    new_w = int(new_h * aspect_ratio)
    return {"height_pad": 0, "width_pad": (image_size - new_w) // 2, "original_size": (h, w), "resized_size": (new_h, new_w)}


def remove_padding(masks, pad_info: Dict[str, Any]):
    if pad_info["height_pad"] > 0:
        masks = masks[:, pad_info["height_pad"]:-pad_info["height_pad"], :]
    if pad_info["width_pad"] > 0:
        masks = masks[:, :, pad_info["width_pad"]:-pad_info["width_pad"]]
    return masks
