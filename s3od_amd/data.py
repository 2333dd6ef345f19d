"""Training data path: the reference's folder dataset with its augmentation on device.

``MaskDataset`` keeps the constructor, file discovery and train/val split of
``synth_sod.model_training.dataset.MaskDataset`` (dataset.py:34-131): ``root_dir/images`` +
``root_dir/masks`` (same stem, .png/.jpg/.jpeg), sorted, ``random.seed(seed)`` shuffle, the first
``int(n * val_split)`` files are the validation split, optional ``debug_subset_fraction``.
Workers only decode (PIL -> uint8); ``GpuAugment`` turns a list of decoded samples into the
reference's batch dict ``{"images": fp32 [B,3,S,S] (ImageNet-normalised), "masks": fp32 [B,S,S]}``
on the GPU with one fused HIP launch per sample (``s3od_augment_sample``, data_ops.hip):

* mode "test": LongestMaxSize(S) + centred PadIfNeeded(S, fill 0) + Normalize (transforms.py:14-28);
* mode "regular": + HorizontalFlip 0.5, VerticalFlip 0.2, RandomRotate90 0.2, RandomResizedCrop
  0.5 (scale 0.85-1, ratio 0.9-1.1), Rotate ±15° 0.2 (composed into one affine map), ColorJitter
  (brightness 0.5, contrast 0.5, saturation 0.2, hue 0.2; p 0.7 inside OneOf p 0.5), noise OneOf
  p 0.3 of Gaussian (std 0.2-0.44) / multiplicative (0.9-1.1) (transforms.py:30-71);
* mode "synthetic" uses the "regular" pipeline: its extra albumentations effects (JPEG, weather,
  CLAHE, distortions, ...) are not built (documented gap).

albumentations / cv2 are not in this image, so the augmentations follow the published semantics
of those transforms but are NOT bit-matched to them ("parity unpinned"); the "test" mode is
checked against a numpy restatement in tests/test_gpu_data.py.
"""
from __future__ import annotations

import ctypes
import math
import os
import random
from typing import Dict, List, Optional

import numpy as np
import torch
from torch.utils.data import Dataset

from ._lib import lib, stream

_EXT = (".jpg", ".jpeg", ".png")


class MaskDataset(Dataset):
    def __init__(self, root_dir: str, image_size: int, split: str = "train", val_split: float = 0.1,
                 transform_mode: str = "regular", seed: int = 42, debug_subset_fraction: Optional[float] = None):
        self.root_dir, self.image_size, self.split = root_dir, image_size, split
        self.transform_mode = transform_mode
        self.images_dir = os.path.join(root_dir, "images")
        self.masks_dir = os.path.join(root_dir, "masks")
        train, val = self._get_splits(val_split, seed)
        self.files = train if split == "train" else val
        if debug_subset_fraction is not None:
            self.files = self.files[:int(len(self.files) * debug_subset_fraction)]

    def _get_splits(self, val_split: float, seed: int = 42):
        files = [f for f in os.listdir(self.images_dir) if f.lower().endswith(_EXT)]
        valid = sorted(f for f in files if os.path.exists(self.get_mask_path(f)))
        random.seed(seed)
        random.shuffle(valid)
        n_val = int(len(valid) * val_split)
        return valid[n_val:], valid[:n_val]

    def get_mask_path(self, img_file: str) -> str:
        base = os.path.splitext(img_file)[0]
        for ext in (".png", ".jpg", ".jpeg"):
            p = os.path.join(self.masks_dir, base + ext)
            if os.path.exists(p):
                return p
        return os.path.join(self.masks_dir, base + ".png")

    def __len__(self) -> int:
        return len(self.files)

    def __getitem__(self, idx: int) -> Dict[str, np.ndarray]:
        from PIL import Image
        img = np.ascontiguousarray(np.array(Image.open(os.path.join(self.images_dir, self.files[idx])).convert("RGB")))
        mask = np.ascontiguousarray(np.array(Image.open(self.get_mask_path(self.files[idx])).convert("L")))
        if img.shape[:2] != mask.shape[:2]:          # dataset.py:120-121: resample another item
            return self.__getitem__(random.randint(0, len(self) - 1))
        return {"image": img, "mask": mask}

    @staticmethod
    def collate(samples: List[Dict[str, np.ndarray]]) -> List[Dict[str, np.ndarray]]:
        """DataLoader collate_fn: keep the decoded samples as a list (augmentation runs on device)."""
        return samples


class AugParams(ctypes.Structure):
    _fields_ = [("A", ctypes.c_float * 6), ("H0", ctypes.c_int), ("W0", ctypes.c_int), ("new_h", ctypes.c_int),
                ("new_w", ctypes.c_int), ("pad_h", ctypes.c_int), ("pad_w", ctypes.c_int), ("bright", ctypes.c_float),
                ("contrast", ctypes.c_float), ("sat", ctypes.c_float), ("hue", ctypes.c_float),
                ("gray_mean", ctypes.c_float), ("mult", ctypes.c_float * 3), ("gauss_std", ctypes.c_float),
                ("seed", ctypes.c_uint)]


def letterbox(h0: int, w0: int, S: int):
    """LongestMaxSize(S) + centred PadIfNeeded(S): (new_h, new_w, pad_h, pad_w)."""
    sc = S / max(h0, w0)
    nh, nw = max(1, min(S, int(round(h0 * sc)))), max(1, min(S, int(round(w0 * sc))))
    return nh, nw, (S - nh) // 2, (S - nw) // 2


def _T(tx, ty):
    return np.array([[1, 0, tx], [0, 1, ty], [0, 0, 1]], np.float64)


class GpuAugment:
    """Callable: list of decoded samples -> device batch dict (see module docstring)."""

    def __init__(self, image_size: int, mode: str = "regular", device=None, seed: Optional[int] = None):
        self.S, self.mode = int(image_size), mode
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        # every data-parallel rank draws its own augmentation stream (the reference seeds each
        # worker from torch.initial_seed(), which differs per rank / worker)
        rank = torch.distributed.get_rank() if torch.distributed.is_available() and torch.distributed.is_initialized() else 0
        base = torch.initial_seed() if seed is None else int(seed)
        self.rng = random.Random(base * 1000003 + rank)

    def sample_params(self, h0: int, w0: int, img: Optional[np.ndarray] = None) -> AugParams:
        S, r = self.S, self.rng
        nh, nw, ph, pw = letterbox(h0, w0, S)
        M = np.eye(3)                              # forward map canvas -> output (pixel-centre coords)
        bright = contrast = sat = 1.0
        hue, mult, gstd = 0.0, [1.0, 1.0, 1.0], 0.0
        if self.mode != "test":
            c = S / 2.0
            if r.random() < 0.5:
                M = _T(c, c) @ np.diag([-1.0, 1.0, 1.0]) @ _T(-c, -c) @ M
            if r.random() < 0.2:
                M = _T(c, c) @ np.diag([1.0, -1.0, 1.0]) @ _T(-c, -c) @ M
            if r.random() < 0.2:
                k = r.randint(0, 3)
                cs, sn = (1, 0, -1, 0)[k], (0, -1, 0, 1)[k]   # exact rotation by -k*90 degrees
                R = np.array([[cs, -sn, 0], [sn, cs, 0], [0, 0, 1]], np.float64)
                M = _T(c, c) @ R @ _T(-c, -c) @ M
            if r.random() < 0.5:                      # RandomResizedCrop(scale .85-1, ratio .9-1.1)
                area = S * S
                for _ in range(10):
                    a = area * r.uniform(0.85, 1.0)
                    ar = math.exp(r.uniform(math.log(0.9), math.log(1.1)))
                    cw, ch = int(round(math.sqrt(a * ar))), int(round(math.sqrt(a / ar)))
                    if 0 < cw <= S and 0 < ch <= S:
                        x0, y0 = r.randint(0, S - cw), r.randint(0, S - ch)
                        M = np.diag([S / cw, S / ch, 1.0]) @ _T(-x0, -y0) @ M
                        break
            if r.random() < 0.2:                      # Rotate(limit=15), constant-0 border
                th = math.radians(r.uniform(-15, 15))
                R = np.array([[math.cos(th), math.sin(th), 0], [-math.sin(th), math.cos(th), 0], [0, 0, 1]])
                M = _T(c, c) @ R @ _T(-c, -c) @ M
            if r.random() < 0.5 and r.random() < 0.7:  # OneOf(ColorJitter p.7, Sharpen p.3) p.5
                bright, contrast = r.uniform(0.5, 1.5), r.uniform(0.5, 1.5)
                sat, hue = r.uniform(0.8, 1.2), r.uniform(-0.2, 0.2)
            if r.random() < 0.3:                      # OneOf(GaussNoise, ISONoise, MultiplicativeNoise) p.3
                if r.random() < 0.5:
                    gstd = r.uniform(0.2, 0.44)
                else:
                    mult = [r.uniform(0.9, 1.1) for _ in range(3)]
        Minv = np.linalg.inv(M)
        p = AugParams()
        for i, v in enumerate(list(Minv[0]) + list(Minv[1])):
            p.A[i] = float(v)
        p.H0, p.W0, p.new_h, p.new_w, p.pad_h, p.pad_w = h0, w0, nh, nw, ph, pw
        p.bright, p.contrast, p.sat, p.hue = bright, contrast, sat, hue
        gm = 0.0
        if contrast != 1.0 and img is not None:       # mean grey of the padded canvas after brightness
            g = (img[..., 0] * 0.299 + img[..., 1] * 0.587 + img[..., 2] * 0.114).mean() / 255.0
            gm = min(1.0, g * bright) * (nh * nw) / (S * S)
        p.gray_mean = gm
        for i in range(3):
            p.mult[i] = mult[i]
        p.gauss_std = gstd
        p.seed = r.getrandbits(32)
        return p

    def __call__(self, samples: List[Dict[str, np.ndarray]]) -> Dict[str, torch.Tensor]:
        B, S, dev = len(samples), self.S, self.device
        images = torch.empty((B, 3, S, S), dtype=torch.float32, device=dev)
        masks = torch.empty((B, S, S), dtype=torch.float32, device=dev)
        keep = []
        for b, smp in enumerate(samples):
            img = torch.from_numpy(np.ascontiguousarray(smp["image"], dtype=np.uint8)).pin_memory().to(dev, non_blocking=True)
            msk = torch.from_numpy(np.ascontiguousarray(smp["mask"], dtype=np.uint8)).pin_memory().to(dev, non_blocking=True)
            h0, w0 = smp["image"].shape[:2]
            prm = self.sample_params(h0, w0, smp["image"])
            lib()("s3od_augment_sample", img, msk, ctypes.addressof(prm), S, images[b], masks[b], stream())
            keep.append((img, msk))
        self._inflight = keep                          # keep the uploads alive until the kernels ran
        return {"images": images, "masks": masks}
