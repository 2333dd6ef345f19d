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
* mode "synthetic" (transforms.py:65-220): the "regular" geometry + the synthetic groups, each a
  OneOf with the reference's probabilities and member weights: colour (ColorJitter 0.4/0.4/0.3/0.2 |
  HueSaturationValue 25/35/30 | CLAHE*), noise (ISONoise | GaussNoise 0.25-0.6 | MultiplicativeNoise),
  quality (ImageCompression* | Downscale 0.4-0.7), lighting (RandomShadow 1-3 | RandomBrightnessContrast
  0.4/0.4), blur (MotionBlur | GaussianBlur 3-7 | Defocus 2-6 | ZoomBlur*), colour space (ToSepia |
  ToGray | ChannelShuffle, p 0.05), distortion (OpticalDistortion 0.3 | GridDistortion* |
  ElasticTransform* | Perspective 0.05-0.1, geometry also applied to the mask), detail (Emboss |
  Sharpen | Posterize 5 bits) and weather (RandomSnow* | RandomRain*, p 0.15).  Members marked * are
  not built: when the OneOf draws one of them the group is a no-op.  Three HIP passes per sample:
  geometry -> raw [0,1] RGB, per-pixel photometric chain, then one composed (blur * sharpen/emboss)
  filter with the Downscale sampling, colour space, posterize and Normalize (s3od_augment_synthetic).

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
    """Mirror of struct AugParams (csrc/data_ops.hip)."""
    _fields_ = [("A", ctypes.c_float * 6), ("H0", ctypes.c_int), ("W0", ctypes.c_int), ("new_h", ctypes.c_int),
                ("new_w", ctypes.c_int), ("pad_h", ctypes.c_int), ("pad_w", ctypes.c_int), ("bright", ctypes.c_float),
                ("contrast", ctypes.c_float), ("sat", ctypes.c_float), ("hue", ctypes.c_float),
                ("gray_mean", ctypes.c_float), ("mult", ctypes.c_float * 3), ("gauss_std", ctypes.c_float),
                ("seed", ctypes.c_uint), ("persp", ctypes.c_float * 2), ("kdist", ctypes.c_float), ("raw", ctypes.c_int)]


class SynthParams(ctypes.Structure):
    """Mirror of struct SynthParams (csrc/data_ops.hip): the synthetic-mode photometric chain."""
    _fields_ = [("bright", ctypes.c_float), ("contrast", ctypes.c_float), ("sat", ctypes.c_float), ("hue", ctypes.c_float),
                ("gray_mean", ctypes.c_float), ("hsv_h", ctypes.c_float), ("hsv_s", ctypes.c_float), ("hsv_v", ctypes.c_float),
                ("iso_int", ctypes.c_float), ("iso_color", ctypes.c_float), ("gauss_std", ctypes.c_float),
                ("mult", ctypes.c_float * 3), ("rbc_alpha", ctypes.c_float), ("rbc_beta", ctypes.c_float),
                ("n_shadow", ctypes.c_int), ("shadow", (ctypes.c_float * 6) * 3), ("shadow_dim", ctypes.c_float),
                ("down", ctypes.c_float), ("ksize", ctypes.c_int), ("color_op", ctypes.c_int), ("perm", ctypes.c_int * 3),
                ("post_bits", ctypes.c_int), ("seed", ctypes.c_uint)]

    @classmethod
    def identity(cls):
        p = cls()
        p.bright = p.contrast = p.sat = 1.0
        p.mult[0] = p.mult[1] = p.mult[2] = 1.0
        p.rbc_alpha, p.shadow_dim, p.down, p.ksize, p.post_bits = 1.0, 1.0, 1.0, 1, 8
        p.perm[0], p.perm[1], p.perm[2] = 0, 1, 2
        return p


def _one_of(r, p, weights):
    """albumentations OneOf(p): with probability p pick one member with probability proportional to its p."""
    if r.random() >= p:
        return None
    tot = sum(weights)
    u, acc = r.random() * tot, 0.0
    for i, w in enumerate(weights):
        acc += w
        if u < acc:
            return i
    return len(weights) - 1


def _gauss_kernel(k, sigma=None):
    sigma = sigma or 0.3 * ((k - 1) * 0.5 - 1) + 0.8            # cv2.getGaussianKernel default
    x = np.arange(k) - (k - 1) / 2
    g = np.exp(-x ** 2 / (2 * sigma ** 2))
    g /= g.sum()
    return np.outer(g, g)


def _motion_kernel(r, k):
    ker = np.zeros((k, k))
    th = r.uniform(0, np.pi)
    c = (k - 1) / 2
    for t in np.linspace(-c, c, 4 * k):
        ker[int(round(c + t * np.sin(th))), int(round(c + t * np.cos(th)))] = 1.0
    return ker / ker.sum()


def _disk_kernel(radius, alias_sigma):
    k = 2 * radius + 1
    y, x = np.mgrid[-radius:radius + 1, -radius:radius + 1]
    ker = (x ** 2 + y ** 2 <= radius ** 2).astype(np.float64)
    ker /= ker.sum()
    if alias_sigma > 0:                                           # Defocus alias blur (small Gaussian)
        from scipy.signal import convolve2d
        ker = convolve2d(ker, _gauss_kernel(3, alias_sigma), mode="same")
        ker /= ker.sum()
    return ker


def _sharpen_kernel(alpha, lightness):
    ident = np.zeros((3, 3)); ident[1, 1] = 1.0
    sh = np.array([[-1, -1, -1], [-1, 8 + lightness, -1], [-1, -1, -1]], np.float64)
    return (1 - alpha) * ident + alpha * sh


def _emboss_kernel(alpha, strength):
    ident = np.zeros((3, 3)); ident[1, 1] = 1.0
    em = np.array([[-1 - strength, -strength, 0], [-strength, 1, strength], [0, strength, 1 + strength]], np.float64)
    return (1 - alpha) * ident + alpha * em


def letterbox(h0: int, w0: int, S: int):
    """LongestMaxSize(S) + centred PadIfNeeded(S): (new_h, new_w, pad_h, pad_w)."""
    sc = S / max(h0, w0)
    nh, nw = max(1, min(S, int(round(h0 * sc)))), max(1, min(S, int(round(w0 * sc))))
    return nh, nw, (S - nh) // 2, (S - nw) // 2


def _T(tx, ty):
    return np.array([[1, 0, tx], [0, 1, ty], [0, 0, 1]], np.float64)


def _homography(src, dst):
    """3x3 H with H @ [src, 1] ~ [dst, 1] for 4 point pairs (DLT)."""
    A = []
    for (x, y), (u, v) in zip(src, dst):
        A.append([x, y, 1, 0, 0, 0, -u * x, -u * y, -u])
        A.append([0, 0, 0, x, y, 1, -v * x, -v * y, -v])
    _, _, vt = np.linalg.svd(np.asarray(A))
    return vt[-1].reshape(3, 3) / vt[-1][-1]


def _conv_full(a, b):
    from scipy.signal import convolve2d
    return convolve2d(a, b, mode="full")


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
        kdist = 0.0
        if self.mode == "synthetic":
            M = self._geometry(M)
            g = _one_of(r, 0.4, [0.3, 0.3, 0.2, 0.15])           # Optical | Grid* | Elastic* | Perspective
            if g == 0:
                kdist = r.uniform(-0.3, 0.3) * 0.25                 # distort_limit 0.3 on the normalised radius
            elif g == 3:                                        # Perspective(scale 0.05-0.1): corner jitter
                sc = r.uniform(0.05, 0.1)
                src = np.array([[0, 0], [S, 0], [S, S], [0, S]], np.float64)
                dst = src + np.array([[r.gauss(0, sc) * S, r.gauss(0, sc) * S] for _ in range(4)])
                Hm = _homography(dst, src)                      # output -> canvas
                Mi = np.linalg.inv(M)
                Tot = Mi @ Hm
                Tot /= Tot[2, 2]
                p = AugParams()
                for i, v in enumerate(list(Tot[0]) + list(Tot[1])):
                    p.A[i] = float(v)
                self._fill(p, h0, w0, nh, nw, ph, pw)
                p.persp[0], p.persp[1] = float(Tot[2, 0]), float(Tot[2, 1])
                p.raw = 1
                return p
        elif self.mode != "test":
            M = self._geometry(M)
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
        self._fill(p, h0, w0, nh, nw, ph, pw)
        p.kdist = kdist
        p.raw = int(self.mode == "synthetic")
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

    @staticmethod
    def _fill(p, h0, w0, nh, nw, ph, pw):
        p.H0, p.W0, p.new_h, p.new_w, p.pad_h, p.pad_w = h0, w0, nh, nw, ph, pw
        p.bright = p.contrast = p.sat = 1.0
        p.mult[0] = p.mult[1] = p.mult[2] = 1.0

    def _geometry(self, M):
        """transforms.py:30-39 geometric group (shared by "regular" and "synthetic")."""
        S, r = self.S, self.rng
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
        return M

    def synth_params(self, img: Optional[np.ndarray] = None):
        """The synthetic-mode photometric groups (transforms.py:65-216): SynthParams + the composed filter."""
        S, r = self.S, self.rng
        q = SynthParams.identity()
        g = _one_of(r, 0.7, [0.7, 0.4, 0.2])                  # ColorJitter | HueSaturationValue | CLAHE*
        if g == 0:
            q.bright, q.contrast = r.uniform(0.6, 1.4), r.uniform(0.6, 1.4)
            q.sat, q.hue = r.uniform(0.7, 1.3), r.uniform(-0.2, 0.2)
            if img is not None:
                gm = (img[..., 0] * 0.299 + img[..., 1] * 0.587 + img[..., 2] * 0.114).mean() / 255.0
                q.gray_mean = min(1.0, gm * q.bright)
        elif g == 1:
            q.hsv_h, q.hsv_s, q.hsv_v = r.uniform(-25, 25), r.uniform(-35, 35) / 255.0, r.uniform(-30, 30) / 255.0
        g = _one_of(r, 0.6, [0.4, 0.4, 0.4])                  # ISONoise | GaussNoise | MultiplicativeNoise
        if g == 0:
            q.iso_color, q.iso_int = r.uniform(0.01, 0.03), r.uniform(0.08, 0.3) * 0.2
        elif g == 1:
            q.gauss_std = r.uniform(0.25, 0.6)
        elif g == 2:
            for i in range(3):
                q.mult[i] = r.uniform(0.9, 1.1)
        g = _one_of(r, 0.5, [0.4, 0.3])                       # ImageCompression* | Downscale
        if g == 1:
            q.down = r.uniform(0.4, 0.7)
        g = _one_of(r, 0.5, [0.4, 0.4])                       # RandomShadow | RandomBrightnessContrast
        if g == 0:
            q.n_shadow, q.shadow_dim = r.randint(1, 3), 0.5
            for t in range(q.n_shadow):                         # shadow_roi (0, 0.1, 1, 1)
                for v in range(3):
                    q.shadow[t][2 * v], q.shadow[t][2 * v + 1] = r.uniform(0, S), r.uniform(0.1 * S, S)
        elif g == 1:
            q.rbc_alpha, q.rbc_beta = 1.0 + r.uniform(-0.4, 0.4), r.uniform(-0.4, 0.4)
        ker = np.ones((1, 1))
        g = _one_of(r, 0.5, [0.4, 0.4, 0.3, 0.2])             # MotionBlur | GaussianBlur | Defocus | ZoomBlur*
        if g in (0, 1):
            k = r.choice([3, 5, 7])
            ker = _motion_kernel(r, k) if g == 0 else _gauss_kernel(k)
        elif g == 2:
            ker = _disk_kernel(r.randint(2, 6), r.uniform(0.1, 0.3))
        g = _one_of(r, 0.05, [0.5, 0.5, 0.3])                 # ToSepia | ToGray | ChannelShuffle
        if g is not None:
            q.color_op = g + 1
            perm = [0, 1, 2]
            r.shuffle(perm)
            q.perm[0], q.perm[1], q.perm[2] = perm
        g = _one_of(r, 0.3, [0.3, 0.3, 0.2])                  # Emboss | Sharpen | Posterize
        if g == 0:
            ker = _conv_full(ker, _emboss_kernel(r.uniform(0.2, 0.4), r.uniform(0.2, 0.5)))
        elif g == 1:
            ker = _conv_full(ker, _sharpen_kernel(r.uniform(0.2, 0.6), r.uniform(0.5, 1.2)))
        elif g == 2:
            q.post_bits = 5
        _one_of(r, 0.15, [0.1, 0.1])                           # RandomSnow* | RandomRain*
        q.ksize = ker.shape[0]
        q.seed = r.getrandbits(32)
        kw = torch.tensor(ker.reshape(-1), dtype=torch.float32).to(self.device, non_blocking=True) if q.ksize > 1 else None
        return q, kw

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
            if self.mode == "synthetic":
                raw = torch.empty((3, S, S), dtype=torch.float32, device=dev)
                lib()("s3od_augment_sample", img, msk, ctypes.addressof(prm), S, raw, masks[b], stream())
                q, kw = self.synth_params(smp["image"])
                lib()("s3od_augment_synthetic", raw, ctypes.addressof(q), kw, S, images[b], stream())
                keep.append((img, msk, raw, kw))
                continue
            lib()("s3od_augment_sample", img, msk, ctypes.addressof(prm), S, images[b], masks[b], stream())
            keep.append((img, msk))
        self._inflight = keep                          # keep the uploads alive until the kernels ran
        return {"images": images, "masks": masks}
