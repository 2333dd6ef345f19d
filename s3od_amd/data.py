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
  0.5 (scale 0.85-1, ratio 0.9-1.1), Rotate ±15° 0.2 (composed into one affine map), OneOf p 0.5 of
  ColorJitter (brightness 0.5, contrast 0.5, saturation 0.2, hue 0.2; weight 0.7) / Sharpen (alpha
  0.2-0.5, lightness 0.5-1.0; weight 0.3), noise OneOf p 0.3 of Gaussian (std 0.2-0.44) / ISONoise
  (colour shift 0.01-0.05, intensity 0.1-0.5; HLS + Poisson) / multiplicative (0.9-1.1)
  (transforms.py:30-71).  A draw of Sharpen or ISONoise runs the two-stage chain of
  ``s3od_augment_synthetic`` (order 1) after the geometry pass;
* mode "synthetic" (transforms.py:65-220): the "regular" geometry + the synthetic groups, each a
  OneOf with the reference's probabilities and member weights: colour (ColorJitter 0.4/0.4/0.3/0.2 |
  HueSaturationValue 25/35/30 | CLAHE 4.0 / 8x8 tiles), noise (ISONoise | GaussNoise 0.25-0.6 |
  MultiplicativeNoise), quality (ImageCompression 30-80: 8x8 DCT, 4:2:0 chroma, libjpeg tables |
  Downscale 0.4-0.7), lighting (RandomShadow 1-3 pentagons | RandomBrightnessContrast 0.4/0.4), blur
  (MotionBlur | GaussianBlur 3-7 | Defocus 2-6 | ZoomBlur 1-1.1), colour space (ToSepia | ToGray |
  ChannelShuffle, p 0.05), distortion (OpticalDistortion 0.3 | GridDistortion 6 steps | ElasticTransform |
  Perspective 0.05-0.1, geometry also applied to the mask), detail (Emboss | Sharpen | Posterize 5 bits)
  and weather (RandomSnow | RandomRain, p 0.15).  Three HIP passes per sample: geometry + distortion ->
  raw [0,1] RGB, the per-pixel photometric chain (with the CLAHE / JPEG / ZoomBlur / rain / snow
  stages), then one composed (blur * sharpen/emboss) filter with the Downscale sampling, colour space,
  posterize and Normalize (s3od_augment_synthetic).

albumentations / cv2 are not in this image, so the augmentations follow the published semantics
of albumentations 2.0.8 but are NOT bit-matched to it ("parity unpinned"); every member is checked
against the numpy restatement in oracle/augment_oracle.py (tests/test_gpu_augment.py, JPEG pinned
to libjpeg through PIL) and the "test" mode against tests/test_gpu_data.py.
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
                ("seed", ctypes.c_uint), ("persp", ctypes.c_float * 2), ("kdist", ctypes.c_float), ("raw", ctypes.c_int),
                ("grid", ctypes.c_void_p), ("elastic", ctypes.c_void_p)]


class SynthParams(ctypes.Structure):
    """Mirror of struct SynthParams (csrc/data_ops.hip): the photometric chain after the geometry pass."""
    _fields_ = [("bright", ctypes.c_float), ("contrast", ctypes.c_float), ("sat", ctypes.c_float), ("hue", ctypes.c_float),
                ("gray_mean", ctypes.c_float), ("hsv_h", ctypes.c_float), ("hsv_s", ctypes.c_float), ("hsv_v", ctypes.c_float),
                ("clahe_clip", ctypes.c_float), ("iso_intensity", ctypes.c_float), ("iso_color_shift", ctypes.c_float),
                ("gauss_std", ctypes.c_float), ("mult", ctypes.c_float * 3), ("jpeg_quality", ctypes.c_int),
                ("down", ctypes.c_float), ("rbc_alpha", ctypes.c_float), ("rbc_beta", ctypes.c_float),
                ("n_shadow", ctypes.c_int), ("shadow", (ctypes.c_float * 10) * 3), ("shadow_dim", ctypes.c_float),
                ("ksize", ctypes.c_int), ("zoom_n", ctypes.c_int), ("zoom", ctypes.c_float * 4),
                ("color_op", ctypes.c_int), ("perm", ctypes.c_int * 3), ("post_bits", ctypes.c_int),
                ("snow_point", ctypes.c_float), ("snow_coeff", ctypes.c_float),
                ("rain_n", ctypes.c_int), ("rain_slant", ctypes.c_int), ("rain_len", ctypes.c_int), ("rain_blur", ctypes.c_int),
                ("rain_color", ctypes.c_float), ("rain_bright", ctypes.c_float), ("order", ctypes.c_int),
                ("seed", ctypes.c_uint), ("rain_drops", ctypes.c_void_p), ("ws", ctypes.c_void_p)]

    @classmethod
    def identity(cls):
        p = cls()
        p.bright = p.contrast = p.sat = 1.0
        p.mult[0] = p.mult[1] = p.mult[2] = 1.0
        p.rbc_alpha, p.shadow_dim, p.down, p.ksize, p.post_bits = 1.0, 1.0, 1.0, 1, 8
        p.perm[0], p.perm[1], p.perm[2] = 0, 1, 2
        return p


class ElasticParams(ctypes.Structure):
    """Mirror of struct ElasticParams (csrc/data_ops.hip)."""
    _fields_ = [("w", ctypes.c_float * 33), ("ksize", ctypes.c_int), ("alpha", ctypes.c_float), ("seed", ctypes.c_uint)]


def augment_ws_floats(S: int) -> int:
    """Size (floats) of SynthParams.ws for canvas size S (s3od_augment_ws_floats)."""
    n = ctypes.c_long(0)
    lib()("s3od_augment_ws_floats", int(S), ctypes.addressof(n))
    return int(n.value)


def gaussian_taps(ksize: int, sigma: float) -> np.ndarray:
    """cv2.getGaussianKernel(ksize, sigma) (sigma > 0)."""
    x = np.arange(ksize) - (ksize - 1) / 2
    g = np.exp(-x ** 2 / (2 * sigma ** 2))
    return g / g.sum()


def elastic_params(seed: int, alpha: float = 1.0, sigma: float = 25.0, ksize: int = 17) -> ElasticParams:
    """ElasticTransform(alpha=1, sigma=25) displacement parameters (transforms.py:169-173; albumentations
    2.0.8 generate_displacement_fields with approximate=False, i.e. a 17x17 Gaussian)."""
    e = ElasticParams()
    for i, v in enumerate(gaussian_taps(ksize, sigma)):
        e.w[i] = float(v)
    e.ksize, e.alpha, e.seed = ksize, float(alpha), seed & 0xFFFFFFFF
    return e


def grid_distortion_maps(S: int, steps_x, steps_y, num_steps: int = 6):
    """GridDistortion(num_steps=6, distort_limit=0.3, normalized=True) (transforms.py:164-168): the
    albumentations 2.0.8 step normalisation (last step scaled to its true width, steps rescaled so the
    distorted grid ends at the image border) and the separable per-column / per-row source maps
    (index coordinates) that cv2.remap reads."""
    def one(size, steps):
        step = size // num_steps
        steps = np.asarray(steps, np.float64).copy()
        last = min(size, (num_steps + 1) * step) - num_steps * step
        steps[-1] *= last / step
        steps *= (size / math.floor(size / num_steps)) / steps.sum()
        m = np.zeros(size, np.float32)
        prev = 0.0
        for idx, st in enumerate(steps):
            start = idx * step
            end = min(start + step, size)
            if start >= size:
                break
            cur = prev + step * st
            m[start:end] = np.linspace(prev, cur, end - start, dtype=np.float64).astype(np.float32)
            prev = cur
        return m
    return one(S, steps_x), one(S, steps_y)


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
        if mode == "synthetic" and self.S % 8:
            # CLAHE's 8x8 tile grid (drawn for ~10 % of synthetic samples) is built for S % 8 == 0: fail here,
            # not at a random step
            raise ValueError(f"GpuAugment: synthetic mode needs image_size divisible by 8 (CLAHE tiles), got {self.S}")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        # every data-parallel rank draws its own augmentation stream (the reference seeds each
        # worker from torch.initial_seed(), which differs per rank / worker)
        rank = torch.distributed.get_rank() if torch.distributed.is_available() and torch.distributed.is_initialized() else 0
        base = torch.initial_seed() if seed is None else int(seed)
        self.rng = random.Random(base * 1000003 + rank)
        self._ws = None            # SynthParams.ws (CLAHE / ISONoise / JPEG / rain / regular chain)
        self._elastic = None       # ElasticTransform displacement [2][S][S] + its scratch

    # ------------------------------------------------------------------ draws
    def sample_params(self, h0: int, w0: int, img: Optional[np.ndarray] = None) -> AugParams:
        """Geometry (+ the regular mode's one-pass photometrics) of one sample."""
        return self._draw(h0, w0, img)[0]

    def _draw(self, h0, w0, img=None):
        """-> (AugParams, extra) where extra holds the host-side pieces of the sample's chain: the regular
        chain's SynthParams + Sharpen kernel when it drew Sharpen or ISONoise, and the GridDistortion maps /
        ElasticTransform seed of the synthetic distortion group."""
        S, r = self.S, self.rng
        nh, nw, ph, pw = letterbox(h0, w0, S)
        M = np.eye(3)                              # forward map canvas -> output (pixel-centre coords)
        bright = contrast = sat = 1.0
        hue, mult, gstd = 0.0, [1.0, 1.0, 1.0], 0.0
        kdist = 0.0
        extra = {}
        if self.mode == "synthetic":
            M = self._geometry(M)
            g = _one_of(r, 0.4, [0.3, 0.3, 0.2, 0.15])           # Optical | Grid | Elastic | Perspective
            if g == 0:
                kdist = r.uniform(-0.3, 0.3) * 0.25                 # distort_limit 0.3 on the normalised radius
            elif g == 1:                                        # GridDistortion(num_steps 6, distort_limit 0.3)
                sx = [1 + r.uniform(-0.3, 0.3) for _ in range(7)]
                sy = [1 + r.uniform(-0.3, 0.3) for _ in range(7)]
                extra["grid"] = grid_distortion_maps(S, sx, sy, 6)
            elif g == 2:                                        # ElasticTransform(alpha 1, sigma 25)
                extra["elastic"] = r.getrandbits(32)
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
                return p, extra
        elif self.mode != "test":
            M = self._geometry(M)
            q = None
            g = _one_of(r, 0.5, [0.7, 0.3])                     # OneOf(ColorJitter p.7, Sharpen p.3) p.5
            if g == 0:
                bright, contrast = r.uniform(0.5, 1.5), r.uniform(0.5, 1.5)
                sat, hue = r.uniform(0.8, 1.2), r.uniform(-0.2, 0.2)
            elif g == 1:                                        # Sharpen(alpha 0.2-0.5, lightness 0.5-1.0)
                q = SynthParams.identity()
                extra["kernel"] = _sharpen_kernel(r.uniform(0.2, 0.5), r.uniform(0.5, 1.0))
            n = _one_of(r, 0.3, [0.5, 0.5, 0.5])                # OneOf(GaussNoise, ISONoise, MultiplicativeNoise) p.3
            if n == 0:
                gstd = r.uniform(0.2, 0.44)
            elif n == 1:                                        # ISONoise defaults: color_shift 0.01-0.05, intensity 0.1-0.5
                q = q or SynthParams.identity()
                q.iso_color_shift, q.iso_intensity = r.uniform(0.01, 0.05), r.uniform(0.1, 0.5)
            elif n == 2:                                        # MultiplicativeNoise(0.9-1.1): one multiplier per channel
                # (albumentations 2.0.8, pinned uv.lock:249-267, samples shape [num_channels] unless elementwise;
                # its per_channel argument is deprecated.  Parity unpinned: albumentations is not installed here)
                mult = [r.uniform(0.9, 1.1) for _ in range(3)]
            if q is not None:                                   # Sharpen / ISONoise: the two-stage regular chain
                q.order = 1
                q.bright, q.contrast, q.sat, q.hue = bright, contrast, sat, hue
                q.gauss_std = gstd
                for i in range(3):
                    q.mult[i] = mult[i]
                if "kernel" in extra:
                    q.ksize = 3
                extra["chain"] = q
        Minv = np.linalg.inv(M)
        p = AugParams()
        for i, v in enumerate(list(Minv[0]) + list(Minv[1])):
            p.A[i] = float(v)
        self._fill(p, h0, w0, nh, nw, ph, pw)
        p.kdist = kdist
        p.raw = int(self.mode == "synthetic" or "chain" in extra)
        p.bright, p.contrast, p.sat, p.hue = bright, contrast, sat, hue
        gm = 0.0
        if contrast != 1.0 and img is not None:       # mean grey of the padded canvas after brightness
            gm = (img[..., 0] * 0.299 + img[..., 1] * 0.587 + img[..., 2] * 0.114).mean() / 255.0
            gm = min(1.0, gm * bright) * (nh * nw) / (S * S)
        p.gray_mean = gm
        if "chain" in extra:
            extra["chain"].gray_mean = gm
        for i in range(3):
            p.mult[i] = mult[i]
        p.gauss_std = gstd
        p.seed = r.getrandbits(32)
        if "chain" in extra:
            extra["chain"].seed = p.seed
        return p, extra

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
        """The synthetic-mode photometric groups (transforms.py:65-216, albumentations 2.0.8 defaults for the
        arguments the reference leaves unset): SynthParams + the composed filter taps + the rain drops."""
        S, r = self.S, self.rng
        q = SynthParams.identity()
        g = _one_of(r, 0.7, [0.7, 0.4, 0.2])                  # ColorJitter | HueSaturationValue | CLAHE
        if g == 0:
            q.bright, q.contrast = r.uniform(0.6, 1.4), r.uniform(0.6, 1.4)
            q.sat, q.hue = r.uniform(0.7, 1.3), r.uniform(-0.2, 0.2)
            if img is not None:
                gm = (img[..., 0] * 0.299 + img[..., 1] * 0.587 + img[..., 2] * 0.114).mean() / 255.0
                q.gray_mean = min(1.0, gm * q.bright)
        elif g == 1:                                          # uint8 HSV: hue in cv2 units of 2 degrees
            q.hsv_h, q.hsv_s, q.hsv_v = 2.0 * r.uniform(-25, 25), r.uniform(-35, 35) / 255.0, r.uniform(-30, 30) / 255.0
        elif g == 2:                                          # CLAHE(clip_limit 4.0 -> U(1, 4), 8x8 tiles)
            q.clahe_clip = r.uniform(1.0, 4.0)
        g = _one_of(r, 0.6, [0.4, 0.4, 0.4])                  # ISONoise | GaussNoise | MultiplicativeNoise
        if g == 0:
            q.iso_color_shift, q.iso_intensity = r.uniform(0.01, 0.03), r.uniform(0.08, 0.3)
        elif g == 1:
            q.gauss_std = r.uniform(0.25, 0.6)
        elif g == 2:                                          # one multiplier per channel (as the regular mode)
            for i in range(3):
                q.mult[i] = r.uniform(0.9, 1.1)
        g = _one_of(r, 0.5, [0.4, 0.3])                       # ImageCompression | Downscale
        if g == 0:
            q.jpeg_quality = r.randint(30, 80)
        elif g == 1:
            q.down = r.uniform(0.4, 0.7)
        g = _one_of(r, 0.5, [0.4, 0.4])                       # RandomShadow | RandomBrightnessContrast
        if g == 0:                                            # 1-3 pentagons in shadow_roi (0, 0.1, 1, 1)
            q.n_shadow, q.shadow_dim = r.randint(1, 3), 0.5
            for t in range(q.n_shadow):
                for v in range(5):
                    q.shadow[t][2 * v], q.shadow[t][2 * v + 1] = r.randrange(0, S), r.randrange(int(0.1 * S), S)
        elif g == 1:
            q.rbc_alpha, q.rbc_beta = 1.0 + r.uniform(-0.4, 0.4), r.uniform(-0.4, 0.4)
        ker = np.ones((1, 1))
        g = _one_of(r, 0.5, [0.4, 0.4, 0.3, 0.2])             # MotionBlur | GaussianBlur | Defocus | ZoomBlur
        if g in (0, 1):
            k = r.choice([3, 5, 7])
            ker = _motion_kernel(r, k) if g == 0 else _gauss_kernel(k)
        elif g == 2:
            ker = _disk_kernel(r.randint(2, 6), r.uniform(0.1, 0.3))
        elif g == 3:                                          # ZoomBlur(max_factor 1.03, step_factor 0.01-0.03)
            z = np.arange(1.0, r.uniform(1.0, 1.03), r.uniform(0.01, 0.03))[:4]
            q.zoom_n = len(z)
            for i, v in enumerate(z):
                q.zoom[i] = float(v)
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
        drops = None
        g = _one_of(r, 0.15, [0.1, 0.1])                      # RandomSnow | RandomRain
        if g == 0:                                            # bleach, snow_point 0.1-0.3, brightness_coeff 2.5
            q.snow_point, q.snow_coeff = r.uniform(0.1, 0.3), 2.5
        elif g == 1:                                          # default rain: S*S // 600 drops of length 20
            slant = int(r.uniform(-10, 10))
            n = S * S // 600
            lo, hi = (-slant, S) if slant < 0 else (0, S - slant)
            drops = np.array([[r.randrange(lo, hi), r.randrange(0, S - 20)] for _ in range(n)], np.int32)
            q.rain_n, q.rain_slant, q.rain_len, q.rain_blur = n, slant, 20, 7
            q.rain_color, q.rain_bright = 200.0 / 255.0, 0.7
        q.ksize = ker.shape[0]
        q.seed = r.getrandbits(32)
        kw = torch.tensor(ker.reshape(-1), dtype=torch.float32).to(self.device, non_blocking=True) if q.ksize > 1 else None
        dr = torch.from_numpy(drops).to(self.device, non_blocking=True) if drops is not None else None
        if dr is not None:
            q.rain_drops = dr.data_ptr()
        return q, kw, dr

    # ------------------------------------------------------------------ device buffers
    def workspace(self):
        if self._ws is None:
            self._ws = torch.empty(augment_ws_floats(self.S), dtype=torch.float32, device=self.device)
        return self._ws

    def _elastic_field(self, seed):
        S = self.S
        if self._elastic is None:
            self._elastic = torch.empty((2, 2, S, S), dtype=torch.float32, device=self.device)
        e = elastic_params(seed)
        lib()("s3od_elastic_field", ctypes.addressof(e), S, self._elastic[1], self._elastic[0], stream())
        return self._elastic[0]

    def _attach(self, p, extra, keep):
        """Device tables of the distortion group -> AugParams pointers."""
        if "grid" in extra:
            gx, gy = extra["grid"]
            g = torch.from_numpy(np.concatenate([gx, gy]).astype(np.float32)).to(self.device, non_blocking=True)
            p.grid = g.data_ptr()
            keep.append(g)
        if "elastic" in extra:
            p.elastic = self._elastic_field(extra["elastic"]).data_ptr()

    def __call__(self, samples: List[Dict[str, np.ndarray]]) -> Dict[str, torch.Tensor]:
        B, S, dev = len(samples), self.S, self.device
        images = torch.empty((B, 3, S, S), dtype=torch.float32, device=dev)
        masks = torch.empty((B, S, S), dtype=torch.float32, device=dev)
        keep = []
        for b, smp in enumerate(samples):
            img = torch.from_numpy(np.ascontiguousarray(smp["image"], dtype=np.uint8)).pin_memory().to(dev, non_blocking=True)
            msk = torch.from_numpy(np.ascontiguousarray(smp["mask"], dtype=np.uint8)).pin_memory().to(dev, non_blocking=True)
            h0, w0 = smp["image"].shape[:2]
            prm, extra = self._draw(h0, w0, smp["image"])
            self._attach(prm, extra, keep)
            if self.mode == "synthetic":
                raw = torch.empty((3, S, S), dtype=torch.float32, device=dev)
                lib()("s3od_augment_sample", img, msk, ctypes.addressof(prm), S, raw, masks[b], stream())
                q, kw, dr = self.synth_params(smp["image"])
                q.ws = self.workspace().data_ptr()
                lib()("s3od_augment_synthetic", raw, ctypes.addressof(q), kw, S, images[b], stream())
                keep.append((img, msk, raw, kw, dr))
                continue
            if "chain" in extra:                       # regular mode drew Sharpen and / or ISONoise
                raw = torch.empty((3, S, S), dtype=torch.float32, device=dev)
                lib()("s3od_augment_sample", img, msk, ctypes.addressof(prm), S, raw, masks[b], stream())
                q = extra["chain"]
                q.ws = self.workspace().data_ptr()
                kw = torch.tensor(extra["kernel"].reshape(-1), dtype=torch.float32).to(dev) if "kernel" in extra else None
                lib()("s3od_augment_synthetic", raw, ctypes.addressof(q), kw, S, images[b], stream())
                keep.append((img, msk, raw, kw))
                continue
            lib()("s3od_augment_sample", img, msk, ctypes.addressof(prm), S, images[b], masks[b], stream())
            keep.append((img, msk))
        self._inflight = keep                          # keep the uploads alive until the kernels ran
        return {"images": images, "masks": masks}
