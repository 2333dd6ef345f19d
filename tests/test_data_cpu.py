"""MaskDataset file discovery and train/val split (synth_sod/.../dataset.py:34-106) on CPU."""
import random

import numpy as np
from PIL import Image

from s3od_amd.data import MaskDataset, letterbox


def _make(root, names, mask_ext=".png", skip_mask=()):
    (root / "images").mkdir()
    (root / "masks").mkdir()
    for n in names:
        Image.fromarray(np.full((6, 8, 3), 7, np.uint8)).save(root / "images" / n)
        stem = n.rsplit(".", 1)[0]
        if stem not in skip_mask:
            Image.fromarray(np.full((6, 8), 255, np.uint8)).save(root / "masks" / (stem + mask_ext))


def test_split_matches_reference_rule(tmp_path):
    names = [f"img_{i:03d}.jpg" for i in range(37)] + ["x.png", "notes.txt"]
    _make(tmp_path, [n for n in names if not n.endswith(".txt")], skip_mask=("img_005",))
    (tmp_path / "images" / "notes.txt").write_text("not an image")
    tr = MaskDataset(str(tmp_path), 64, split="train", val_split=0.2, seed=42)
    va = MaskDataset(str(tmp_path), 64, split="val", val_split=0.2, seed=42)
    # restated reference rule: valid = sorted(images with a mask); random.seed(seed); shuffle; val first
    valid = sorted(n for n in names if not n.endswith(".txt") and not n.startswith("img_005"))
    random.seed(42)
    random.shuffle(valid)
    nv = int(len(valid) * 0.2)
    assert va.files == valid[:nv] and tr.files == valid[nv:]
    item = tr[0]
    assert item["image"].shape == (6, 8, 3) and item["image"].dtype == np.uint8 and item["mask"].shape == (6, 8)
    sub = MaskDataset(str(tmp_path), 64, split="train", val_split=0.2, seed=42, debug_subset_fraction=0.5)
    assert sub.files == tr.files[:int(len(tr.files) * 0.5)]


def test_letterbox_geometry():
    assert letterbox(480, 640, 1024) == (768, 1024, 128, 0)
    assert letterbox(1024, 1024, 1024) == (1024, 1024, 0, 0)
    nh, nw, ph, pw = letterbox(300, 1000, 512)
    assert nw == 512 and nh == 154 and ph == (512 - 154) // 2 and pw == 0


def test_synthetic_params_host_logic():
    """Host half of mode="synthetic": every draw is inside the kernel's contract (odd filter <= 15,
    normalised blur taps, valid colour op / posterize / downscale), and the perspective branch gives
    a finite projective map with the same geometry as the mask (one AugParams drives both)."""
    import torch
    from s3od_amd.data import GpuAugment
    aug = GpuAugment(128, mode="synthetic", device="cpu", seed=3)
    img = np.random.default_rng(0).integers(0, 256, (90, 140, 3), dtype=np.uint8)
    seen_k, seen_op, persp = set(), set(), 0
    seen = set()
    for _ in range(400):
        q, kw, dr = aug.synth_params(img)
        assert q.clahe_clip == 0 or 1.0 <= q.clahe_clip <= 4.0
        assert q.jpeg_quality == 0 or 30 <= q.jpeg_quality <= 80
        assert 0 <= q.zoom_n <= 3 and (q.zoom_n == 0 or (q.zoom[0] == 1.0 and all(1.0 <= q.zoom[i] < 1.03 for i in range(q.zoom_n))))
        assert q.snow_point == 0 or 0.1 <= q.snow_point <= 0.3
        assert (dr is None) == (q.rain_n == 0)
        if dr is not None:                                   # drops stay on the canvas (x + slant too)
            d = dr.numpy()
            assert d.shape == (128 * 128 // 600, 2) and -10 < q.rain_slant < 10
            assert (d[:, 0] + min(q.rain_slant, 0) >= 0).all() and (d[:, 0] + max(q.rain_slant, 0) < 128).all()
            assert (d[:, 1] >= 0).all() and (d[:, 1] + 20 < 128).all()
        seen.update(k for k, on in (("clahe", q.clahe_clip > 0), ("iso", q.iso_intensity > 0), ("jpeg", q.jpeg_quality > 0),
                                    ("zoom", q.zoom_n > 0), ("snow", q.snow_point > 0), ("rain", q.rain_n > 0),
                                    ("shadow", q.n_shadow > 0)) if on)
        assert q.ksize % 2 == 1 and 1 <= q.ksize <= 15
        assert (kw is None) == (q.ksize == 1)
        if kw is not None:
            assert kw.numel() == q.ksize ** 2 and torch.isfinite(kw).all() and float(kw.sum()) > 0.3
        assert 0 <= q.color_op <= 3 and sorted(q.perm) == [0, 1, 2]
        assert q.post_bits in (5, 8) and 0.4 <= q.down <= 1.0 and 0 <= q.n_shadow <= 3
        assert 0.0 <= q.gray_mean <= 1.0
        seen_k.add(q.ksize); seen_op.add(q.color_op)
        p = aug.sample_params(90, 140, img)
        assert p.raw == 1 and all(np.isfinite(list(p.A))) and np.isfinite(p.persp[0]) and np.isfinite(p.persp[1])
        persp += p.persp[0] != 0 or p.persp[1] != 0
    assert len(seen_k) >= 4 and len(seen_op) >= 2 and persp > 0
    assert seen == {"clahe", "iso", "jpeg", "zoom", "snow", "rain", "shadow"}, seen
    # reproducible from the seed
    a = GpuAugment(128, mode="synthetic", device="cpu", seed=11)
    b = GpuAugment(128, mode="synthetic", device="cpu", seed=11)
    for _ in range(20):
        qa, _, _ = a.synth_params(img); qb, _, _ = b.synth_params(img)
        qa.rain_drops = qb.rain_drops = None
        assert bytes(qa) == bytes(qb)


def test_synthetic_mode_rejects_sizes_clahe_cannot_tile():
    """CLAHE's 8x8 tile grid needs S % 8 == 0: the synthetic pipeline fails when built, not at the random
    step that first draws CLAHE."""
    import pytest
    from s3od_amd.data import GpuAugment
    with pytest.raises(ValueError, match="divisible by 8"):
        GpuAugment(100, mode="synthetic", device="cpu", seed=1)
    GpuAugment(100, mode="regular", device="cpu", seed=1)     # regular mode draws no CLAHE


def test_multiplicative_noise_draws_one_multiplier_per_channel():
    """albumentations 2.x MultiplicativeNoise samples shape [num_channels] (per_channel deprecated)."""
    from s3od_amd.data import GpuAugment
    aug = GpuAugment(64, mode="synthetic", device="cpu", seed=7)
    img = np.zeros((64, 64, 3), np.uint8)
    seen = 0
    for _ in range(300):
        q, _, _ = aug.synth_params(img)
        m = list(q.mult)
        if m != [1.0, 1.0, 1.0]:
            assert len(set(m)) == 3 and all(0.9 <= v <= 1.1 for v in m)
            seen += 1
    assert seen > 0


def test_grid_distortion_maps_cover_the_image():
    """GridDistortion(num_steps=6) normalised steps: the source maps start at 0, increase, and end at the
    image width (so the distorted grid never leaves the image), for sizes that are not multiples of 6."""
    from s3od_amd.data import grid_distortion_maps
    r = np.random.default_rng(0)
    for S in (64, 100, 1024):
        for _ in range(5):
            gx, gy = grid_distortion_maps(S, 1 + r.uniform(-0.3, 0.3, 7), 1 + r.uniform(-0.3, 0.3, 7), 6)
            for g in (gx, gy):
                assert g.shape == (S,) and g[0] == 0 and np.all(np.diff(g) >= 0)      # segment ends repeat (linspace endpoints)
                assert abs(float(g[-1]) - S) < 1e-3 * S


def test_regular_mode_draws_sharpen_and_iso_chain():
    """mode="regular": Sharpen (OneOf weight 0.3 of p 0.5) and ISONoise (1/3 of p 0.3) are drawn at their
    reference rates and route the sample through the two-stage chain (raw geometry + order-1 chain)."""
    from s3od_amd.data import GpuAugment
    aug = GpuAugment(64, mode="regular", device="cpu", seed=5)
    n, sharpen, iso = 4000, 0, 0
    for _ in range(n):
        p, extra = aug._draw(50, 60)
        q = extra.get("chain")
        if q is not None:
            assert p.raw == 1 and q.order == 1
            sharpen += q.ksize == 3
            iso += q.iso_intensity > 0
            if q.ksize == 3:
                assert extra["kernel"].shape == (3, 3)
            if q.iso_intensity > 0:
                assert 0.1 <= q.iso_intensity <= 0.5 and 0.01 <= q.iso_color_shift <= 0.05
        else:
            assert p.raw == 0
    assert abs(sharpen / n - 0.5 * 0.3) < 0.025 and abs(iso / n - 0.3 / 3) < 0.02, (sharpen / n, iso / n)


def test_jpeg_restatement_matches_libjpeg():
    """The ImageCompression restatement (oracle/augment_oracle.py jpeg, which the device kernels are
    tested against) vs a real libjpeg encode/decode (PIL, quality q, 4:2:0): the same codec family
    cv2.imencode / imdecode use.  Differences come from libjpeg's integer DCT and fixed-point colour
    conversion: mean <= 1 8-bit step, and the restatement's loss vs the input within 5 % of libjpeg's."""
    import io
    from PIL import Image
    from oracle import augment_oracle as AO
    r = np.random.default_rng(0)
    for S in (64, 72):
        yy, xx = np.mgrid[0:S, 0:S] / S
        x = np.clip(np.stack([xx, yy, 0.5 + 0.3 * np.sin(6 * xx)]) + 0.15 * r.random((3, S, S)), 0, 1)
        for q in (30, 55, 80):
            u8 = np.rint(x * 255).astype(np.uint8).transpose(1, 2, 0)
            buf = io.BytesIO()
            Image.fromarray(u8).save(buf, format="JPEG", quality=q, subsampling=2)
            lj = np.asarray(Image.open(io.BytesIO(buf.getvalue())).convert("RGB")).transpose(2, 0, 1) / 255.0
            o = AO.jpeg(x, q)
            assert np.abs(o - lj).mean() * 255 <= 1.0, (S, q, np.abs(o - lj).mean() * 255)
            lo, ll = np.abs(o - u8.transpose(2, 0, 1) / 255.0).mean(), np.abs(lj - u8.transpose(2, 0, 1) / 255.0).mean()
            assert abs(lo - ll) <= 0.05 * ll, (S, q, lo, ll)
