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
    for _ in range(400):
        q, kw = aug.synth_params(img)
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
    # reproducible from the seed
    a = GpuAugment(128, mode="synthetic", device="cpu", seed=11)
    b = GpuAugment(128, mode="synthetic", device="cpu", seed=11)
    for _ in range(20):
        qa, _ = a.synth_params(img); qb, _ = b.synth_params(img)
        assert bytes(qa) == bytes(qb)
