"""Device batch construction (s3od_augment_sample via GpuAugment).  "test" mode against a numpy
restatement of LongestMaxSize + centred PadIfNeeded + Normalize (bilinear, half-pixel, edge
replicate; masks nearest) to 1e-5; geometric augmentations checked as exact pixel permutations;
reproducibility from the seed.  Parity with albumentations itself is unpinned (not installed)."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
MEAN = np.array([0.485, 0.456, 0.406])
STD = np.array([0.229, 0.224, 0.225])


def _sample(h, w, seed=0):
    r = np.random.default_rng(seed)
    img = r.integers(0, 256, (h, w, 3), dtype=np.uint8)
    mask = (r.random((h, w)) > 0.5).astype(np.uint8) * 255
    return {"image": img, "mask": mask}


def _ref_test_mode(smp, S):
    from s3od_amd.data import letterbox
    img, mask = smp["image"].astype(np.float64), smp["mask"]
    h0, w0 = mask.shape
    nh, nw, ph, pw = letterbox(h0, w0, S)
    canvas = np.zeros((S, S, 3))
    mcan = np.zeros((S, S))
    ys, xs = np.arange(nh), np.arange(nw)
    v = np.clip((ys + 0.5) * (h0 / nh) - 0.5, 0, h0 - 1)
    u = np.clip((xs + 0.5) * (w0 / nw) - 0.5, 0, w0 - 1)
    y0, x0 = v.astype(int), u.astype(int)
    y1, x1 = np.minimum(y0 + 1, h0 - 1), np.minimum(x0 + 1, w0 - 1)
    fy, fx = (v - y0)[:, None, None], (u - x0)[None, :, None]
    top = img[y0][:, x0] * (1 - fx) + img[y0][:, x1] * fx
    bot = img[y1][:, x0] * (1 - fx) + img[y1][:, x1] * fx
    canvas[ph:ph + nh, pw:pw + nw] = (top * (1 - fy) + bot * fy) / 255.0
    sy = np.minimum(np.floor(ys * (h0 / nh)).astype(int), h0 - 1)
    sx = np.minimum(np.floor(xs * (w0 / nw)).astype(int), w0 - 1)
    mcan[ph:ph + nh, pw:pw + nw] = mask[sy][:, sx] / 255.0
    return ((canvas - MEAN) / STD).transpose(2, 0, 1), mcan


@pytest.mark.parametrize("hw", [(300, 200), (97, 160), (128, 128)])
def test_test_mode_matches_restatement(hw):
    from s3od_amd.data import GpuAugment
    smp = _sample(*hw)
    out = GpuAugment(128, mode="test")([smp])
    torch.cuda.synchronize()
    ri, rm = _ref_test_mode(smp, 128)
    assert np.abs(out["images"][0].cpu().numpy() - ri).max() < 1e-4
    assert np.array_equal(out["masks"][0].cpu().numpy(), rm)


def test_flip_and_rot90_are_exact_permutations():
    from s3od_amd.data import GpuAugment, AugParams
    from s3od_amd._lib import lib, stream
    S = 64
    smp = _sample(50, 64, 3)
    aug = GpuAugment(S, mode="test")
    base = aug([smp])
    img = torch.from_numpy(smp["image"]).cuda()
    msk = torch.from_numpy(smp["mask"]).cuda()

    def run(Minv):
        p = aug.sample_params(50, 64)
        for i, v in enumerate(list(Minv[0]) + list(Minv[1])):
            p.A[i] = float(v)
        oi = torch.empty((3, S, S), device="cuda"); om = torch.empty((S, S), device="cuda")
        lib()("s3od_augment_sample", img, msk, ctypes.addressof(p), S, oi, om, stream())
        torch.cuda.synchronize()
        return oi.cpu(), om.cpu()

    fl = np.array([[-1, 0, S], [0, 1, 0], [0, 0, 1]], np.float64)        # x -> S - x (its own inverse)
    oi, om = run(fl)
    assert torch.equal(oi, base["images"][0].cpu().flip(-1)) and torch.equal(om, base["masks"][0].cpu().flip(-1))
    r90 = np.array([[0, -1, S], [1, 0, 0], [0, 0, 1]], np.float64)      # output (x,y) <- canvas (S-y, x)
    oi, om = run(r90)
    assert torch.equal(oi, torch.rot90(base["images"][0].cpu(), 1, (1, 2)))
    assert torch.equal(om, torch.rot90(base["masks"][0].cpu(), 1, (0, 1)))


def test_regular_mode_reproducible_and_sane():
    from s3od_amd.data import GpuAugment
    smps = [_sample(120 + 7 * i, 90 + 11 * i, i) for i in range(6)]
    a = GpuAugment(96, mode="regular", seed=5)(smps)
    b = GpuAugment(96, mode="regular", seed=5)(smps)
    torch.cuda.synchronize()
    assert torch.equal(a["images"], b["images"]) and torch.equal(a["masks"], b["masks"])
    assert torch.isfinite(a["images"]).all()
    lo = torch.tensor(((0 - MEAN) / STD), dtype=torch.float32).view(1, 3, 1, 1).cuda()
    hi = torch.tensor(((1 - MEAN) / STD), dtype=torch.float32).view(1, 3, 1, 1).cuda()
    assert (a["images"] >= lo - 1e-5).all() and (a["images"] <= hi + 1e-5).all()
    assert set(torch.unique(a["masks"]).tolist()) <= {0.0, 1.0}


def _denorm(t):
    return t.cpu().numpy() * STD[:, None, None] + MEAN[:, None, None]


def test_synthetic_identity_chain_equals_test_mode():
    """raw geometry pass + the synthetic photometric passes with every effect at identity == the
    test-mode (letterbox + Normalize) output: the plumbing of the three-pass pipeline is exact."""
    from s3od_amd.data import GpuAugment, SynthParams
    from s3od_amd._lib import lib, stream
    S = 96
    smp = _sample(80, 120, 4)
    base = GpuAugment(S, mode="test")([smp])
    aug = GpuAugment(S, mode="test")
    p = aug.sample_params(80, 120, smp["image"])
    p.raw = 1
    img = torch.from_numpy(smp["image"]).cuda(); msk = torch.from_numpy(smp["mask"]).cuda()
    raw = torch.empty(3, S, S, device="cuda"); om = torch.empty(S, S, device="cuda"); out = torch.empty(3, S, S, device="cuda")
    lib()("s3od_augment_sample", img, msk, ctypes.addressof(p), S, raw, om, stream())
    q = SynthParams.identity()
    lib()("s3od_augment_synthetic", raw, ctypes.addressof(q), None, S, out, stream())
    torch.cuda.synchronize()
    assert float((out - base["images"][0]).abs().max()) < 1e-5
    assert torch.equal(om, base["masks"][0])


@pytest.mark.parametrize("what", ["gray", "posterize", "blur_const", "shuffle"])
def test_synthetic_effects_exact_properties(what):
    from s3od_amd.data import SynthParams
    from s3od_amd._lib import lib, stream
    S = 64
    g = torch.Generator(device="cuda").manual_seed(1)
    raw = torch.rand(3, S, S, device="cuda", generator=g)
    if what == "blur_const":
        raw = torch.full((3, S, S), 0.3, device="cuda")
    ref = raw.clone()
    q = SynthParams.identity()
    kw = None
    if what == "gray":
        q.color_op = 2
    elif what == "posterize":
        q.post_bits = 5
    elif what == "blur_const":
        q.ksize = 5
        kw = torch.full((25,), 1 / 25, device="cuda")
    elif what == "shuffle":
        q.color_op = 3
        q.perm[0], q.perm[1], q.perm[2] = 2, 0, 1
    out = torch.empty(3, S, S, device="cuda")
    lib()("s3od_augment_synthetic", raw, ctypes.addressof(q), kw, S, out, stream())
    torch.cuda.synchronize()
    v = _denorm(out)
    r = ref.cpu().numpy()
    if what == "gray":
        assert np.abs(v[0] - v[1]).max() < 1e-5 and np.abs(v[1] - v[2]).max() < 1e-5
        assert np.abs(v[0] - (0.299 * r[0] + 0.587 * r[1] + 0.114 * r[2])).max() < 1e-5
    elif what == "posterize":
        q8 = np.round(v * 255)
        assert np.abs(v * 255 - q8).max() < 1e-3 and (q8.astype(int) % 8 == 0).all()
    elif what == "blur_const":
        assert np.abs(v - 0.3).max() < 1e-5
    elif what == "shuffle":
        assert np.abs(v - r[[2, 0, 1]]).max() < 1e-5


def test_synthetic_mode_reproducible_and_sane():
    from s3od_amd.data import GpuAugment
    smps = [_sample(120 + 7 * i, 90 + 11 * i, i) for i in range(8)]
    a = GpuAugment(96, mode="synthetic", seed=9)(smps)
    b = GpuAugment(96, mode="synthetic", seed=9)(smps)
    torch.cuda.synchronize()
    assert torch.equal(a["images"], b["images"]) and torch.equal(a["masks"], b["masks"])
    lo = torch.tensor(((0 - MEAN) / STD), dtype=torch.float32).view(1, 3, 1, 1).cuda()
    hi = torch.tensor(((1 - MEAN) / STD), dtype=torch.float32).view(1, 3, 1, 1).cuda()
    assert torch.isfinite(a["images"]).all()
    assert (a["images"] >= lo - 1e-5).all() and (a["images"] <= hi + 1e-5).all()
    assert set(torch.unique(a["masks"]).tolist()) <= {0.0, 1.0}
    assert a["masks"].sum() > 0
