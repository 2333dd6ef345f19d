"""GPU checks of the drop-in inference API on the reference's own fixture image
(tests/fixture/image.jpg, copied from the reference's tests/fixture) with the synthetic weights.

strict (f32): IoU scores ≤ 1e-5 relative, best_idx bit-exact, mask-logit sign agreement
(per-pixel IoU of logit>0) ≥ 0.999, predicted mask ≤ 1e-4, alpha channel sum within 0.1 %.
bf16: best_idx bit-exact and mask IoU vs the reference ≥ 0.99 (reported).
Reference contract checks (tests/test_fixture_inference.py:92-116): 3 masks, 3 ious in [0,1],
predicted_mask == all_masks[argmax(all_ious)] bit-exact, RGBA size == input size.
"""
import numpy as np
import pytest
import torch
from PIL import Image

from conftest import GOLDEN, FIXTURE

pytestmark = pytest.mark.gpu


def iou(a, b):
    u = np.logical_or(a, b).sum()
    return 1.0 if u == 0 else float(np.logical_and(a, b).sum() / u)


@pytest.fixture(scope="module")
def br():
    from s3od import BackgroundRemoval
    return BackgroundRemoval("synthetic", compute_dtype="f32")


def test_fixture_strict(br):
    g = np.load(GOLDEN / "fixture_1024.npz")
    img = Image.open(FIXTURE / "image.jpg").convert("RGB")
    arr = np.array(img)
    assert int(arr.astype(np.int64).sum()) == int(g["image_u8_sum"])
    x, pad = br._preprocess(arr)
    assert np.abs(x[0, :, ::8, ::8].cpu().numpy() - g["x_sub"]).max() == 0.0   # bit-exact normalisation
    res = br.remove_background(img)
    assert res.all_masks.shape == (3, 1024, 1024) and res.all_ious.shape == (3,)
    assert np.all(res.all_ious >= 0) and np.all(res.all_ious <= 1)
    np.testing.assert_array_equal(res.predicted_mask, res.all_masks[res.all_ious.argmax()])
    assert res.rgba_image.size == img.size and res.rgba_image.mode == "RGBA"
    assert int(res.all_ious.argmax()) == int(g["best_idx"])
    assert np.abs(res.all_ious - g["all_ious"]).max() <= 1e-5 * np.abs(g["all_ious"]).max()
    assert np.abs(res.predicted_mask[::8, ::8] - g["predicted_mask_sub"]).max() <= 1e-4
    alpha = np.array(res.rgba_image)[:, :, 3].astype(np.int64)
    assert abs(alpha.sum() - int(g["alpha_sum"])) <= 1e-3 * int(g["alpha_sum"])
    with torch.no_grad():
        lg = br.model(x)["pred_masks"][0].cpu().numpy()
    ref_bits = np.unpackbits(g["mask_pos_bits"])[: lg.size].astype(bool).reshape(lg.shape)
    m_iou = iou(lg > 0, ref_bits)
    print(f"strict fixture: mask IoU vs reference {m_iou:.6f}")
    assert m_iou >= 0.999


def test_fixture_bf16(br):
    """bf16 on the fixture: best_idx bit-exact; mask IoU vs the reference's sign bits, with the flip band
    SURVEY §8(c) asks for (the fraction of pixels whose strict logit |l| < 2·max|Δ_bf16|: IoU >= 0.999 only
    means something when that band is < 1e-3; with the synthetic weights most logits sit near 0).  The
    strict f32 logits stand in for the reference's values (pinned above: sign IoU >= 0.999, ≤ 1e-4 on
    the mask).  The numbers are written to gpurun_out/bf16_fixture_iou.json when that directory exists."""
    import json
    import os
    g = np.load(GOLDEN / "fixture_1024.npz")
    img = Image.open(FIXTURE / "image.jpg").convert("RGB")
    x, _ = br._preprocess(np.array(img))
    with torch.no_grad():
        l32 = br.model(x)["pred_masks"][0].float().cpu().numpy()
    br.model.compute_dtype = "bf16"
    try:
        res = br.remove_background(img)
        with torch.no_grad():
            lg = br.model(x)["pred_masks"][0].float().cpu().numpy()
    finally:
        br.model.compute_dtype = "f32"
    ref_bits = np.unpackbits(g["mask_pos_bits"])[: lg.size].astype(bool).reshape(lg.shape)
    m_iou = iou(lg > 0, ref_bits)
    d = np.abs(lg - l32)
    maxd = float(d.max())
    band = float((np.abs(l32) < 2 * maxd).mean())
    outside = np.abs(l32) >= 2 * maxd
    rec = {"mask_iou_vs_reference": m_iou, "mask_iou_vs_strict": iou(lg > 0, l32 > 0),
           "max_abs_logit_diff": maxd, "rel_l2_logits": float(np.linalg.norm(lg - l32) / np.linalg.norm(l32)),
           "flip_band_fraction": band, "sign_agreement_outside_band": float(((lg > 0) == (l32 > 0))[outside].mean()),
           "median_abs_logit": float(np.median(np.abs(l32))), "best_idx": int(res.all_ious.argmax()),
           "best_idx_ref": int(g["best_idx"]),
           "note": "synthetic weights (real ones are not available offline); strict f32 logits stand in for the reference's"}
    print("bf16 fixture:", json.dumps(rec))
    if os.path.isdir("gpurun_out"):
        json.dump(rec, open("gpurun_out/bf16_fixture_iou.json", "w"), indent=1)
    assert int(res.all_ious.argmax()) == int(g["best_idx"])
    assert rec["sign_agreement_outside_band"] == 1.0
    assert m_iou >= 0.99


@pytest.mark.parametrize("shape", [(100, 100), (400, 800), (800, 400), (2000, 2000), (480, 640), (20, 30), (31, 31), (40, 4000)])
def test_output_shape_matches_input(br, shape):
    """tests/test_inference_package.py:49-122 (shape contract; resize parity unpinned: cv2 absent)."""
    rng = np.random.default_rng(0)
    img = rng.integers(0, 255, (*shape, 3), dtype=np.uint8)
    res = br.remove_background(img)
    assert res.predicted_mask.shape == shape
    assert res.all_masks.shape == (3, *shape)
    assert np.all(np.isfinite(res.all_masks)) and res.all_masks.min() >= 0 and res.all_masks.max() <= 1 + 1e-6


def test_odd_padding_quirk(br):
    img = np.zeros((100, 152, 3), np.uint8)       # 1024 - int(1024/1.52) = 351 is odd
    with pytest.raises(ValueError):
        br.remove_background(img)


def test_missing_model_raises():
    from s3od import BackgroundRemoval
    with pytest.raises(ValueError):
        BackgroundRemoval(model_id="nonexistent_model.pt")
