"""Pin the CPU oracle (oracle/s3od_oracle.py) to the reference's own outputs.

The goldens were produced by importing /root/reference in the build container
(tests/golden/make_golden.py) on the synthetic weights of s3od_amd/weights.py.
Tolerance: fp32 vs fp32 with different op order → ≤1e-4 relative (max-abs / max-ref).
"""
import numpy as np
import pytest
import torch

from conftest import GOLDEN, FIXTURE
from oracle import s3od_oracle as O


def rel(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-12))


@pytest.mark.parametrize("name", ["fwd_eval_224x224_b2", "fwd_eval_160x256_b1"])
def test_forward_eval(name, synth_sd_torch):
    g = np.load(GOLDEN / f"{name}.npz")
    with torch.no_grad():
        x = torch.from_numpy(g["x"])
        taps = O.encoder_taps(x, synth_sd_torch)
        out = O.dpt_head(taps, synth_sd_torch, x.shape[2] // 16, x.shape[3] // 16)
    for i, t in enumerate(taps):
        assert rel(t[:, :, ::8].numpy(), g[f"tap{i}_sub"]) < 1e-4
    assert rel(out["pred_masks"].numpy(), g["pred_masks"]) < 1e-4
    assert rel(out["pred_iou"].numpy(), g["pred_iou"]) < 1e-4
    assert rel(out["features"][:, :, ::4, ::4].numpy(), g["features_sub"]) < 1e-4


def test_fixture_1024(synth_sd_torch):
    from PIL import Image
    g = np.load(GOLDEN / "fixture_1024.npz")
    img = np.array(Image.open(FIXTURE / "image.jpg").convert("RGB"))
    assert int(img.astype(np.int64).sum()) == int(g["image_u8_sum"])     # same JPEG decode
    x = O.normalize(img)
    assert rel(x[0, :, ::8, ::8].numpy(), g["x_sub"]) < 1e-6
    with torch.no_grad():
        out = O.forward(x, synth_sd_torch)
    lg = out["pred_masks"][0].numpy()
    assert rel(lg[:, ::8, ::8], g["logits_sub"]) < 1e-4
    assert rel(out["pred_iou"][0].numpy(), g["pred_iou"]) < 1e-4
    bits = np.unpackbits(g["mask_pos_bits"])[: lg.size].astype(bool)
    agree = (bits == (lg.reshape(-1) > 0)).mean()
    assert agree > 0.9999
    pad = O.get_pad_info(1024, 1024, 1024)
    allm, ious, best = O.postprocess(out["pred_masks"], out["pred_iou"], pad)
    assert int(best) == int(g["best_idx"])
    assert rel(ious, g["all_ious"]) < 1e-5
    assert rel(allm[best][::8, ::8], g["predicted_mask_sub"]) < 1e-4


@pytest.mark.parametrize("cfgname", ["focal_iou", "bce_iou_ssim"])
@pytest.mark.parametrize("epoch", [0, 3])
def test_loss(cfgname, epoch):
    g = np.load(GOLDEN / "loss_goldens.npz")
    cfg = O.FOCAL_IOU if cfgname == "focal_iou" else O.BCE_IOU_SSIM
    lg = torch.from_numpy(g["logits"]).requires_grad_(True)
    pi = torch.from_numpy(g["pred_iou"]).requires_grad_(True)
    loss, parts, best, ious = O.multi_mask_loss({"pred_masks": lg, "pred_iou": pi}, torch.from_numpy(g["masks"]), epoch, cfg)
    loss.backward()
    tag = f"{cfgname}_e{epoch}"
    assert abs(loss.item() - float(g[f"{tag}_loss"])) <= 1e-5 * abs(float(g[f"{tag}_loss"]))
    names = list(g[f"{tag}_parts_names"])
    vals = g[f"{tag}_parts_values"]
    for n, v in zip(names, vals):
        assert abs(float(parts[n]) - v) <= 1e-5 * max(abs(v), 1e-6), n
    assert rel(lg.grad.numpy(), g[f"{tag}_grad_logits"]) < 1e-4
    assert rel(pi.grad.numpy(), g[f"{tag}_grad_iou"]) < 1e-4


def is_bn_fed_bias(n):
    return "resConfUnit" in n and (n.endswith("conv1.bias") or n.endswith("conv2.bias"))


def test_train_step(synth_sd_torch):
    g = np.load(GOLDEN / "train_256_b2.npz")
    sd = {k: (v.clone().float() if v.is_floating_point() else v.clone()) for k, v in synth_sd_torch.items()}
    params = {k: v.requires_grad_(True) for k, v in sd.items()
              if v.is_floating_point() and "running" not in k}
    x = torch.from_numpy(g["x"])
    out = O.forward(x, sd, train=True, rope_rescale=float(g["rescale"]))
    loss, parts, best, ious = O.multi_mask_loss(out, torch.from_numpy(g["masks"]), int(g["epoch"]))
    loss.backward()
    assert abs(loss.item() - float(g["loss"])) < 1e-4 * abs(float(g["loss"]))
    assert rel(out["pred_masks"].detach().numpy(), g["pred_masks"]) < 1e-4
    for n, v in zip(g["parts_names"], g["parts_values"]):
        assert abs(float(parts[n]) - v) <= 1e-4 * max(abs(v), 1e-6), n
    names = list(g["grad_names"])
    got = {n for n, p in params.items() if p.grad is not None and p.grad.abs().sum() > 0}
    assert set(names) <= set(params)
    for n, nrm, sl in zip(names, g["grad_norms"], g["grad_slices"]):
        gr = params[n].grad
        assert gr is not None, n
        if is_bn_fed_bias(n):
            # conv bias feeding a train-mode BN: exact gradient is 0, both sides are noise
            w = params[n.replace(".bias", ".weight")].grad
            assert float(gr.norm()) < 1e-3 * float(w.norm()), n
            continue
        assert abs(float(gr.norm()) - nrm) <= 1e-3 * max(nrm, 1e-8) + 1e-9, (n, float(gr.norm()), nrm)
        rms = nrm / np.sqrt(gr.numel())
        k = np.isfinite(sl)
        a = np.pad(gr.reshape(-1)[:32].numpy(), (0, 32 - min(32, gr.numel())))[k]
        assert np.abs(a - sl[k]).max() <= 3e-2 * rms + 1e-12, n
    # parameters that never receive a gradient in the reference (layer 11, final norm,
    # mask_token, refinenet4.resConfUnit1): SURVEY §8a A6
    unused = set(params) - set(names)
    assert any(".layer.11." in n for n in unused) and "encoder.norm.weight" in unused
    bn = dict(zip(g["bn_names"], g["bn_values"]))
    for n, v in bn.items():
        k = n if n.startswith("seg_head") else n
        assert rel(sd[k].numpy(), v) < 1e-4, n


def _dinol_sd():
    from s3od_amd.weights import synthetic_state_dict
    return {k: torch.from_numpy(v) for k, v in synthetic_state_dict(0, "dinol", 1).items()}


def test_dinol_forward_eval():
    """dinol (ViT-L/16, taps [4,11,17,23], num_outputs=1) vs the reference built by make_golden.py --dinol."""
    g = np.load(GOLDEN / "dinol.npz")
    with torch.no_grad():
        out = O.forward(torch.from_numpy(g["fwd_x"]), _dinol_sd())
    assert tuple(out["pred_masks"].shape) == tuple(g["fwd_pred_masks"].shape) == (1, 1, 128, 160)
    assert rel(out["pred_masks"].numpy(), g["fwd_pred_masks"]) < 1e-4
    assert rel(out["pred_iou"].numpy(), g["fwd_pred_iou"]) < 1e-4
    assert rel(out["features"][:, :, ::4, ::4].numpy(), g["fwd_features_sub"]) < 1e-4


def test_dinol_train_step_single_mask_loss():
    """loss.py:166-188 single-mask branch + backward through ViT-L: loss, parts, grad norms / slices,
    the 32 parameters without gradient (layer 23, final norm, mask_token, refinenet4.resConfUnit1,
    classifier_head), BN running stats."""
    g = np.load(GOLDEN / "dinol.npz")
    sd = _dinol_sd()
    params = {k: v.requires_grad_(True) for k, v in sd.items() if v.is_floating_point() and "running" not in k}
    out = O.forward(torch.from_numpy(g["train_x"]), sd, train=True, rope_rescale=float(g["rescale"]))
    loss, parts = O.single_mask_loss(out, torch.from_numpy(g["train_masks"]))
    loss.backward()
    assert abs(loss.item() - float(g["loss"])) < 1e-4 * abs(float(g["loss"]))
    for n, v in zip(g["parts_names"], g["parts_values"]):
        assert abs(float(parts[n]) - v) <= 1e-4 * max(abs(v), 1e-6), n
    for n, nrm, sl in zip(g["grad_names"], g["grad_norms"], g["grad_slices"]):
        gr = params[n].grad
        assert gr is not None, n
        if is_bn_fed_bias(n):
            continue
        assert abs(float(gr.norm()) - nrm) <= 1e-3 * max(nrm, 1e-8) + 1e-9, (n, float(gr.norm()), nrm)
        rms = nrm / np.sqrt(gr.numel())
        k = np.isfinite(sl)
        a = np.pad(gr.reshape(-1)[:32].numpy(), (0, 32 - min(32, gr.numel())))[k]
        assert np.abs(a - sl[k]).max() <= 3e-2 * rms + 1e-12, n
    nograd = set(g["nograd_names"])
    assert len(nograd) == 32 and any(".layer.23." in n for n in nograd)
    assert "seg_head.classifier_head.4.weight" in nograd
    for n, v in zip(g["bn_names"], g["bn_values"]):
        assert rel(sd[n].numpy(), v) < 1e-4, n


# ---------------------------------------------------------------- evaluation metrics (f4)
METRIC_TOL = {"mae": 1e-12, "max_f": 1e-7, "avg_f": 5e-7, "s_score": 5e-7, "em": 1e-12, "wfm": 1e-12}


def test_metrics_oracle_matches_reference_goldens():
    """oracle/metrics_oracle.py vs the reference's EvaluationMetrics run on CPU (metrics.npz)."""
    from oracle import metrics_oracle as M
    d = np.load(GOLDEN / "metrics.npz")
    per = []
    for n in d["names"]:
        r = M.step(d[f"{n}/pred"], d[f"{n}/gt"])
        v = np.array([r[k] for k in M.KEYS])
        g = d[f"{n}/values"]
        per.append(v)
        for i, k in enumerate(M.KEYS):
            if np.isnan(g[i]):
                assert np.isnan(v[i]), (n, k)
            else:
                assert abs(v[i] - g[i]) <= METRIC_TOL[k] * max(1.0, abs(g[i])), (n, k, v[i], g[i])
        s = M.step(d[f"{n}/pred"], d[f"{n}/gt"], sm_only=True)["s_score"]
        assert (np.isnan(s) and np.isnan(d[f"{n}/sm_only"][0])) or abs(s - d[f"{n}/sm_only"][0]) < 5e-7
    agg = dict(zip(d["aggregate_keys"], d["aggregate"]))
    per = np.array(per)
    for i, k in enumerate(("MAE", "MaxF", "AvgF", "Sm", "Em", "wF")):
        a, b = np.mean(per[:, i]), agg[k]
        assert (np.isnan(a) and np.isnan(b)) or abs(a - b) < 1e-6, k


def test_edt_restatement_matches_scipy_ties():
    """The distance-transform algorithm the HIP kernel runs picks scipy's nearest foreground pixel,
    ties included (so the weighted-F 'Et' gather is identical)."""
    from scipy.ndimage import distance_transform_edt
    from oracle.metrics_oracle import edt_nearest
    r = np.random.default_rng(4)
    for t in range(25):
        H, W = r.integers(4, 26, 2)
        fg = r.random((H, W)) < r.uniform(0.02, 0.35)
        if t % 5 == 0:
            yy, xx = np.mgrid[:H, :W]
            fg = ((yy - H / 2) ** 2 / 9 + (xx - W / 3) ** 2 / 16) < 1
        if not fg.any():
            fg[H // 2, W // 2] = True
        _, idx = distance_transform_edt(fg == 0, return_indices=True)
        iy, ix = edt_nearest(fg)
        assert (iy == idx[0]).all() and (ix == idx[1]).all()
