"""Generate the committed golden fixtures by running the REFERENCE itself (this container only).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference (``/root/reference``, read-only) is imported with two shims that SURVEY.md §8c
documents: a stub ``cv2`` (``s3od/__init__`` imports predictor → cv2; only the identity
resize of a square 1024² image is ever used here) and a stub ``AutoImageProcessor`` (needs
torchvision, unused in forward).  ``hydra.utils.instantiate`` is stubbed for LossModule.
Weights are the deterministic synthetic scheme of ``s3od_amd/weights.py``.

Outputs (small .npz files next to this script) are DATA: inputs + reference outputs.
Nothing under /root/reference is copied; the GPU box never needs it.
"""
from __future__ import annotations

import importlib
import math
import os
import sys
import types
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
REF = Path("/root/reference")
sys.path.insert(0, str(REPO))

from s3od_amd.weights import synthetic_state_dict  # noqa: E402


def _install_shims():
    sys.modules.setdefault("cv2", types.SimpleNamespace(
        resize=lambda img, size, *a, **k: _identity_resize(img, size)))
    hydra = types.ModuleType("hydra")
    utils = types.ModuleType("hydra.utils")

    def instantiate(cfg, **kw):
        cfg = {k: _num(v) for k, v in dict(cfg).items()}
        target = cfg.pop("_target_")
        mod, name = target.rsplit(".", 1)
        return getattr(importlib.import_module(mod), name)(**cfg, **kw)
    utils.instantiate = instantiate
    hydra.utils = utils
    sys.modules["hydra"] = hydra
    sys.modules["hydra.utils"] = utils
    sys.path.insert(0, str(REF / "src"))
    sys.path.insert(0, str(REF / "synth_sod" / "src"))


def _num(v):
    """OmegaConf's YAML loader reads '1e-6' as a float; PyYAML's safe_load does not."""
    if isinstance(v, str):
        try:
            return float(v)
        except ValueError:
            return v
    return v


def _identity_resize(img, size):
    if tuple(size) != (img.shape[1], img.shape[0]):
        raise RuntimeError("stub cv2.resize only supports the identity (square 1024² fixture)")
    return img


def build_reference_model(seed=0):
    import s3od.model as M
    M.AutoImageProcessor = types.SimpleNamespace(from_pretrained=lambda *a, **k: None)
    m = M.DPTSegmentation(num_classes=1, num_outputs=3, encoder_name="dinov3_base")
    sd = {k: torch.from_numpy(v) for k, v in synthetic_state_dict(seed).items()}
    m.load_state_dict(sd, strict=True)
    return m


def seeded_images(B, H, W, seed):
    """uint8 ~ U[0,255] normalised with the ImageNet mean/std."""
    g = np.random.Generator(np.random.Philox(key=seed))
    u8 = g.integers(0, 256, size=(B, H, W, 3), dtype=np.uint8)
    x = (u8.astype(np.float32) / 255.0 - np.array([0.485, 0.456, 0.406])) / np.array([0.229, 0.224, 0.225])
    return torch.from_numpy(x).permute(0, 3, 1, 2).float().contiguous()


def ellipse_masks(B, H, W, seed):
    """1–3 random filled ellipses per image, binary float."""
    g = np.random.Generator(np.random.Philox(key=seed))
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    out = np.zeros((B, H, W), np.float32)
    for b in range(B):
        for _ in range(int(g.integers(1, 4))):
            cy, cx = g.uniform(0.2, 0.8) * H, g.uniform(0.2, 0.8) * W
            ry, rx = g.uniform(0.08, 0.3) * H, g.uniform(0.08, 0.3) * W
            out[b][((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 <= 1.0] = 1.0
    return torch.from_numpy(out)


def _taps(m, x):
    feats = m.extract_intermediate_features(x)
    return [f[0] for f in feats]


def gen_forward(m, name, B, H, W, seed):
    x = seeded_images(B, H, W, seed)
    with torch.no_grad():
        out = m(x)
        taps = _taps(m, x)
    np.savez_compressed(HERE / f"{name}.npz", x=x.numpy(), pred_masks=out["pred_masks"].numpy(),
                        pred_iou=out["pred_iou"].numpy(),
                        features_sub=out["features"][:, :, ::4, ::4].numpy(),
                        **{f"tap{i}_sub": t[:, :, ::8].numpy() for i, t in enumerate(taps)})
    print(name, out["pred_masks"].shape, float(out["pred_masks"].abs().mean()))


def gen_fixture(m):
    from PIL import Image
    import s3od.predictor as P
    img = np.array(Image.open(REF / "tests" / "fixture" / "image.jpg").convert("RGB"))
    br = P.BackgroundRemoval.__new__(P.BackgroundRemoval)
    br.image_size, br.device, br.model = 1024, "cpu", m
    br.mean = np.array([0.485, 0.456, 0.406]); br.std = np.array([0.229, 0.224, 0.225])
    x, pad = br._preprocess(img)
    with torch.no_grad():
        out = m(x)
    res = br.remove_background(img)
    lg = out["pred_masks"][0].numpy()
    alpha = np.array(res.rgba_image)[:, :, 3]
    np.savez_compressed(
        HERE / "fixture_1024.npz",
        image_u8_sum=np.int64(img.astype(np.int64).sum()), image_u8_sub=img[::16, ::16],
        x_sub=x[0, :, ::8, ::8].numpy(),
        pred_iou=out["pred_iou"][0].numpy(), best_idx=np.int64(res.all_ious.argmax()),
        mask_pos_bits=np.packbits((lg > 0).reshape(-1)), logits_sub=lg[:, ::8, ::8],
        frac_small=np.float64((np.abs(lg) < 0.05).mean()),
        all_ious=res.all_ious, predicted_mask_sub=res.predicted_mask[::8, ::8],
        all_masks_sum=res.all_masks.astype(np.float64).sum(axis=(1, 2)),
        alpha_sum=np.int64(alpha.astype(np.int64).sum()), alpha_sub=alpha[::8, ::8])
    print("fixture best", res.all_ious, res.all_ious.argmax())


def gen_train_step(m, seed=3, rescale=1.37):
    """One train-mode step at 256² bs=2: BN batch stats, pinned RoPE rescale, focal_iou."""
    import transformers.models.dinov3_vit.modeling_dinov3_vit as D
    from synth_sod.model_training.loss import LossModule
    orig = D.augment_patches_center_coordinates
    D.augment_patches_center_coordinates = lambda coords, shift=None, jitter=None, rescale_=None, **k: coords * rescale
    try:
        crit = [
            {"name": "focal_loss", "target_key": "masks", "output_key": "pred_masks", "weight": 20,
             "loss": {"_target_": "synth_sod.model_training.loss.FocalLoss", "reduction": "none"}},
            {"name": "iou_loss", "target_key": "masks", "output_key": "pred_masks", "weight": 1.0,
             "loss": {"_target_": "synth_sod.model_training.loss.IoULoss", "smooth": 1e-6, "reduction": "none"}},
            {"name": "mse_ious_loss", "target_key": "gt_ious", "output_key": "pred_iou", "weight": 0.05,
             "loss": {"_target_": "torch.nn.MSELoss"}},
        ]
        lm = LossModule(crit, full_mask_lambda=0.1, decay_rate=0.2)
        m.train()
        x = seeded_images(2, 256, 256, seed)
        masks = ellipse_masks(2, 256, 256, seed + 1)
        m.zero_grad()
        out = m(x)
        loss, parts = lm(out, {"images": x, "masks": masks}, 1)
        loss.backward()
        names, norms, slices = [], [], []
        for n, p in m.named_parameters():
            if p.grad is None:
                continue
            names.append(n)
            norms.append(float(p.grad.norm()))
            sl = np.full(32, np.nan, np.float32)
            g = p.grad.reshape(-1)[:32].numpy()
            sl[:g.size] = g
            slices.append(sl)
        bn = {n: b.numpy().copy() for n, b in m.named_buffers() if "running" in n}
        np.savez_compressed(
            HERE / "train_256_b2.npz", x=x.numpy(), masks=masks.numpy(), rescale=np.float64(rescale), epoch=np.int64(1),
            loss=np.float64(loss.item()), parts_names=np.array(sorted(parts)),
            parts_values=np.array([float(parts[k]) for k in sorted(parts)]),
            pred_masks=out["pred_masks"].detach().numpy(), pred_iou=out["pred_iou"].detach().numpy(),
            grad_names=np.array(names), grad_norms=np.array(norms), grad_slices=np.stack(slices),
            bn_names=np.array(sorted(bn)), bn_values=np.stack([bn[k] for k in sorted(bn)]))
        print("train loss", loss.item(), {k: float(v) for k, v in parts.items()})
        m.eval()
    finally:
        D.augment_patches_center_coordinates = orig


def gen_losses(seed=5):
    from synth_sod.model_training.loss import LossModule
    import yaml
    out = {}
    g = torch.Generator().manual_seed(seed)
    B, M, H, W = 2, 3, 64, 64
    logits = (torch.randn(B, M, H, W, generator=g) * 3.0)
    piou = torch.randn(B, M, generator=g)
    masks = ellipse_masks(B, H, W, seed)
    out.update(logits=logits.numpy(), pred_iou=piou.numpy(), masks=masks.numpy())
    cfgdir = REF / "synth_sod/src/synth_sod/model_training/config/loss"
    for cfgname in ("focal_iou", "bce_iou_ssim"):
        cfg = yaml.safe_load(open(cfgdir / f"{cfgname}.yaml"))
        lm = LossModule(cfg["criterions"], cfg["full_mask_lambda"], cfg["decay_rate"])
        for epoch in (0, 3):
            lg = logits.clone().requires_grad_(True)
            pi = piou.clone().requires_grad_(True)
            loss, parts = lm({"pred_masks": lg, "pred_iou": pi}, {"masks": masks}, epoch)
            loss.backward()
            tag = f"{cfgname}_e{epoch}"
            out[f"{tag}_loss"] = np.float64(loss.item())
            out[f"{tag}_parts_names"] = np.array(sorted(parts))
            out[f"{tag}_parts_values"] = np.array([float(parts[k]) for k in sorted(parts)])
            out[f"{tag}_grad_logits"] = lg.grad.numpy()
            out[f"{tag}_grad_iou"] = pi.grad.numpy()
    np.savez_compressed(HERE / "loss_goldens.npz", **out)
    print("losses done")


def build_reference_dinol(seed=0):
    """The reference's DPTSegmentation with encoder_name="dinov3_large" (taps [4,11,17,23]) and
    num_outputs=1 (config/model/dinol.yaml).  The reference ships only the ViT-B config file
    (src/s3od/dinov3_config/config.json), so AutoConfig is substituted by that same config with
    transformers' DINOv3 ViT-L/16 geometry (hidden 1024, 24 layers, 16 heads, intermediate 4096);
    everything else (RoPE, LayerScale, key_bias=False, registers, the DPT head) is the reference code."""
    import json
    import s3od.model as M
    from transformers import DINOv3ViTConfig
    base = json.load(open(REF / "src" / "s3od" / "dinov3_config" / "config.json"))
    base = {k: v for k, v in base.items() if k not in ("architectures", "model_type", "transformers_version", "torch_dtype")}
    base.update(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16, intermediate_size=4096)
    cfg = DINOv3ViTConfig(**base)
    M.AutoImageProcessor = types.SimpleNamespace(from_pretrained=lambda *a, **k: None)
    M.AutoConfig = types.SimpleNamespace(from_pretrained=lambda *a, **k: cfg)
    m = M.DPTSegmentation(num_classes=1, num_outputs=1, encoder_name="dinov3_large")
    sd = {k: torch.from_numpy(v) for k, v in synthetic_state_dict(seed, "dinol", 1).items()}
    m.load_state_dict(sd, strict=True)
    return m


def gen_dinol(seed=7, rescale=0.83):
    """dinol goldens: eval forward at 128x160 bs=1 and one train step at 128^2 bs=2 with the
    single-mask loss (loss.py:166-188, focal_iou criterions) -> tests/golden/dinol.npz."""
    import transformers.models.dinov3_vit.modeling_dinov3_vit as D
    from synth_sod.model_training.loss import LossModule
    m = build_reference_dinol(0).eval()
    out = {}
    x = seeded_images(1, 128, 160, seed)
    with torch.no_grad():
        o = m(x)
    out.update(fwd_x=x.numpy(), fwd_pred_masks=o["pred_masks"].numpy(), fwd_pred_iou=o["pred_iou"].numpy(),
               fwd_features_sub=o["features"][:, :, ::4, ::4].numpy())
    orig = D.augment_patches_center_coordinates
    D.augment_patches_center_coordinates = lambda coords, shift=None, jitter=None, rescale_=None, **k: coords * rescale
    try:
        crit = [
            {"name": "focal_loss", "target_key": "masks", "output_key": "pred_masks", "weight": 20,
             "loss": {"_target_": "synth_sod.model_training.loss.FocalLoss", "reduction": "none"}},
            {"name": "iou_loss", "target_key": "masks", "output_key": "pred_masks", "weight": 1.0,
             "loss": {"_target_": "synth_sod.model_training.loss.IoULoss", "smooth": 1e-6, "reduction": "none"}},
            {"name": "mse_ious_loss", "target_key": "gt_ious", "output_key": "pred_iou", "weight": 0.05,
             "loss": {"_target_": "torch.nn.MSELoss"}},
        ]
        lm = LossModule(crit, full_mask_lambda=0.1, decay_rate=0.2)
        m.train()
        x = seeded_images(2, 128, 128, seed + 1)
        masks = ellipse_masks(2, 128, 128, seed + 2)
        m.zero_grad()
        o = m(x)
        loss, parts = lm(o, {"images": x, "masks": masks}, 1)
        loss.backward()
        names, norms, slices, nograd = [], [], [], []
        for n, p in m.named_parameters():
            if p.grad is None:
                nograd.append(n)
                continue
            names.append(n)
            norms.append(float(p.grad.norm()))
            sl = np.full(32, np.nan, np.float32)
            g = p.grad.reshape(-1)[:32].numpy()
            sl[:g.size] = g
            slices.append(sl)
        bn = {n: b.numpy().copy() for n, b in m.named_buffers() if "running" in n}
        out.update(train_x=x.numpy(), train_masks=masks.numpy(), rescale=np.float64(rescale), epoch=np.int64(1),
                   loss=np.float64(loss.item()), parts_names=np.array(sorted(parts)),
                   parts_values=np.array([float(parts[k]) for k in sorted(parts)]),
                   train_pred_masks=o["pred_masks"].detach().numpy(),
                   grad_names=np.array(names), grad_norms=np.array(norms), grad_slices=np.stack(slices),
                   nograd_names=np.array(nograd),
                   bn_names=np.array(sorted(bn)), bn_values=np.stack([bn[k] for k in sorted(bn)]))
        print("dinol train loss", loss.item(), {k: float(v) for k, v in parts.items()}, "no-grad params", len(nograd))
    finally:
        D.augment_patches_center_coordinates = orig
    np.savez_compressed(HERE / "dinol.npz", **out)


def metric_cases(seed=11):
    """(name, pred float32 [H,W] in [0,1], gt float64 {0,1}) pairs covering the metric edge cases."""
    r = np.random.default_rng(seed)

    def ell(H, W, cy, cx, ry, rx):
        yy, xx = np.mgrid[:H, :W]
        return ((yy - cy) ** 2 / ry ** 2 + (xx - cx) ** 2 / rx ** 2) < 1

    def smooth(H, W):
        from scipy.ndimage import gaussian_filter
        f = gaussian_filter(r.standard_normal((H, W)), 4)
        return (1 / (1 + np.exp(-6 * f / f.std()))).astype(np.float32)

    cases = []
    g = ell(48, 64, 20, 30, 12, 18)
    cases.append(("random_48x64", r.random((48, 64)).astype(np.float32), g))
    g = ell(97, 131, 50, 60, 30, 45) & ~ell(97, 131, 50, 60, 8, 10)
    p = np.clip(0.7 * g + 0.3 * smooth(97, 131), 0, 1).astype(np.float32)
    cases.append(("holes_97x131", p, g))
    cases.append(("empty_gt_160x120", r.random((160, 120)).astype(np.float32), np.zeros((160, 120), bool)))
    cases.append(("full_gt_64x64", r.random((64, 64)).astype(np.float32), np.ones((64, 64), bool)))
    g = np.zeros((80, 100), bool); g[37, 61] = True
    cases.append(("single_px_80x100", smooth(80, 100), g))
    thr = torch.linspace(0, 1 - 1e-10, 255).numpy()
    p = thr[r.integers(0, 255, (120, 90))].astype(np.float32)
    p[:5] = 0.0; p[-5:] = 1.0
    cases.append(("on_thresholds_120x90", p, ell(120, 90, 60, 45, 40, 30)))
    g = ell(256, 256, 120, 140, 70, 50) | ell(256, 256, 200, 60, 20, 30)
    p = np.clip(g * 0.85 + 0.15 * smooth(256, 256) + 0.05 * r.standard_normal((256, 256)), 0, 1).astype(np.float32)
    cases.append(("two_blobs_256", p, g))
    g = np.zeros((33, 47), bool); g[5:20, 0] = True
    cases.append(("left_column_33x47", smooth(33, 47), g))
    p = np.zeros((40, 52), np.float32); p[10:30, 12:40] = 1.0
    cases.append(("binary_pred_40x52", p, ell(40, 52, 20, 26, 11, 15)))
    return [(n, p.astype(np.float32), g.astype(np.float64)) for n, p, g in cases]


def gen_metrics():
    """tests/golden/metrics.npz: the reference's EvaluationMetrics (metrics.py:213-424) on CPU
    (device=None) for every metric_cases() pair, per-image values + the aggregate dict."""
    from synth_sod.model_training.metrics import EvaluationMetrics
    out = {}
    names = []
    full = EvaluationMetrics(device=None)
    for name, p, g in metric_cases():
        em = EvaluationMetrics(device=None)
        em.step(torch.from_numpy(p.copy()), torch.from_numpy(g.copy()))
        full.step(torch.from_numpy(p.copy()), torch.from_numpy(g.copy()))
        sm = EvaluationMetrics(device=None, sm_only=True)
        sm.step(torch.from_numpy(p.copy()), torch.from_numpy(g.copy()))
        vals = [em.metrics["mae"][0], em.metrics["max_f"][0], em.metrics["avg_f"][0], em.metrics["s_score"][0],
                float(np.mean(em.emeasure.metrics["changeable_ems"][0])), float(em.weighted_fmeasure.metrics["weighted_fms"][0])]
        out[f"{name}/pred"] = p
        out[f"{name}/gt"] = g
        out[f"{name}/values"] = np.array(vals, np.float64)
        out[f"{name}/sm_only"] = np.array([sm.metrics["s_score"][0]], np.float64)
        names.append(name)
    agg = full.compute_metrics()
    out["aggregate_keys"] = np.array(list(agg.keys()))
    out["aggregate"] = np.array([float(v) for v in agg.values()], np.float64)
    out["names"] = np.array(names)
    np.savez_compressed(HERE / "metrics.npz", **out)
    for n in names:
        print(n, out[f"{n}/values"])


def main():
    _install_shims()
    if "--metrics" in sys.argv:
        gen_metrics()
        return
    if "--dinol" in sys.argv:
        torch.set_num_threads(os.cpu_count())
        gen_dinol()
        return
    torch.manual_seed(0)
    torch.set_num_threads(os.cpu_count())
    m = build_reference_model(0).eval()
    if "--train-only" not in sys.argv:
        gen_losses()
        gen_forward(m, "fwd_eval_224x224_b2", 2, 224, 224, seed=1)
        gen_forward(m, "fwd_eval_160x256_b1", 1, 160, 256, seed=2)
        gen_fixture(m)
    gen_train_step(m)


if __name__ == "__main__":
    main()
