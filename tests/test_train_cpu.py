"""CPU: host logic of the training launcher (s3od_amd/train.py) and the step metrics.

* ``compose_config`` composes the reference's own Hydra tree (train.yaml defaults + group overrides +
  ``${...}`` / ``${eval:...}`` interpolation + OmegaConf's float rule) -- checked against the values the
  reference's YAML files spell out (read in place when /root/reference exists), and on a self-contained
  tree written here;
* ``TopK`` = ModelCheckpoint(monitor="val_dice_epoch", mode="max", save_top_k=3, save_last=True);
* ``EarlyStop`` = EarlyStopping(monitor, min_delta, patience, mode);
* ``binary_iou`` / ``dice_score`` (lightning_module.py:217-232; torchmetrics BinaryJaccardIndex /
  DiceScore micro, whose parity is unpinned -- torchmetrics is absent) vs a numpy restatement.
"""
from pathlib import Path

import numpy as np
import pytest
import torch

REF_CFG = Path("/root/reference/synth_sod/src/synth_sod/model_training/config")


@pytest.mark.skipif(not REF_CFG.exists(), reason="reference config tree not present")
def test_compose_reference_tree():
    from s3od_amd.train import compose_config
    c = compose_config(REF_CFG, ["backend=8gpu", "dataset=synth", "base_dir=/b", "data_dir=/d"])
    assert c["backend"]["devices"] == 8 and c["backend"]["accumulate_grad_batches"] == 16
    assert c["dataset"]["transform_mode"] == "synthetic" and c["dataset"]["train_batch_size"] == 4
    assert c["dataset"]["datasets"][0] == "/d/data/Train_Dataset/SynthSODDataFiltered"
    assert c["optimizer"]["lr"] == 1e-5 and isinstance(c["optimizer"]["lr"], float)
    assert c["scheduler"]["schedulers"][1]["T_max"] == 170          # ${eval:'${backend.max_epochs} - 30'}
    assert c["scheduler"]["milestones"] == [30]
    assert c["loss"]["criterions"][0]["name"] == "focal_loss" and c["loss"]["full_mask_lambda"] == 0.1
    assert c["model"]["num_outputs"] == 3
    assert c["train_stage"]["save_dir"] == "/b/checkpoints"
    assert c["train_stage"]["early_stopping"]["min_delta"] == 1e-4
    d = compose_config(REF_CFG, ["model=dinol", "loss=bce_iou_ssim", "backend.max_epochs=50"])
    assert d["model"]["num_outputs"] == 1 and "vitl16" in d["model"]["encoder_name"]
    assert d["scheduler"]["schedulers"][1]["T_max"] == 20
    assert [x["name"] for x in d["loss"]["criterions"]][:3] == ["bce_loss", "iou_loss", "ssim_loss"]


def test_compose_selfcontained(tmp_path):
    from s3od_amd.train import compose_config
    (tmp_path / "backend").mkdir()
    (tmp_path / "backend" / "a.yaml").write_text("devices: 2\nmax_epochs: 40\nlr: 3e-4\n")
    (tmp_path / "backend" / "b.yaml").write_text("devices: 4\nmax_epochs: 10\nlr: 1e-3\n")
    (tmp_path / "sched").mkdir()
    (tmp_path / "sched" / "c.yaml").write_text("T_max: ${eval:'${backend.max_epochs} - 30'}\nname: run_${backend.devices}\n")
    (tmp_path / "train.yaml").write_text("defaults:\n  - backend: a\n  - sched: c\nroot: /r\nsave: ${root}/ck\n")
    c = compose_config(tmp_path)
    assert c["backend"] == {"devices": 2, "max_epochs": 40, "lr": 3e-4}
    assert c["sched"] == {"T_max": 10, "name": "run_2"} and c["save"] == "/r/ck"
    c = compose_config(tmp_path, ["backend=b", "backend.devices=8", "root=/x"])
    assert c["backend"]["devices"] == 8 and c["sched"]["T_max"] == -20 and c["save"] == "/x/ck"


def test_topk_checkpoints(tmp_path):
    from s3od_amd.train import TopK
    saved = []
    tk = TopK(tmp_path, monitor="val_dice_epoch", mode="max", k=3)

    def save(p):
        Path(p).write_text("x")
        saved.append(Path(p).name)
    for ep, s in enumerate([0.5, 0.7, 0.6, 0.4, 0.8, 0.65]):
        tk.update(ep, {"val_dice_epoch": s}, save)
    names = sorted(p.name for p in tmp_path.glob("epoch=*.ckpt"))
    assert names == ["epoch=01-val_dice_epoch=0.7000.ckpt", "epoch=04-val_dice_epoch=0.8000.ckpt",
                     "epoch=05-val_dice_epoch=0.6500.ckpt"]
    assert (tmp_path / "last.ckpt").exists()
    assert tk.best_model_path.endswith("epoch=04-val_dice_epoch=0.8000.ckpt")
    assert "epoch=03-val_dice_epoch=0.4000.ckpt" not in saved          # never better than the 3rd best


def test_early_stop():
    from s3od_amd.train import EarlyStop
    es = EarlyStop("val_loss", min_delta=0.1, patience=2, mode="min")
    seq = [1.0, 0.95, 0.94, 0.5, 0.45, 0.41]
    out = [es.should_stop({"val_loss": v}) for v in seq]
    assert out == [False, False, True, False, False, True]


def _np_iou(p, t):
    p = p > 0.5; t = t.astype(bool)
    u = (p | t).sum()
    return (p & t).sum() / u if u else 0.0


def _np_dice(p, t):
    p = (p > 0.5).astype(np.float64); t = t.astype(np.float64)
    return 2 * (p * t).sum() / max(p.sum() + t.sum(), 1e-6)


def test_step_metrics_vs_numpy():
    from s3od_amd.lightning_module import SegmentationLightningModule, binary_iou, dice_score
    g = torch.Generator().manual_seed(0)
    logits = torch.randn(4, 3, 32, 32, generator=g) * 3
    ious = torch.randn(4, 3, generator=g)
    tgt = (torch.rand(4, 32, 32, generator=g) > 0.6).float()
    m = SegmentationLightningModule.calculate_metrics(None, {"pred_masks": logits, "pred_iou": ious}, tgt)
    best = torch.sigmoid(logits)[torch.arange(4), ious.argmax(1)].numpy()
    assert float(m["iou"]) == pytest.approx(_np_iou(best, tgt.numpy() > 0.5), rel=1e-6)
    assert float(m["dice"]) == pytest.approx(_np_dice(best, tgt.numpy() > 0.5), rel=1e-6)
    # single-mask (dinol) branch: the one mask is the prediction
    m1 = SegmentationLightningModule.calculate_metrics(None, {"pred_masks": logits[:, :1], "pred_iou": ious[:, :1]}, tgt)
    assert float(m1["iou"]) == pytest.approx(_np_iou(torch.sigmoid(logits[:, 0]).numpy(), tgt.numpy()), rel=1e-6)
    # empty prediction and empty target: torchmetrics' zero_division default (0)
    z = torch.zeros(2, 8, 8)
    assert float(binary_iou(z, z)) == 0.0
    assert float(dice_score(z, z)) == 0.0
