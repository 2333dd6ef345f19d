"""GPU: the training launcher (s3od_amd/train.py = synth_sod/model_training/train.py:72-142) end to end
on a tiny images/ + masks/ folder dataset: 2 epochs x 2 micro-batches with accumulate_grad_batches=2
(one optimizer step per epoch), per-epoch scheduler steps, validation epoch means, save_last + top-k
checkpoints named like Lightning's ModelCheckpoint, and a full-state resume that continues the epoch
and step counters."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dataset(root, n=3, S=96):
    from PIL import Image
    (root / "images").mkdir(parents=True)
    (root / "masks").mkdir()
    rng = np.random.default_rng(0)
    for i in range(n):
        h, w = S + 8 * i, S
        Image.fromarray(rng.integers(0, 255, (h, w, 3), dtype=np.uint8)).save(root / "images" / f"im{i}.png")
        m = np.zeros((h, w), np.uint8)
        m[h // 4: 3 * h // 4, w // 3: 2 * w // 3] = 255
        Image.fromarray(m).save(root / "masks" / f"im{i}.png")


def _config(tmp_path, data, max_epochs, ckpt=None, evaluate=False):
    from s3od_amd.loss import FOCAL_IOU
    return {
        "backend": {"seed": 42, "devices": 1, "max_epochs": max_epochs, "accumulate_grad_batches": 2},
        "dataset": {"datasets": [str(data)], "train_batch_size": 1, "val_batch_size": 2, "num_workers": 0,
                    "image_size": 96, "val_split": 0.34, "transform_mode": "regular"},
        "loss": {"criterions": FOCAL_IOU, "full_mask_lambda": 0.1, "decay_rate": 0.2},
        "model": {"_target_": "synth_sod.model_training.model.DPTSegmentation", "num_classes": 1, "num_outputs": 3,
                  "encoder_name": "facebook/dinov3-vitb16-pretrain-lvd1689m"},
        "optimizer": {"_target_": "torch.optim.AdamW", "lr": 1e-5},
        "scheduler": {"schedulers": [
            {"_target_": "torch.optim.lr_scheduler.LinearLR", "start_factor": 1.0, "end_factor": 1.0, "total_iters": 1},
            {"_target_": "torch.optim.lr_scheduler.CosineAnnealingLR", "T_max": 4, "eta_min": 1e-6}], "milestones": [1]},
        "train_stage": {"save_dir": str(tmp_path / "ckpt"), "experiment_name": "t", "checkpoint_path": ckpt,
                        "weights_only": False,
                        "evaluation": {"input_dir": str(data.parent), "enabled": evaluate, "image_size": 96,
                                       "datasets": [data.name]},
                        "early_stopping": {"monitor": "val_iou_loss_full_epoch", "min_delta": 1e-4, "patience": 50,
                                           "mode": "min"}},
    }


def test_fit_two_epochs_accumulate_and_resume(tmp_path):
    from s3od_amd.train import fit
    data = tmp_path / "data"
    _dataset(data)
    out = fit(_config(tmp_path, data, 2, evaluate=True), log=lambda s: print(s))
    # EvaluationCallback.on_fit_end (train.py:30-55): the best checkpoint scored with the device metrics
    ev = out["evaluation"][data.name]
    assert set(ev) == {"MAE", "MaxF", "AvgF", "Sm", "Em", "wF"} and all(np.isfinite(v) for v in ev.values())
    assert out["epochs"] == 2
    assert out["global_step"] == 2                       # 2 micro-batches / accumulate 2, per epoch
    h = out["history"]
    for k in ("train_loss_epoch", "train_dice_epoch", "val_dice_epoch", "val_loss_epoch", "val_iou_loss_full_epoch"):
        assert k in h[-1] and np.isfinite(h[-1][k]), k
    # LinearLR(1.0 -> 1.0, 1 epoch) then cosine: the lr moved after the second epoch only
    assert h[0]["lr"] == pytest.approx([1e-5, 1e-4])
    assert h[1]["lr"][0] < 1e-5
    from pathlib import Path
    d = Path(out["best_model_path"]).parent            # <save_dir>/<experiment_name>_<timestamp> (train.py:58-69,101)
    assert d.parent == tmp_path / "ckpt" and d.name.startswith("t_") and len(d.name) == len("t_20260101_000000")
    assert (d / "last.ckpt").exists()
    top = sorted(p.name for p in d.glob("epoch=*-val_dice_epoch=*.ckpt"))
    assert len(top) == 2 and out["best_model_path"] is not None
    opt_state = out["optimizer"].state_dict()["state"]
    assert float(next(iter(opt_state.values()))["step"]) == 2.0
    # full-state resume: epoch counter, global step, optimizer step and LR schedule continue
    out2 = fit(_config(tmp_path, data, 3, ckpt=str(d / "last.ckpt")), log=lambda s: print(s))
    assert out2["epochs"] == 1 and out2["history"][0]["epoch"] == 2
    assert out2["global_step"] == 3
    assert float(next(iter(out2["optimizer"].state_dict()["state"].values()))["step"]) == 3.0


def test_fit_stops_on_non_finite_loss(tmp_path, monkeypatch):
    """The launcher's loss guard: a NaN loss raises FloatingPointError at the next check."""
    from s3od_amd.lightning_module import SegmentationLightningModule
    from s3od_amd.train import fit
    data = tmp_path / "data"
    _dataset(data)
    cfg = _config(tmp_path, data, 1)
    cfg["backend"]["nan_check_every"] = 1

    def nan_step(self, batch, i):
        return next(self.model.parameters()).sum() * float("nan")
    monkeypatch.setattr(SegmentationLightningModule, "training_step", nan_step)
    with pytest.raises(FloatingPointError):
        fit(cfg, log=lambda s: None)
