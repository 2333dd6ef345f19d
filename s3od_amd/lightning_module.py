"""Training surface (synth_sod/src/synth_sod/model_training/lightning_module.py:147-285).

``SegmentationLightningModule(config)``: builds the model from ``config.model`` (Hydra-style
``_target_`` dict; the reference's ``synth_sod.model_training.model.DPTSegmentation`` resolves
to ``s3od_amd.model.DPTSegmentation``), the fused ``LossModule`` from ``config.loss``, and
exposes ``training_step`` / ``validation_step`` / ``configure_optimizers`` / ``calculate_metrics``
/ ``_step`` with the reference's semantics (10 logged scalars per step, best-IoU-mask Jaccard and
Dice metrics, AdamW wd=0.05 with encoder lr and seg_head lr*10, SequentialLR LinearLR -> Cosine).
pytorch_lightning / hydra / torchmetrics are not installed in this image, so the class is a
plain ``torch.nn.Module`` duck-typed to the LightningModule hooks; when Lightning is importable
it subclasses ``pl.LightningModule`` instead.  ``log(..., sync_dist=True)`` all-reduces over the
data-parallel group (one fused all-reduce per step, see ``flush_logs``).
"""
from __future__ import annotations

import importlib
import math

import torch
import torch.distributed as dist
import torch.nn as nn

from .loss import LossModule
from .optim import FusedAdamW

try:  # pragma: no cover - lightning is not in this image
    import pytorch_lightning as pl
    _Base = pl.LightningModule
except Exception:  # noqa: BLE001
    _Base = nn.Module

_ALIASES = {"synth_sod.model_training.model.DPTSegmentation": "s3od_amd.model.DPTSegmentation",
            "s3od.model.DPTSegmentation": "s3od_amd.model.DPTSegmentation"}


def _get(cfg, key, default=None):
    if cfg is None:
        return default
    if isinstance(cfg, dict):
        return cfg.get(key, default)
    return getattr(cfg, key, default)


def instantiate(cfg, **kw):
    """Minimal hydra.utils.instantiate for the model / scheduler configs."""
    cfg = dict(cfg) if isinstance(cfg, dict) else {k: getattr(cfg, k) for k in dir(cfg) if not k.startswith("__")}
    raw = cfg.pop("_target_")
    target = _ALIASES.get(raw, raw)
    mod, name = target.rsplit(".", 1)
    return getattr(importlib.import_module(mod), name)(**cfg, **kw)


def binary_iou(pred, target, thr=0.5):
    """torchmetrics BinaryJaccardIndex on thresholded probabilities."""
    p = pred > thr
    t = target.bool()
    inter = (p & t).sum().float()
    union = (p | t).sum().float()
    # empty union -> zero_division (0.0, torchmetrics' default; parity unpinned: torchmetrics absent)
    return torch.where(union > 0, inter / union.clamp_min(1), torch.zeros_like(union))


def dice_score(pred, target, thr=0.5):
    p = (pred > thr).float()
    t = target.float()
    return (2 * (p * t).sum() / (p.sum() + t.sum()).clamp_min(1e-6))


class SegmentationLightningModule(_Base):
    def __init__(self, config):
        super().__init__()
        self.config = config
        self.model = instantiate(_get(config, "model"))
        loss_cfg = _get(config, "loss")
        self.loss_module = LossModule(_get(loss_cfg, "criterions"), full_mask_lambda=_get(loss_cfg, "full_mask_lambda", 0.01),
                                      decay_rate=_get(loss_cfg, "decay_rate", 0.2))
        self.current_epoch_ = 0
        self.logged = {}
        self._pending = {}

    # Lightning compatibility ------------------------------------------------------------
    @property
    def current_epoch(self):
        t = getattr(self, "trainer", None)
        return getattr(t, "current_epoch", self.current_epoch_) if t is not None else self.current_epoch_

    def log(self, name, value, on_step=True, on_epoch=True, prog_bar=False, sync_dist=False, **kw):
        v = value.detach() if torch.is_tensor(value) else torch.tensor(float(value))
        self._pending[name] = (v.float().reshape(()), sync_dist)
        if _Base is not nn.Module:   # real Lightning: its logger / ModelCheckpoint(monitor=...) see every key
            super().log(name, value, on_step=on_step, on_epoch=on_epoch, prog_bar=prog_bar, sync_dist=sync_dist, **kw)

    def flush_logs(self):
        """One fused all-reduce (mean) of every sync_dist scalar logged this step."""
        if not self._pending:
            return self.logged
        names = list(self._pending)
        vals = torch.stack([self._pending[n][0].to(next(self.model.parameters()).device) for n in names])
        if dist.is_available() and dist.is_initialized() and any(s for _, s in self._pending.values()):
            dist.all_reduce(vals, op=dist.ReduceOp.SUM)
            vals = vals / dist.get_world_size()
        self.logged = dict(zip(names, vals.tolist()))
        self._pending.clear()
        return self.logged

    # reference hooks --------------------------------------------------------------------
    def configure_optimizers(self):
        lr = float(_get(_get(self.config, "optimizer"), "lr", 1e-5))
        groups = [{"params": list(self.model.encoder.parameters()), "lr": lr},
                  {"params": list(self.model.seg_head.parameters()), "lr": lr * 10}]
        opt = FusedAdamW(groups, weight_decay=0.05, betas=(0.9, 0.999), eps=1e-8)
        sch_cfg = _get(self.config, "scheduler")
        if sch_cfg is None:
            return {"optimizer": opt}
        scheds = _get(sch_cfg, "schedulers")
        if scheds:
            sch = torch.optim.lr_scheduler.SequentialLR(
                opt, schedulers=[instantiate(s, optimizer=opt) for s in scheds], milestones=list(_get(sch_cfg, "milestones")))
        else:
            sch = instantiate(sch_cfg, optimizer=opt)
        return {"optimizer": opt, "lr_scheduler": {"scheduler": sch}}

    def training_step(self, batch, batch_idx):
        return self._step(batch, batch_idx, "train")

    def validation_step(self, batch, batch_idx):
        with torch.no_grad():
            return self._step(batch, batch_idx, "val")

    def calculate_metrics(self, predictions, targets):
        pred_masks = torch.sigmoid(predictions["pred_masks"])
        pred_ious = predictions["pred_iou"].squeeze(-1)
        if pred_masks.size(1) == 1:
            best = pred_masks.squeeze(1)
        else:
            idx = pred_ious.argmax(dim=1)
            best = pred_masks[torch.arange(pred_masks.size(0), device=pred_masks.device), idx]
        tgt = (targets > 0.5).int()
        return {"iou": binary_iou(best, tgt), "dice": dice_score(best, tgt)}

    def _check_grad_sync(self):
        """The native backward writes gradients straight into a flat buffer (no AccumulateGrad
        hooks), so torch/Lightning DDP or FSDP strategies would never all-reduce them and the
        replicas would drift silently.  Multi-GPU training must install ``s3od_amd.ddp.GradSync``
        (``s3od_amd.train`` does); fail loudly otherwise."""
        if (torch.is_grad_enabled() and self.model.training and dist.is_available() and dist.is_initialized()
                and dist.get_world_size() > 1 and self.model.grad_ready_callback is None):
            raise RuntimeError("data-parallel training needs s3od_amd.ddp.GradSync(model) (a torch/Lightning DDP "
                               "strategy cannot see the native gradients); see s3od_amd/train.py")

    def _step(self, batch, batch_idx, split="train"):
        images, targets = batch["images"], batch["masks"]
        self._check_grad_sync()
        predictions = self.model(images)
        loss, parts = self.loss_module(predictions, batch, self.current_epoch)
        for name, value in parts.items():
            self.log(f"{split}_{name}", value, on_step=True, on_epoch=True, sync_dist=True)
        metrics = self.calculate_metrics({k: (v.detach() if torch.is_tensor(v) else v) for k, v in predictions.items()}, targets)
        self.log(f"{split}_loss", loss, on_step=True, on_epoch=True, prog_bar=True, sync_dist=True)
        for k, v in metrics.items():
            self.log(f"{split}_{k}", v, on_step=True, on_epoch=True, sync_dist=True)
        return loss
