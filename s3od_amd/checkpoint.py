"""Checkpoint interoperability (reference: scripts/export_model.py:27-119,
synth_sod/.../predictor.py:358-372, Lightning's .ckpt layout used by train.py).

* ``save_checkpoint`` writes the Lightning layout the reference's tools read:
  ``{"epoch", "global_step", "state_dict": {"model.<key>": tensor}, "optimizer_states": [...],
  "lr_schedulers": [...], "hyper_parameters": {"config": ...}}``.
* ``load_checkpoint`` restores a model (any of the accepted key layouts: bare, ``model.``-prefixed,
  transformers-4 ``encoder.layer.N``), and optionally the optimizer / LR-scheduler state, so a
  run resumes bit-for-bit (the FusedAdamW state is ``torch.optim.AdamW``-compatible: ``step`` is
  a float tensor, ``exp_avg`` / ``exp_avg_sq`` per parameter).
* ``export_checkpoint`` = ``scripts/export_model.py:export_checkpoint``: strips the Lightning
  metadata to the ``{"state_dict": ...}`` file ``BackgroundRemoval`` loads.

Loading uses ``torch.load(weights_only=True)``: a checkpoint whose ``hyper_parameters.config`` is
an arbitrary Python object (e.g. an OmegaConf tree) must be re-saved with a plain-dict config.
"""
from __future__ import annotations

from pathlib import Path

import torch


def _model_of(module):
    return getattr(module, "model", module)


def _cpu(obj):
    if torch.is_tensor(obj):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_cpu(v) for v in obj)
    return obj


def save_checkpoint(path, module, optimizer=None, scheduler=None, epoch: int = 0, global_step: int = 0, config=None):
    """Lightning-layout checkpoint of a SegmentationLightningModule (or a bare DPTSegmentation)."""
    model = _model_of(module)
    sd = {f"model.{k}": v.detach().cpu() for k, v in model.state_dict().items()}
    cfg = config if config is not None else getattr(module, "config", None)
    ckpt = {
        "epoch": int(epoch),
        "global_step": int(global_step),
        "pytorch-lightning_version": "s3od_amd",
        "state_dict": sd,
        "optimizer_states": [_cpu(optimizer.state_dict())] if optimizer is not None else [],
        "lr_schedulers": [_cpu(scheduler.state_dict())] if scheduler is not None else [],
        "hyper_parameters": {"config": cfg} if cfg is not None else {},
    }
    torch.save(ckpt, str(path))
    return ckpt


def read_checkpoint(path, map_location="cpu"):
    return torch.load(str(path), map_location=map_location, weights_only=True)


def model_state_dict(ckpt):
    """The model weights of a Lightning checkpoint (``model.``-prefixed keys) or a clean one."""
    sd = ckpt["state_dict"] if "state_dict" in ckpt else ckpt
    if any(k.startswith("model.") for k in sd):
        sd = {k[len("model."):]: v for k, v in sd.items() if k.startswith("model.")}
    return sd


def load_checkpoint(path, module, optimizer=None, scheduler=None, strict: bool = True):
    """Restore weights (+ optimizer / scheduler state when given).  Returns the checkpoint dict."""
    ckpt = read_checkpoint(path)
    model = _model_of(module)
    model.load_state_dict(model_state_dict(ckpt), strict=strict)
    if optimizer is not None:
        states = ckpt.get("optimizer_states") or []
        if not states:
            raise KeyError(f"{path}: no optimizer state to resume from")
        optimizer.load_state_dict(states[0])
    if scheduler is not None:
        scheds = ckpt.get("lr_schedulers") or []
        if not scheds:
            raise KeyError(f"{path}: no LR-scheduler state to resume from")
        scheduler.load_state_dict(scheds[0])
    if hasattr(module, "current_epoch_"):
        module.current_epoch_ = int(ckpt.get("epoch", 0))
    return ckpt


def export_checkpoint(checkpoint_path, output_path):
    """Lightning .ckpt -> clean ``{"state_dict": ...}`` inference checkpoint."""
    ckpt = read_checkpoint(checkpoint_path)
    clean = {"state_dict": model_state_dict(ckpt)}
    torch.save(clean, str(output_path))
    return Path(output_path)
