"""Alias of synth_sod/.../model_training/loss.py's LossModule (fused on MI355X)."""
from s3od_amd.loss import LossModule, LossComponent  # noqa: F401
