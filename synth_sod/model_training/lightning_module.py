"""Alias of synth_sod/.../model_training/lightning_module.py."""
from s3od_amd.lightning_module import SegmentationLightningModule  # noqa: F401
