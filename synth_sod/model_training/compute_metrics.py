"""Alias of synth_sod/.../model_training/compute_metrics.py's dataset loop (device metrics on MI355X)."""
from s3od_amd.metrics import find_gt_mask_path, process_dataset  # noqa: F401
