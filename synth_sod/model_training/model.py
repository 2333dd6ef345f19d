"""Alias: Hydra config model/dinob.yaml targets synth_sod.model_training.model.DPTSegmentation."""
from s3od_amd.model import DPTSegmentation  # noqa: F401
