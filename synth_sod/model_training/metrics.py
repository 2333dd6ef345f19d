"""Alias of synth_sod/.../model_training/metrics.py's EvaluationMetrics (HIP kernels on MI355X)."""
from s3od_amd.metrics import EvaluationMetrics  # noqa: F401
