"""Alias of synth_sod/.../model_training/predictor.py's SODPredictor / PredictionResult (MI355X)."""
from s3od_amd.sod_predictor import PredictionResult, SODPredictor  # noqa: F401
