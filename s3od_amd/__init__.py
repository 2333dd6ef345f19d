"""MI355X-native (gfx950) S3OD hot path: DINOv3 ViT-B/16 + DPT decoder + 3-mask head, forward and
backward, multi-mask loss, fused AdamW and RCCL data parallelism, behind the reference's
``BackgroundRemoval`` / ``DPTSegmentation`` / ``LossModule`` / LightningModule surfaces."""
__version__ = "0.1.0"
__all__ = ["BackgroundRemoval", "RemovalResult", "DPTSegmentation", "LossModule"]


def __getattr__(name):   # lazy: importing the package must not require a GPU
    if name in ("BackgroundRemoval", "RemovalResult"):
        from . import predictor
        return getattr(predictor, name)
    if name == "DPTSegmentation":
        from .model import DPTSegmentation
        return DPTSegmentation
    if name == "LossModule":
        from .loss import LossModule
        return LossModule
    raise AttributeError(name)
