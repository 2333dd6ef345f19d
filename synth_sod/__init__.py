"""Drop-in alias of the reference's training package for the hot path only
(Hydra ``_target_: synth_sod.model_training.model.DPTSegmentation``, ``LossModule``,
``SegmentationLightningModule``)."""
