"""GPU: the LightningModule surface runs the reference's step semantics end to end
(Hydra-style config with the reference's own _target_ strings, loss parts, metrics, the fused
AdamW with two lr groups and the SequentialLR schedule)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

CFG = {
    "model": {"_target_": "synth_sod.model_training.model.DPTSegmentation", "num_classes": 1, "num_outputs": 3,
              "encoder_name": "facebook/dinov3-vitb16-pretrain-lvd1689m"},
    "loss": {"criterions": [
        {"name": "focal_loss", "target_key": "masks", "output_key": "pred_masks", "weight": 20,
         "loss": {"_target_": "synth_sod.model_training.loss.FocalLoss", "reduction": "none"}},
        {"name": "iou_loss", "target_key": "masks", "output_key": "pred_masks", "weight": 1.0,
         "loss": {"_target_": "synth_sod.model_training.loss.IoULoss", "smooth": 1e-6, "reduction": "none"}},
        {"name": "mse_ious_loss", "target_key": "gt_ious", "output_key": "pred_iou", "weight": 0.05,
         "loss": {"_target_": "torch.nn.MSELoss"}}], "full_mask_lambda": 0.1, "decay_rate": 0.2},
    "optimizer": {"_target_": "torch.optim.AdamW", "lr": 1e-5},
    "scheduler": {"schedulers": [
        {"_target_": "torch.optim.lr_scheduler.LinearLR", "start_factor": 1.0, "end_factor": 1.0, "total_iters": 30},
        {"_target_": "torch.optim.lr_scheduler.CosineAnnealingLR", "T_max": 170, "eta_min": 1e-6}], "milestones": [30]},
}


def test_lightning_training_steps():
    from synth_sod.model_training.lightning_module import SegmentationLightningModule
    lm = SegmentationLightningModule(CFG).cuda().train()
    opt_cfg = lm.configure_optimizers()
    opt, sch = opt_cfg["optimizer"], opt_cfg["lr_scheduler"]["scheduler"]
    assert [g["lr"] for g in opt.param_groups] == [1e-5, 1e-4]
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 3, 128, 128, generator=g).cuda()
    masks = (torch.rand(2, 128, 128, generator=g) > 0.5).float().cuda()
    w0 = lm.model.seg_head.projects[0].weight.detach().clone()
    losses = []
    for step in range(3):
        loss = lm.training_step({"images": x, "masks": masks}, step)
        loss.backward()
        opt.step()
        lm.model.zero_grad(set_to_none=False)
        logs = lm.flush_logs()
        losses.append(loss.item())
    sch.step()
    assert all(math.isfinite(v) for v in losses)
    for k in ("train_loss", "train_focal_loss_best", "train_iou_loss_full", "train_mse_ious_loss", "train_iou", "train_dice",
              "train_best_iou", "train_gt_ious"):
        assert k in logs, k
    assert not torch.equal(w0, lm.model.seg_head.projects[0].weight.detach())
    # unused parameters never receive gradients nor updates (reference semantics)
    assert lm.model.encoder.norm.weight.grad is None
