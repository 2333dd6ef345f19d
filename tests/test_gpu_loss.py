"""GPU parity of the fused multi-mask loss (LossModule -> s3od_mask_loss_fwd/bwd) against the
reference-generated goldens (tests/golden/loss_goldens.npz: focal_iou and bce_iou_ssim, epochs 0
and 3, from synth_sod/.../loss.py:34-275) and, at a ragged size the goldens do not cover, against
the oracle restatement (oracle/s3od_oracle.py:multi_mask_loss).

Tolerances (fp32 kernels, different summation order than the reference's conv2d / reductions):
loss and parts <= 1e-4 relative; logit / pred_iou gradients <= 2e-4 max-relative.
"""
import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-12))


def cfg_of(name):
    from s3od_amd.loss import FOCAL_IOU, BCE_IOU_SSIM
    return FOCAL_IOU if name == "focal_iou" else BCE_IOU_SSIM


def run(cfgname, logits, pred_iou, masks, epoch):
    from s3od_amd.loss import LossModule
    lm = LossModule(cfg_of(cfgname), full_mask_lambda=0.1, decay_rate=0.2)
    lg = logits.cuda().requires_grad_(True)
    pi = pred_iou.cuda().requires_grad_(True)
    loss, parts = lm({"pred_masks": lg, "pred_iou": pi}, {"masks": masks.cuda()}, epoch)
    loss.backward()
    torch.cuda.synchronize()
    return loss, parts, lg.grad.cpu().numpy(), pi.grad.cpu().numpy()


@pytest.mark.parametrize("cfgname", ["focal_iou", "bce_iou_ssim"])
@pytest.mark.parametrize("epoch", [0, 3])
def test_loss_golden(cfgname, epoch):
    g = np.load(GOLDEN / "loss_goldens.npz")
    loss, parts, dl, di = run(cfgname, torch.from_numpy(g["logits"]), torch.from_numpy(g["pred_iou"]),
                              torch.from_numpy(g["masks"]), epoch)
    tag = f"{cfgname}_e{epoch}"
    ref = float(g[f"{tag}_loss"])
    assert abs(loss.item() - ref) <= 1e-4 * abs(ref)
    for n, v in zip(list(g[f"{tag}_parts_names"]), g[f"{tag}_parts_values"]):
        assert abs(float(parts[n]) - v) <= 1e-4 * max(abs(v), 1e-6), (n, float(parts[n]), v)
    assert rel(dl, g[f"{tag}_grad_logits"]) < 2e-4
    assert rel(di, g[f"{tag}_grad_iou"]) < 2e-4


@pytest.mark.parametrize("shape", [(1, 3, 50, 70), (2, 3, 33, 97)])
def test_ssim_ragged_vs_oracle(shape):
    """SSIM tiles (32x32 + halo) at sizes that are not tile multiples, non-square."""
    from oracle import s3od_oracle as O
    torch.manual_seed(0)
    B, M, H, W = shape
    logits = torch.randn(B, M, H, W) * 2
    pred_iou = torch.randn(B, M)
    yy, xx = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    masks = torch.stack([(((yy - H / 2) / (H / 3)) ** 2 + ((xx - W / 2 - b) / (W / 4)) ** 2 <= 1).float() for b in range(B)])
    loss, parts, dl, di = run("bce_iou_ssim", logits, pred_iou, masks, 1)
    lg = logits.clone().requires_grad_(True)
    pi = pred_iou.clone().requires_grad_(True)
    rl, rparts, _, _ = O.multi_mask_loss({"pred_masks": lg, "pred_iou": pi}, masks, 1, O.BCE_IOU_SSIM)
    rl.backward()
    assert abs(loss.item() - rl.item()) <= 1e-4 * abs(rl.item())
    for n in ("ssim_loss_best", "ssim_loss_full", "bce_loss_full", "iou_loss_best"):
        assert abs(float(parts[n]) - float(rparts[n])) <= 1e-4 * max(abs(float(rparts[n])), 1e-6), n
    assert rel(dl, lg.grad.numpy()) < 2e-4
    assert rel(di, pi.grad.numpy()) < 2e-4
