"""GPU resume: a run saved with save_checkpoint and restored with load_checkpoint continues
bit-identically (same weights, same FusedAdamW moments and step -> same update)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_resume_is_bit_exact(tmp_path):
    from s3od_amd.checkpoint import save_checkpoint, load_checkpoint
    from s3od_amd.loss import LossModule, FOCAL_IOU
    from s3od_amd.model import DPTSegmentation
    from s3od_amd.optim import FusedAdamW, reference_param_groups
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    m = DPTSegmentation(compute_dtype="bf16").to(dev).train()
    opt = FusedAdamW(reference_param_groups(m, 1e-4), weight_decay=0.05)
    crit = LossModule(FOCAL_IOU, full_mask_lambda=0.1, decay_rate=0.2)
    x = torch.randn(1, 3, 128, 128, device=dev)
    masks = (torch.rand(1, 128, 128, device=dev) > 0.5).float()

    def train_step(model):
        out = model(x)
        loss, _ = crit(out, {"images": x, "masks": masks}, 0)
        loss.backward()

    train_step(m)
    opt.step()
    m.zero_grad(set_to_none=False)
    save_checkpoint(tmp_path / "r.ckpt", m, opt, epoch=1)

    m2 = DPTSegmentation(compute_dtype="bf16").to(dev).train()
    opt2 = FusedAdamW(reference_param_groups(m2, 1e-4), weight_decay=0.05)
    load_checkpoint(tmp_path / "r.ckpt", m2, opt2)
    for (k, a), b in zip(m.state_dict().items(), m2.state_dict().values()):
        assert torch.equal(a, b), k

    train_step(m)                      # one more step: identical gradients into both optimizers
    for (n, p), p2 in zip(m.named_parameters(), m2.parameters()):
        p2.grad = None if p.grad is None else p.grad.detach().clone()
    opt.step()
    opt2.step()
    torch.cuda.synchronize()
    for (n, p), p2 in zip(m.named_parameters(), m2.parameters()):
        assert torch.equal(p, p2), n
