"""GPU parity of the dinol variant (config/model/dinol.yaml: ViT-L/16 encoder, taps [4,11,17,23],
num_outputs=1) and the single-mask loss branch (loss.py:166-188) against tests/golden/dinol.npz,
which make_golden.py --dinol produced by running the reference itself.

strict (f32 MFMA): logits / iou / features max-rel <= 2e-4; train step loss and parts <= 1e-4,
grad norms <= 2e-3, grad slices <= 3e-2 RMS, BN running stats <= 1e-4, and the parameters the
reference leaves without gradient (layer 23, final norm, mask_token, refinenet4.resConfUnit1, the
classifier head -- pred_iou is unused by the single-mask loss) have grad None.
bf16: logits rel-L2 <= 3e-2; train loss <= 2e-2; per-parameter cosine vs strict >= 0.99.
"""
import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

DINOL = dict(num_classes=1, num_outputs=1, encoder_name="facebook/dinov3-vitl16-pretrain-lvd1689m")


def rel_max(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-12))


def rel_l2(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-12))


def is_bn_fed_bias(n):
    return "resConfUnit" in n and (n.endswith("conv1.bias") or n.endswith("conv2.bias"))


@pytest.fixture(scope="module")
def golden():
    return np.load(GOLDEN / "dinol.npz")


def test_hydra_target_builds_dinol():
    from s3od_amd.lightning_module import instantiate
    m = instantiate({"_target_": "synth_sod.model_training.model.DPTSegmentation", **DINOL})
    assert m.variant == "dinol" and m.num_outputs == 1
    sd = m.state_dict()
    assert sd["encoder.embeddings.patch_embeddings.weight"].shape == (1024, 3, 16, 16)
    assert sd["seg_head.classifier_head.4.weight"].shape == (1, 64)
    assert "encoder.model.layer.23.mlp.up_proj.weight" in sd and sd["encoder.model.layer.23.mlp.up_proj.weight"].shape == (4096, 1024)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_dinol_forward(golden, dtype):
    from s3od_amd.model import DPTSegmentation
    m = DPTSegmentation(compute_dtype=dtype, **DINOL).cuda().eval()
    with torch.no_grad():
        out = m(torch.from_numpy(golden["fwd_x"]).cuda())
    torch.cuda.synchronize()
    pm = out["pred_masks"].cpu().numpy()
    assert pm.shape == golden["fwd_pred_masks"].shape == (1, 1, 128, 160)
    if dtype == "f32":
        assert rel_max(pm, golden["fwd_pred_masks"]) < 2e-4
        assert rel_max(out["pred_iou"].cpu().numpy(), golden["fwd_pred_iou"]) < 2e-4
        assert rel_max(out["features"].float().cpu().numpy()[:, :, ::4, ::4], golden["fwd_features_sub"]) < 2e-4
    else:
        e = rel_l2(pm, golden["fwd_pred_masks"])
        print(f"dinol bf16 forward rel-L2 {e:.4g}")
        assert e < 3e-2


def _train(golden, dtype):
    from s3od_amd.model import DPTSegmentation
    from s3od_amd.loss import LossModule, FOCAL_IOU
    m = DPTSegmentation(compute_dtype=dtype, **DINOL).cuda().train()
    m._rope_rescale = float(golden["rescale"])
    lm = LossModule(FOCAL_IOU, full_mask_lambda=0.1, decay_rate=0.2)
    x = torch.from_numpy(golden["train_x"]).cuda()
    out = m(x)
    loss, parts = lm(out, {"images": x, "masks": torch.from_numpy(golden["train_masks"]).cuda()}, int(golden["epoch"]))
    loss.backward()
    torch.cuda.synchronize()
    return m, out, loss, parts


def test_dinol_train_step_strict(golden):
    m, out, loss, parts = _train(golden, "f32")
    assert abs(loss.item() - float(golden["loss"])) <= 1e-4 * abs(float(golden["loss"]))
    assert set(parts) == set(golden["parts_names"])          # {focal_loss, iou_loss}: no aux MSE, no _best/_full
    for n, v in zip(golden["parts_names"], golden["parts_values"]):
        assert abs(float(parts[n]) - v) <= 1e-4 * max(abs(v), 1e-6), n
    assert rel_max(out["pred_masks"].detach().cpu().numpy(), golden["train_pred_masks"]) <= 2e-4
    params = dict(m.named_parameters())
    for n, nrm, sl in zip(golden["grad_names"], golden["grad_norms"], golden["grad_slices"]):
        gr = params[n].grad
        assert gr is not None, n
        if is_bn_fed_bias(n):
            continue
        gr = gr.cpu()
        assert abs(float(gr.norm()) - nrm) <= 2e-3 * max(nrm, 1e-8) + 1e-9, (n, float(gr.norm()), nrm)
        rms = nrm / np.sqrt(gr.numel())
        k = np.isfinite(sl)
        a = np.pad(gr.reshape(-1)[:32].numpy(), (0, 32 - min(32, gr.numel())))[k]
        assert np.abs(a - sl[k]).max() <= 3e-2 * rms + 1e-12, n
    for n in golden["nograd_names"]:
        assert params[n].grad is None, n
    bufs = dict(m.named_buffers())
    for n, v in zip(golden["bn_names"], golden["bn_values"]):
        assert np.abs(bufs[n].cpu().numpy() - v).max() <= 1e-4 * max(np.abs(v).max(), 1e-6), n


def test_dinol_train_step_bf16(golden):
    m, out, loss, parts = _train(golden, "bf16")
    assert abs(loss.item() - float(golden["loss"])) <= 2e-2 * abs(float(golden["loss"]))
    bf = {n: p.grad.detach().double().reshape(-1) for n, p in m.named_parameters() if p.grad is not None}
    m2, *_ = _train(golden, "f32")
    cos = []
    for n, p in m2.named_parameters():
        if p.grad is None or is_bn_fed_bias(n):
            continue
        a, b = bf[n], p.grad.detach().double().reshape(-1)
        cos.append((float(a @ b / (a.norm() * b.norm()).clamp_min(1e-30)), n))
    cos.sort()
    print("dinol bf16 worst grad cosines:", cos[:4])
    assert cos[0][0] >= 0.99, cos[:4]
