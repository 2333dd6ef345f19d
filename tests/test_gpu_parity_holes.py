"""GPU parity of the smaller pieces around the model:

* FusedAdamW (csrc/optim.hip) vs torch.optim.AdamW: 3 steps, 2 lr groups (lightning_module.py:183-193),
  parameters and moments within 1e-6 relative;
* the packed-weight cache follows the optimizer: after 2 FusedAdamW steps the model's forward equals a
  fresh model loaded with the same state_dict, and the 2-step loss trajectory matches torch.optim.AdamW;
* train-mode forward under no_grad (Lightning's validation path with model.train()): outputs and BN
  running-stat updates vs the oracle;
* the antialiased post-resize (predictor.py:117-123) vs F.interpolate(antialias=True) at 480x640,
  2000x2000 and 800x400;
* a transformers-4.x (``encoder.layer.N``) checkpoint loads through BackgroundRemoval;
* reference Quirk 2 (predictor.py:83-90: pad 0 but new_w < S feeds the S x new_w image);
* the gradient of the returned ``features`` (path_1) joins the native backward (vs the oracle).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import FIXTURE

pytestmark = pytest.mark.gpu


def test_fused_adamw_matches_torch():
    from s3od_amd.optim import FusedAdamW
    g = torch.Generator(device="cuda").manual_seed(0)
    shapes = [(300, 70), (1000,), (3, 3, 17), (65536 + 123,)]
    ps = [torch.randn(s, device="cuda", generator=g) for s in shapes]
    a = [torch.nn.Parameter(p.clone()) for p in ps]
    b = [torch.nn.Parameter(p.clone()) for p in ps]
    oa = FusedAdamW([{"params": a[:2], "lr": 1e-3}, {"params": a[2:], "lr": 1e-2}], weight_decay=0.05)
    ob = torch.optim.AdamW([{"params": b[:2], "lr": 1e-3}, {"params": b[2:], "lr": 1e-2}], weight_decay=0.05,
                           betas=(0.9, 0.999), eps=1e-8, foreach=False)
    for step in range(3):
        for pa, pb in zip(a, b):
            gr = torch.randn(pa.shape, device="cuda", generator=g) * (10.0 ** (step - 1))
            pa.grad = gr.clone(); pb.grad = gr.clone()
        oa.step(); ob.step()
    torch.cuda.synchronize()
    for pa, pb in zip(a, b):
        assert float((pa - pb).detach().abs().max() / pb.detach().abs().max()) <= 1e-6
        for key in ("exp_avg", "exp_avg_sq"):
            sa, sb = oa.state[pa][key], ob.state[pb][key]
            assert float((sa - sb).abs().max() / sb.abs().max()) <= 1e-6, key
        assert float(oa.state[pa]["step"]) == float(ob.state[pb]["step"]) == 3.0


def _train(m, opt, x, masks, steps):
    from s3od_amd.loss import LossModule, FOCAL_IOU
    lm = LossModule(FOCAL_IOU, full_mask_lambda=0.1, decay_rate=0.2)
    losses = []
    for _ in range(steps):
        out = m(x)
        loss, _ = lm(out, {"images": x, "masks": masks}, 0)
        loss.backward()
        opt.step()
        m.zero_grad(set_to_none=False)
        losses.append(float(loss))
    return losses


def test_weight_cache_follows_optimizer():
    from s3od_amd.model import DPTSegmentation
    from s3od_amd.optim import FusedAdamW, reference_param_groups
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(2, 3, 128, 128, device="cuda", generator=g)
    masks = (torch.rand(2, 128, 128, device="cuda", generator=g) > 0.5).float()
    m = DPTSegmentation(compute_dtype="f32").cuda().train()
    m._rope_rescale = 1.0
    fl = _train(m, FusedAdamW(reference_param_groups(m, 1e-4), weight_decay=0.05), x, masks, 3)
    # a fresh model / engine with the same weights gives the same forward
    fresh = DPTSegmentation(compute_dtype="f32", init_seed=None).cuda()
    fresh.load_state_dict(m.state_dict())
    m.eval(); fresh.eval()
    with torch.no_grad():
        a = m(x)["pred_masks"]; b = fresh(x)["pred_masks"]
    assert float((a - b).abs().max()) <= 1e-6 * float(b.abs().max())
    # ... and the loss trajectory matches torch.optim.AdamW driving the same model
    t = DPTSegmentation(compute_dtype="f32").cuda().train()
    t._rope_rescale = 1.0
    tl = _train(t, torch.optim.AdamW(reference_param_groups(t, 1e-4), weight_decay=0.05, foreach=False), x, masks, 3)
    print("FusedAdamW losses", fl, "torch AdamW losses", tl)
    assert fl[0] == pytest.approx(tl[0], rel=1e-5)
    assert fl[1] != pytest.approx(fl[0], rel=1e-6)          # the weights did move
    for u, v in zip(fl[1:], tl[1:]):
        assert u == pytest.approx(v, rel=1e-4)


def test_train_mode_forward_under_no_grad():
    from oracle import s3od_oracle as O
    from s3od_amd.model import DPTSegmentation
    from s3od_amd.weights import synthetic_state_dict
    g = torch.Generator().manual_seed(4)
    x = torch.randn(2, 3, 128, 160, generator=g)
    m = DPTSegmentation(compute_dtype="f32").cuda().train()
    m._rope_rescale = 1.2
    with torch.no_grad():
        out = m(x.cuda())
    sd = {k: torch.from_numpy(v).clone() for k, v in synthetic_state_dict(0).items()}
    with torch.no_grad():
        ref = O.forward(x, sd, train=True, rope_rescale=1.2)
    pm = out["pred_masks"].cpu()
    assert float((pm - ref["pred_masks"]).abs().max() / ref["pred_masks"].abs().max()) <= 2e-4
    bufs = dict(m.named_buffers())
    n = 0
    for k, v in sd.items():
        if "running_" in k and "refinenet4.resConfUnit1" not in k:
            got = bufs[k].cpu()
            assert float((got - v).abs().max()) <= 1e-4 * max(float(v.abs().max()), 1e-6), k
            n += 1
    assert n == 28


@pytest.mark.parametrize("hw", [(480, 640), (2000, 2000), (800, 400), (20, 30), (31, 31), (40, 4000), (4000, 40), (1, 1)])
def test_postprocess_antialias_resize(hw):
    from s3od_amd._lib import lib, stream
    from oracle.s3od_oracle import get_pad_info
    H0, W0 = hw
    S = 1024
    info = get_pad_info(H0, W0, S)
    g = torch.Generator(device="cuda").manual_seed(H0 + W0)
    logits = torch.randn(1, 3, S, S, device="cuda", generator=g) * 4
    ph, pw = info["height_pad"], info["width_pad"]
    h, w = S - 2 * ph, S - 2 * pw
    tmp = torch.empty(3, h, W0, device="cuda")
    out = torch.empty(3, H0, W0, device="cuda")
    lib()("s3od_sigmoid_unpad_resize", logits, 3, S, S, ph, pw, h, w, H0, W0, tmp, out, stream())
    m = torch.sigmoid(logits.cpu())[0]
    if ph > 0:
        m = m[:, ph:-ph, :]
    if pw > 0:
        m = m[:, :, pw:-pw]
    ref = F.interpolate(m[None], size=(H0, W0), mode="bilinear", align_corners=False, antialias=True)[0]
    err = float((out.cpu() - ref).abs().max())
    print(f"antialias {hw}: max|d| {err:.3g}")
    assert err <= 2e-6


def _fixture_rgb():
    from PIL import Image
    return np.array(Image.open(FIXTURE / "image.jpg").convert("RGB"))


def test_transformers4_checkpoint_loads(tmp_path):
    from s3od_amd.predictor import BackgroundRemoval
    from s3od_amd.weights import synthetic_state_dict, to_transformers4_layout
    sd4 = {k: torch.from_numpy(np.asarray(v)) for k, v in to_transformers4_layout(synthetic_state_dict(0)).items()}
    assert any(k.startswith("encoder.layer.0.") for k in sd4)
    assert not any(k.startswith("encoder.model.") for k in sd4)
    path = tmp_path / "s3od_tf4.pt"
    torch.save({"state_dict": sd4}, path)
    img = _fixture_rgb()
    r4 = BackgroundRemoval(model_id=str(path), compute_dtype="f32").remove_background(img)
    r5 = BackgroundRemoval(model_id="synthetic", compute_dtype="f32").remove_background(img)
    m4 = dict(BackgroundRemoval(model_id=str(path), compute_dtype="f32").model.state_dict())
    m5 = dict(BackgroundRemoval(model_id="synthetic", compute_dtype="f32").model.state_dict())
    assert m4.keys() == m5.keys() and all(torch.equal(m4[k], m5[k]) for k in m4)      # same weights, bit for bit
    # (fp32 atomics in the average pool make repeated forwards differ in the last ulp)
    assert int(np.argmax(r4.all_ious)) == int(np.argmax(r5.all_ious))
    assert np.abs(r4.all_ious - r5.all_ious).max() <= 1e-6
    assert np.abs(r4.all_masks - r5.all_masks).max() <= 1e-5


def test_quirk2_unpadded_input():
    """1024x1023 image at image_size 1024: new = (1024, 1023), pad 0 -> the reference feeds a
    1024x1023 tensor; the model output is 1024x1008 and is resized back to 1024x1023."""
    from oracle import s3od_oracle as O
    from s3od_amd.predictor import BackgroundRemoval
    from s3od_amd.weights import synthetic_state_dict
    img = np.ascontiguousarray(_fixture_rgb()[:, :1023])
    br = BackgroundRemoval(model_id="synthetic", compute_dtype="f32")
    x, info = br._preprocess(img)
    assert tuple(x.shape) == (1, 3, 1024, 1023)
    with torch.no_grad():
        assert tuple(br.model(x)["pred_masks"].shape) == (1, 3, 1024, 1008)
    res = br.remove_background(img)
    sd = {k: torch.from_numpy(v).cuda() for k, v in synthetic_state_dict(0).items()}
    xr = O.normalize(img).cuda()                       # cv2.resize to the same size is the identity
    with torch.no_grad():
        ref = O.forward(xr, sd)
    allm, ious, best = O.postprocess(ref["pred_masks"].cpu(), ref["pred_iou"].cpu(), info)
    assert res.all_masks.shape == (3, 1024, 1023)
    assert int(np.argmax(res.all_ious)) == int(best)
    assert np.abs(res.all_masks - allm).max() <= 1e-4
    assert np.abs(res.all_ious - ious).max() <= 1e-5
    # the non-quirk mode pads to S x S instead
    br.exact_reference_quirks = False
    x2, _ = br._preprocess(img)
    assert tuple(x2.shape) == (1, 3, 1024, 1024)


def test_features_gradient_vs_oracle():
    """``features`` (path_1) carries grad as in the reference: loss = mask loss + <features, R> on the
    f32-strict HIP path vs the oracle's autograd (per-parameter grad norm <= 2e-3, cosine >= 0.999)."""
    from oracle import s3od_oracle as O
    from s3od_amd.loss import LossModule, FOCAL_IOU
    from s3od_amd.model import DPTSegmentation
    from s3od_amd.weights import synthetic_state_dict
    from bench import synthetic_batch
    torch.manual_seed(5)
    x, masks = synthetic_batch(1, 224, 41, torch.device("cuda"))
    m = DPTSegmentation(compute_dtype="f32").cuda().train()
    m._rope_rescale = 1.0
    m.zero_grad(set_to_none=True)
    out = m(x)
    R = torch.randn_like(out["features"]) * 1e-3
    lm = LossModule(FOCAL_IOU, full_mask_lambda=0.1, decay_rate=0.2)
    loss, _ = lm(out, {"images": x, "masks": masks}, 0)
    (loss + (out["features"] * R).sum()).backward()
    torch.cuda.synchronize()
    sd = {}
    for k, v in synthetic_state_dict(0).items():
        t = torch.from_numpy(v).cuda()
        if t.is_floating_point() and "running" not in k:
            t.requires_grad_(True)
        sd[k] = t
    ref = O.forward(x, sd, train=True, rope_rescale=1.0)
    rloss, *_ = O.multi_mask_loss(ref, masks, 0)
    (rloss + (ref["features"] * R).sum()).backward()
    worst_n, worst_c = (0.0, ""), (1.0, "")
    for n, p in m.named_parameters():
        if p.grad is None:
            continue
        if "resConfUnit" in n and (n.endswith("conv1.bias") or n.endswith("conv2.bias")):
            continue     # a bias feeding train-mode BN has an exactly-zero true gradient (noise only)
        g, rg = p.grad.double(), sd[n].grad.double()
        en = abs(float(g.norm()) - float(rg.norm())) / max(float(rg.norm()), 1e-12)
        c = float((g.reshape(-1) @ rg.reshape(-1)) / (g.norm() * rg.norm()).clamp_min(1e-30))
        worst_n = max(worst_n, (en, n)); worst_c = min(worst_c, (c, n))
    assert worst_n[0] <= 2e-3, worst_n
    assert worst_c[0] >= 0.999, worst_c


def test_failed_call_drops_zero_workspaces():
    """a call that fails between an accumulating kernel and its clearing reader (here: the BN finalize of
    the 3rd train-mode BN raises after its conv has added batch sums into the persistent workspace) must not leak
    those partials or the queued num_batches_tracked bumps into later calls.  The engine drops both; the next
    train-mode forward then equals a fresh model's, buffers included."""
    from s3od_amd.model import DPTSegmentation
    g = torch.Generator().manual_seed(8)
    x = torch.randn(2, 3, 128, 128, generator=g).cuda()
    m = DPTSegmentation(compute_dtype="bf16").cuda().train()
    m._rope_rescale = 1.1
    eng = m.engine()
    orig, calls = eng._bn_train, {"n": 0}

    def boom(*a, **k):
        calls["n"] += 1
        if calls["n"] == 3:
            raise RuntimeError("injected failure")
        return orig(*a, **k)
    eng._bn_train = boom
    with pytest.raises(RuntimeError, match="injected"):
        with torch.no_grad():
            m(x)
    eng._bn_train = orig
    assert eng._zpool == {} and eng._nbt == []
    # the failed forward updated the running stats of the first BNs: restore them from a fresh model
    ref = DPTSegmentation(compute_dtype="bf16").cuda().train()
    ref._rope_rescale = 1.1
    m.load_state_dict(ref.state_dict())
    with torch.no_grad():
        a, b = m(x)["pred_masks"], ref(x)["pred_masks"]
    # (equal up to the fp64 BN-sum atomics' summation order)
    assert float((a - b).abs().max() / b.abs().max()) <= 1e-4
    for (k, u), (_, v) in zip(m.named_buffers(), ref.named_buffers()):
        assert torch.allclose(u.float(), v.float(), rtol=1e-5, atol=1e-6), k
