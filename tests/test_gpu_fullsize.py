"""GPU parity at the BASELINE.json configuration sizes, on the HIP path through the C ABI.

  C2  dinob inference bs=8 1024^2:   the bs-8 batch equals eight bs-1 runs (f32 and bf16); one image
                                      in f32-strict mode vs the oracle (max-rel <= 2e-4, argmax exact).
  C3  train bs=16 1024^2:            one f32-strict train step at bs=1 vs the oracle's autograd
                                      (loss <= 1e-4, logits <= 2e-4, per-parameter grad norm <= 2e-3,
                                      per-parameter cosine >= 0.999); then bs=16 bf16 vs bs=16 f32-strict
                                      on the GPU: per-parameter gradient cosine >= 0.99 and norm <= 6e-2.
  C5  2048^2 bs=4:                   bf16 vs f32-strict (rel-L2 <= 3e-2, sign agreement >= 0.98); one
                                      image f32-strict vs the oracle (max-rel <= 2e-4, argmax exact).

The oracle (oracle/s3od_oracle.py, pinned to the reference by tests/test_oracle_golden.py) runs
here as plain fp32 PyTorch on the GPU device so a 1024^2 / 2048^2 check takes seconds; it is the
checker, never the thing measured.  Weights: the deterministic synthetic checkpoint.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel_max(a, b):
    a = a.double(); b = b.double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))


def rel_l2(a, b):
    a = a.double(); b = b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


def cosine(a, b):
    a = a.double().reshape(-1); b = b.double().reshape(-1)
    return float((a @ b) / (a.norm() * b.norm()).clamp_min(1e-30))


def _oracle_sd(requires_grad=False):
    from s3od_amd.weights import synthetic_state_dict
    sd = {}
    for k, v in synthetic_state_dict(0).items():
        t = torch.from_numpy(v).cuda()
        if requires_grad and t.is_floating_point() and "running" not in k:
            t.requires_grad_(True)
        sd[k] = t
    return sd


def _batch(B, S, seed):
    from bench import synthetic_batch
    return synthetic_batch(B, S, seed, torch.device("cuda"))


@pytest.fixture(scope="module")
def model():
    from s3od_amd.model import DPTSegmentation
    return DPTSegmentation(compute_dtype="f32").cuda().eval()


# ------------------------------------------------------------------------------------ C2
@pytest.mark.parametrize("dtype,tol", [("f32", 1e-5), ("bf16", 1e-5)])
def test_c2_batch_equals_single_images(model, dtype, tol):
    x, _ = _batch(8, 1024, 21)
    model.compute_dtype = dtype
    with torch.no_grad():
        out = model(x)
        pm, iou = out["pred_masks"].clone(), out["pred_iou"].clone()
        worst = 0.0
        for i in range(8):
            o1 = model(x[i:i + 1].contiguous())
            worst = max(worst, rel_max(o1["pred_masks"][0], pm[i]), rel_max(o1["pred_iou"][0], iou[i]))
    torch.cuda.synchronize()
    print(f"C2 {dtype}: bs8 vs 8 x bs1 max-rel {worst:.3g}")
    model.compute_dtype = "f32"
    assert worst <= tol
    assert torch.isfinite(pm).all()


def test_c2_one_image_strict_vs_oracle(model):
    from oracle import s3od_oracle as O
    x, _ = _batch(1, 1024, 22)
    model.compute_dtype = "f32"
    with torch.no_grad():
        out = model(x)
        ref = O.forward(x, _oracle_sd())
    e_m = rel_max(out["pred_masks"], ref["pred_masks"])
    e_i = rel_max(out["pred_iou"], ref["pred_iou"])
    e_f = rel_max(out["features"].float(), ref["features"])
    print(f"C2 strict vs oracle @1024: logits {e_m:.3g}, iou {e_i:.3g}, features {e_f:.3g}")
    assert e_m <= 2e-4 and e_i <= 2e-4 and e_f <= 2e-4
    assert int(out["pred_iou"].argmax(1)) == int(ref["pred_iou"].argmax(1))


# ------------------------------------------------------------------------------------ C3
def _train_grads(m, x, masks, rescale=1.3):
    from s3od_amd.loss import LossModule, FOCAL_IOU
    m.train()
    m._rope_rescale = rescale
    m.zero_grad(set_to_none=True)
    lm = LossModule(FOCAL_IOU, full_mask_lambda=0.1, decay_rate=0.2)
    out = m(x)
    loss, _ = lm(out, {"images": x, "masks": masks}, 0)
    loss.backward()
    torch.cuda.synchronize()
    grads = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
    return float(loss), out["pred_masks"].detach(), grads


def test_c3_train_step_strict_vs_oracle_1024():
    from oracle import s3od_oracle as O
    from s3od_amd.model import DPTSegmentation
    x, masks = _batch(1, 1024, 31)
    m = DPTSegmentation(compute_dtype="f32").cuda()
    loss, pm, grads = _train_grads(m, x, masks)
    sd = _oracle_sd(requires_grad=True)
    ref = O.forward(x, sd, train=True, rope_rescale=1.3)
    rloss, *_ = O.multi_mask_loss(ref, masks, 0)
    rloss.backward()
    assert abs(loss - float(rloss)) <= 1e-4 * abs(float(rloss))
    assert rel_max(pm, ref["pred_masks"].detach()) <= 2e-4
    worst_n, worst_c = (0.0, ""), (1.0, "")
    for n, g in grads.items():
        rg = sd[n].grad
        if "resConfUnit" in n and (n.endswith("conv1.bias") or n.endswith("conv2.bias")):
            continue     # a bias feeding train-mode BN has an exactly-zero true gradient (noise only)
        en = abs(float(g.norm()) - float(rg.norm())) / max(float(rg.norm()), 1e-12)
        c = cosine(g, rg)
        worst_n = max(worst_n, (en, n)); worst_c = min(worst_c, (c, n))
    print(f"C3 strict vs oracle @1024 bs1: loss {loss:.6g}/{float(rloss):.6g}, worst grad-norm {worst_n}, worst cos {worst_c}")
    assert worst_n[0] <= 2e-3, worst_n
    assert worst_c[0] >= 0.999, worst_c


def _grad_report(grads, sd):
    worst_n, worst_c = (0.0, ""), (1.0, "")
    for n, g in grads.items():
        if "resConfUnit" in n and (n.endswith("conv1.bias") or n.endswith("conv2.bias")):
            continue     # a bias feeding train-mode BN has an exactly-zero true gradient (noise only)
        rg = sd[n].grad
        en = abs(float(g.norm()) - float(rg.norm())) / max(float(rg.norm()), 1e-12)
        worst_n = max(worst_n, (en, n)); worst_c = min(worst_c, (cosine(g, rg), n))
    return worst_n, worst_c


def test_c3_multi_image_train_step_vs_oracle_1024():
    """A MULTI-image production-size train step (bs 2 at 1024^2: multi-image BN batch statistics, the M = 2 * 4101
    GEMM tails, split-K wgrads over both images) against the ORACLE's autograd (lightning_module.py:242-244; train-mode
    BN src/s3od/model.py:334-345), not against the build's own f32 path: f32 strict at the bs-1 thresholds (loss 1e-4,
    logits 2e-4 max-rel on every image, per-parameter grad norm 2e-3, cosine 0.999, BN running stats 1e-4), then the
    bf16 fast path (loss 2 %, per-parameter cosine >= 0.99).  bs 2, not 4: the fp32 oracle and the f32-strict engine
    (fp32 MFMA, 1/16 of the bf16 rate) take ~1 min per image each, and the GPU box kills a test that is silent for
    3 min; progress is printed per phase (visible with -s)."""
    from oracle import s3od_oracle as O
    from s3od_amd.model import DPTSegmentation
    B = 2
    x, masks = _batch(B, 1024, 33)
    sd = _oracle_sd(requires_grad=True)
    ref = O.forward(x, sd, train=True, rope_rescale=1.3)
    rloss, *_ = O.multi_mask_loss(ref, masks, 0)
    rloss.backward()
    print(f"C3 bs{B}: oracle step done", flush=True)
    rpm = ref["pred_masks"].detach()
    del ref
    torch.cuda.empty_cache()
    res = {}
    for dt in ("f32", "bf16"):
        m = DPTSegmentation(compute_dtype=dt).cuda()
        loss, pm, grads = _train_grads(m, x, masks)
        bufs = {k: v.detach().clone() for k, v in m.named_buffers()}
        del m
        wn, wc = _grad_report(grads, sd)
        e_m = max(rel_max(pm[i], rpm[i]) for i in range(B))
        res[dt] = (loss, e_m, wn, wc, bufs)
        print(f"C3 bs{B} {dt} vs oracle @1024: loss {loss:.6g}/{float(rloss):.6g}, logits max-rel {e_m:.3g}, "
              f"worst grad-norm {wn}, worst cos {wc}")
    loss, e_m, wn, wc, bufs = res["f32"]
    assert abs(loss - float(rloss)) <= 1e-4 * abs(float(rloss))
    assert e_m <= 2e-4
    assert wn[0] <= 2e-3, wn
    assert wc[0] >= 0.999, wc
    n = 0
    for k, v in sd.items():
        if "running_" in k and "refinenet4.resConfUnit1" not in k:
            assert float((bufs[k] - v.detach()).abs().max()) <= 1e-4 * max(float(v.abs().max()), 1e-6), k
            n += 1
    assert n == 28
    loss, e_m, wn, wc, _ = res["bf16"]
    assert abs(loss - float(rloss)) <= 2e-2 * abs(float(rloss))
    assert wc[0] >= 0.99, wc


def test_c3_bs16_bf16_vs_strict():
    from s3od_amd.model import DPTSegmentation
    x, masks = _batch(16, 1024, 32)
    m = DPTSegmentation(compute_dtype="f32").cuda()
    loss_s, _, g_s = _train_grads(m, x, masks)
    m2 = DPTSegmentation(compute_dtype="bf16").cuda()     # same synthetic init, fresh BN state
    loss_b, _, g_b = _train_grads(m2, x, masks)
    del m, m2
    worst_n, worst_c = (0.0, ""), (1.0, "")
    for n, gs in g_s.items():
        if "resConfUnit" in n and (n.endswith("conv1.bias") or n.endswith("conv2.bias")):
            continue
        gb = g_b[n]
        en = abs(float(gb.norm()) - float(gs.norm())) / max(float(gs.norm()), 1e-12)
        worst_n = max(worst_n, (en, n)); worst_c = min(worst_c, (cosine(gb, gs), n))
    print(f"C3 bs16 bf16 vs f32: loss {loss_b:.6g}/{loss_s:.6g}, worst grad-norm {worst_n}, worst cos {worst_c}")
    assert abs(loss_b - loss_s) <= 2e-2 * abs(loss_s)
    assert worst_n[0] <= 6e-2, worst_n
    assert worst_c[0] >= 0.99, worst_c


# ------------------------------------------------------------------------------------ C5
def test_c5_2048_bf16_vs_strict(model):
    x, _ = _batch(4, 2048, 51)
    with torch.no_grad():
        model.compute_dtype = "f32"
        s = model(x)
        pm_s, iou_s = s["pred_masks"].clone(), s["pred_iou"].clone()
        del s
        model.compute_dtype = "bf16"
        b = model(x)
    model.compute_dtype = "f32"
    e = rel_l2(b["pred_masks"], pm_s)
    agree = float(((b["pred_masks"] > 0) == (pm_s > 0)).float().mean())
    print(f"C5 bf16 vs f32 @2048 bs4: rel-L2 {e:.4g}, sign agreement {agree:.5f}, iou rel-L2 {rel_l2(b['pred_iou'], iou_s):.3g}")
    assert tuple(b["pred_masks"].shape) == (4, 3, 2048, 2048)
    assert e <= 3e-2 and agree >= 0.98
    assert rel_l2(b["pred_iou"], iou_s) <= 3e-2


def test_c5_one_image_strict_vs_oracle(model):
    from oracle import s3od_oracle as O
    import time
    x, _ = _batch(1, 2048, 52)
    model.compute_dtype = "f32"
    t0 = time.time()
    with torch.no_grad():
        out = model(x)
        torch.cuda.synchronize()
        t1 = time.time()
        ref = O.forward(x, _oracle_sd())
        torch.cuda.synchronize()
    print(f"C5 phases: engine f32 forward {t1 - t0:.1f} s, oracle forward {time.time() - t1:.1f} s", flush=True)
    e_m = rel_max(out["pred_masks"], ref["pred_masks"])
    e_i = rel_max(out["pred_iou"], ref["pred_iou"])
    print(f"C5 strict vs oracle @2048: logits {e_m:.3g}, iou {e_i:.3g}")
    assert e_m <= 2e-4 and e_i <= 2e-4
    assert int(out["pred_iou"].argmax(1)) == int(ref["pred_iou"].argmax(1))


# ------------------------------------------------------------------------------------ bf16 vs the oracle
def test_bf16_vs_oracle_production_sizes(model):
    """The bf16 fast path checked against the ORACLE (not against the build's own f32 path) at the sizes the
    metric is quoted on: image 0 of a bs-8 1024^2 batch (C2) and of a bs-4 2048^2 batch (C5), and a bs-1
    1024^2 train step's gradients (C3).  Reported with the flip band of SURVEY §8(c) (pixels whose oracle
    logit lies within 2*max|d| of zero); written to gpurun_out/bf16_vs_oracle.json when that directory exists.
    Bounds: logits rel-L2 <= 3e-2, sign agreement >= 0.98, every pixel outside the flip band agrees,
    pred_iou rel-L2 <= 3e-2; C3 loss within 2 %, per-parameter gradient cosine >= 0.99."""
    import json
    import os
    from oracle import s3od_oracle as O
    from s3od_amd.model import DPTSegmentation
    rec = {}
    sd = _oracle_sd()
    for tag, B, S, seed in (("C2", 8, 1024, 61), ("C5", 4, 2048, 62)):
        x, _ = _batch(B, S, seed)
        model.compute_dtype = "bf16"
        with torch.no_grad():
            out = model(x)
            pm, iou = out["pred_masks"][:1].float().clone(), out["pred_iou"][:1].clone()
            del out
            ref = O.forward(x[:1].contiguous(), sd)
        model.compute_dtype = "f32"
        r = ref["pred_masks"]
        d = (pm - r).abs()
        maxd = float(d.max())
        band = (r.abs() < 2 * maxd)
        agree = ((pm > 0) == (r > 0))
        inter = float(((pm > 0) & (r > 0)).sum()); union = float(((pm > 0) | (r > 0)).sum())
        top2 = torch.topk(ref["pred_iou"][0], 2).values
        rec[tag] = {"batch": B, "size": S, "logits_rel_l2": rel_l2(pm, r), "max_abs_diff": maxd,
                    "median_abs_logit": float(r.abs().median()), "flip_band_fraction": float(band.float().mean()),
                    "sign_agreement": float(agree.double().mean()),
                    "sign_agreement_outside_band": float(agree[~band].double().mean()),
                    "sign_flips_outside_band": int((~agree & ~band).sum()),
                    "mask_iou": inter / max(union, 1.0), "pred_iou_rel_l2": rel_l2(iou, ref["pred_iou"]),
                    "best_idx": int(iou.argmax(1)), "best_idx_ref": int(ref["pred_iou"].argmax(1)),
                    "ref_top2_margin": float(top2[0] - top2[1])}
        del ref, pm, r, d, band, agree, x
        torch.cuda.empty_cache()
    # C3: one train step at bs 1, 1024^2, bf16 vs the oracle's autograd
    x, masks = _batch(1, 1024, 63)
    m = DPTSegmentation(compute_dtype="bf16").cuda()
    loss, _, grads = _train_grads(m, x, masks)
    del m
    sdg = _oracle_sd(requires_grad=True)
    ref = O.forward(x, sdg, train=True, rope_rescale=1.3)
    rloss, *_ = O.multi_mask_loss(ref, masks, 0)
    rloss.backward()
    cos = sorted((cosine(g, sdg[n].grad), n) for n, g in grads.items()
                 if not ("resConfUnit" in n and (n.endswith("conv1.bias") or n.endswith("conv2.bias"))))
    rec["C3"] = {"batch": 1, "size": 1024, "loss": loss, "loss_ref": float(rloss),
                 "worst_grad_cosine": cos[0][0], "worst_param": cos[0][1],
                 "median_grad_cosine": cos[len(cos) // 2][0]}
    print("bf16 vs oracle:", json.dumps(rec))
    if os.path.isdir("gpurun_out"):
        json.dump(rec, open("gpurun_out/bf16_vs_oracle.json", "w"), indent=1)
    for tag in ("C2", "C5"):
        r = rec[tag]
        assert r["logits_rel_l2"] <= 3e-2 and r["sign_agreement"] >= 0.98, (tag, r)
        assert r["sign_flips_outside_band"] == 0, (tag, r)     # counted exactly (a float32 mean over 16M pixels is not)
        assert r["pred_iou_rel_l2"] <= 3e-2, (tag, r)
        if r["ref_top2_margin"] > 0.05:
            assert r["best_idx"] == r["best_idx_ref"], (tag, r)
    assert abs(rec["C3"]["loss"] - rec["C3"]["loss_ref"]) <= 2e-2 * abs(rec["C3"]["loss_ref"])
    assert rec["C3"]["worst_grad_cosine"] >= 0.99, rec["C3"]
