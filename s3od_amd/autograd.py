"""PyTorch autograd wiring for the native forward/backward.

``dpt_train_forward`` runs the training forward (train-mode BatchNorm, sampled RoPE rescale)
through ``DPTEngine`` and returns the reference output dict whose ``pred_masks`` / ``pred_iou``
carry a grad_fn.  Its backward runs ``DPTEngine.backward``, which accumulates (fp32 atomics)
straight into the model's flat gradient buffer; ``p.grad`` are views of that buffer, so
gradient accumulation across micro-batches, ``zero_grad`` and optimizers behave as with the
reference.  Parameters the reference never reaches (layer 11, final norm, mask_token,
refinenet4.resConfUnit1) keep ``grad = None`` exactly like the reference.
"""
from __future__ import annotations

import torch

from .engine import Ctx


class _DPTFn(torch.autograd.Function):
    @staticmethod
    def forward(fctx, x, anchor, model, eng, rescale):
        ctx = Ctx()
        out = eng.forward(x, train=True, rope_rescale=rescale, ctx=ctx)
        fctx.s3od = (model, eng, ctx)
        fctx.set_materialize_grads(False)     # an output the loss never reads arrives as None, not zeros
        # features (= path_1, NCHW view of the NHWC decoder tensor) carries grad like the reference's:
        # its gradient joins path_1's in the native backward.  The input images get no gradient
        # (data, never a leaf that requires grad in the reference's training).
        return out["pred_masks"], out["pred_iou"], out["features"]

    @staticmethod
    def backward(fctx, d_masks, d_iou, d_feat):
        model, eng, ctx = fctx.s3od
        G = model._grad_views()
        nm = model.num_outputs
        if d_masks is None:
            d_masks = torch.zeros((ctx.B, nm, 16 * ctx.ph, 16 * ctx.pw), dtype=torch.float32, device=G["_flat"].device)
        iou_unused = d_iou is None     # e.g. the single-mask loss (loss.py:166-188) never reads pred_iou
        if iou_unused:
            d_iou = torch.zeros((ctx.B, nm), dtype=torch.float32, device=G["_flat"].device)
        eng.grad_hook = model._grad_ready_hook
        try:
            eng.backward(ctx, d_masks.float().contiguous(), d_iou.float().contiguous(), G, d_feat=d_feat)
        finally:
            eng.grad_hook = None
            fctx.s3od = None
        if iou_unused:
            # the reference's classifier_head receives no gradient at all (grad None -> AdamW skips it)
            for p in model.seg_head.classifier_head.parameters():
                p.grad = None
        model._after_backward()
        return None, torch.zeros((), device=d_iou.device), None, None, None


def dpt_train_forward(model, eng, x):
    rescale = model.sample_rope_rescale()
    pm, iou, feat = _DPTFn.apply(x, model._autograd_anchor(), model, eng, rescale)
    return {"pred_masks": pm, "pred_iou": iou, "features": feat}


class _MaskLossFn(torch.autograd.Function):
    """Fused multi-mask loss; returns (loss, packed parts)."""

    @staticmethod
    def forward(fctx, logits, pred_iou, masks, cfg):
        from ._lib import lib, stream
        B, M = logits.shape[:2]
        HW = logits.shape[2] * logits.shape[3]
        dev = logits.device
        sums = torch.empty(B * M * 8, dtype=torch.float64, device=dev)
        coef = torch.empty(B * M * 4, dtype=torch.float32, device=dev)
        iou_ws = torch.empty(B * M * 2, dtype=torch.float32, device=dev)
        diu = torch.empty(B * M, dtype=torch.float32, device=dev)
        out = torch.empty(16 + B * M + B, dtype=torch.float32, device=dev)
        logits = logits.contiguous()
        masks = masks.contiguous().float()
        W = logits.shape[3]
        w_ssim = cfg.get("w_ssim", 0.0)
        lib()("s3od_mask_loss_fwd", logits, masks, pred_iou.contiguous().float(), B, M, HW, W, cfg["w_focal"], cfg["w_iou"],
              cfg["w_bce"], w_ssim, cfg["w_mse"], cfg["lam"], 0.25, 2.0, sums, coef, iou_ws, diu, out, stream())
        fctx.save_for_backward(logits, masks, coef, iou_ws, diu)
        fctx.dims = (B, M, HW, W, int(w_ssim != 0.0))
        fctx.mark_non_differentiable(out)
        return out[0], out

    @staticmethod
    def backward(fctx, g_loss, g_out):
        from ._lib import lib, stream
        logits, masks, coef, iou_ws, diu = fctx.saved_tensors
        B, M, HW, W, with_ssim = fctx.dims
        dl = torch.empty_like(logits)
        di = torch.empty((B, M), dtype=torch.float32, device=logits.device)
        g = g_loss.reshape(1).float().contiguous()
        lib()("s3od_mask_loss_bwd", logits, masks, coef, iou_ws, diu, g, dl, di, B, M, HW, W, with_ssim, 0.25, 2.0, stream())
        return dl, di, None, None


def mask_loss(logits, pred_iou, masks, cfg):
    return _MaskLossFn.apply(logits, pred_iou, masks, cfg)
