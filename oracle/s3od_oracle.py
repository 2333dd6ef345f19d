"""ORACLE — test infrastructure only.  CPU fp32 restatement of the S3OD hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / CPU baseline — never as the product path.
The product (``s3od_amd``) runs every op through ``libs3od_hip.so`` and fails loudly if it
is missing.

It restates, in plain PyTorch fp32 on the CPU with no ``transformers`` import:
  * DINOv3 ViT-B/16 (third-party transformers, pinned 4.57.1 by ``uv.lock:4870-4871``;
    container copy 5.15.0 at ``tf:models/dinov3_vit/modeling_dinov3_vit.py``)
  * the DPT head + MultiMaskHead (``src/s3od/model.py:109-467``)
  * the multi-mask loss (``synth_sod/src/synth_sod/model_training/loss.py:34-275``)
  * remove_background pre/post-processing (``src/s3od/predictor.py:79-139``,
    ``src/s3od/utils.py:6-37``)

Parity pin: ``tests/golden/make_golden.py`` imports the reference itself (this container
only) and writes ``tests/golden/*.npz``; ``tests/test_oracle_golden.py`` checks this
restatement against them.  The reference publishes no numeric golden vectors of its own,
so the pin is "reference run here on synthetic weights" (SURVEY.md §8c).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

HIDDEN, HEADS, HEAD_DIM, N_REG, PATCH, EPS = 768, 12, 64, 4, 16, 1e-5
ROPE_THETA = 100.0
TAPS = (2, 5, 8, 11)
# MT/model.py:28-32 intermediate_layer_idx per encoder (hidden 768 = ViT-B/16, 1024 = ViT-L/16)
TAPS_BY_HIDDEN = {768: (2, 5, 8, 11), 1024: (4, 11, 17, 23)}


def _hidden(sd):
    return sd["encoder.embeddings.patch_embeddings.weight"].shape[0]


# ---------------------------------------------------------------- encoder (DINOv3)
def patch_embed(x, sd):
    """tf:…/modeling_dinov3_vit.py:75-92 — conv k16 s16, then cat(cls, registers, patches)."""
    B = x.shape[0]
    p = F.conv2d(x, sd["encoder.embeddings.patch_embeddings.weight"],
                 sd["encoder.embeddings.patch_embeddings.bias"], stride=PATCH)
    p = p.flatten(2).transpose(1, 2)
    cls = sd["encoder.embeddings.cls_token"].expand(B, -1, -1)
    reg = sd["encoder.embeddings.register_tokens"].expand(B, -1, -1)
    return torch.cat([cls, reg, p], dim=1)


def rope_cos_sin(ph, pw, rescale=None):
    """tf:…:96-121 (patch centres in [-1,1], (y,x) order), :124-150 (train-mode rescale),
    :168-200 (angles = 2*pi*coord*inv_freq, flatten(1,2), tile(2))."""
    inv_freq = 1.0 / ROPE_THETA ** torch.arange(0, 1, 4 / HEAD_DIM, dtype=torch.float32)
    ch = torch.arange(0.5, ph, dtype=torch.float32) / ph
    cw = torch.arange(0.5, pw, dtype=torch.float32) / pw
    coords = torch.stack(torch.meshgrid(ch, cw, indexing="ij"), dim=-1).flatten(0, 1)
    coords = 2.0 * coords - 1.0
    if rescale is not None:
        coords = coords * torch.tensor(rescale, dtype=torch.float32)
    ang = 2 * math.pi * coords[:, :, None] * inv_freq[None, None, :]
    ang = ang.flatten(1, 2).tile(2)
    return torch.cos(ang), torch.sin(ang)


def _rotate_half(x):
    """tf:…:203-207."""
    h = x.shape[-1] // 2
    return torch.cat((-x[..., h:], x[..., :h]), dim=-1)


def attention(h, sd, p, cos, sin):
    """tf:…:294-334 + apply_rotary_pos_emb :238-268 (RoPE on patch tokens only) +
    SDPA (tf:integrations/sdpa_attention.py; eager-equivalent tf:…:210-235)."""
    B, N, D = h.shape
    heads = D // HEAD_DIM
    q = F.linear(h, sd[p + "attention.q_proj.weight"], sd[p + "attention.q_proj.bias"])
    k = F.linear(h, sd[p + "attention.k_proj.weight"])                      # key_bias=false
    v = F.linear(h, sd[p + "attention.v_proj.weight"], sd[p + "attention.v_proj.bias"])
    q, k, v = (t.view(B, N, heads, HEAD_DIM).transpose(1, 2) for t in (q, k, v))
    npfx = N - cos.shape[0]
    qp, kp = q[:, :, npfx:], k[:, :, npfx:]
    qp = qp * cos + _rotate_half(qp) * sin
    kp = kp * cos + _rotate_half(kp) * sin
    q = torch.cat([q[:, :, :npfx], qp], dim=2)
    k = torch.cat([k[:, :, :npfx], kp], dim=2)
    s = torch.matmul(q, k.transpose(2, 3)) * (HEAD_DIM ** -0.5)
    a = torch.softmax(s, dim=-1)
    o = torch.matmul(a, v).transpose(1, 2).reshape(B, N, D)
    return F.linear(o, sd[p + "attention.o_proj.weight"], sd[p + "attention.o_proj.bias"])


def vit_layer(x, sd, i, cos, sin):
    """tf:…:419-445 — pre-LN block with LayerScale; MLP :346-357 with exact (erf) GELU."""
    p = f"encoder.model.layer.{i}."
    D = x.shape[-1]
    h = F.layer_norm(x, (D,), sd[p + "norm1.weight"], sd[p + "norm1.bias"], EPS)
    x = attention(h, sd, p, cos, sin) * sd[p + "layer_scale1.lambda1"] + x
    h = F.layer_norm(x, (D,), sd[p + "norm2.weight"], sd[p + "norm2.bias"], EPS)
    h = F.linear(h, sd[p + "mlp.up_proj.weight"], sd[p + "mlp.up_proj.bias"])
    h = F.gelu(h)
    h = F.linear(h, sd[p + "mlp.down_proj.weight"], sd[p + "mlp.down_proj.bias"])
    return h * sd[p + "layer_scale2.lambda1"] + x


def encoder_taps(x, sd, rope_rescale=None):
    """hidden_states = (emb, L0..L{n-1}) (tf:utils/output_capturing.py:112-117); S3OD taps
    indices [2,5,8,11] for ViT-B, [4,11,17,23] for ViT-L (MT/model.py:28-32, src/s3od/model.py:62-86)
    and drops 1+4 prefix tokens.  Layers from the last tap on and the final norm never reach the
    outputs, so they are not run."""
    ph, pw = x.shape[-2] // PATCH, x.shape[-1] // PATCH
    cos, sin = (t.to(x.device) for t in rope_cos_sin(ph, pw, rope_rescale))
    h = patch_embed(x, sd)
    taps_idx = TAPS_BY_HIDDEN[_hidden(sd)]
    taps = []
    for i in range(max(taps_idx)):
        h = vit_layer(h, sd, i, cos, sin)
        if i + 1 in taps_idx:
            taps.append(h[:, 1 + N_REG:])
    return taps


# ---------------------------------------------------------------- DPT head
def _bn(x, sd, p, train, momentum=0.1):
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"],
                        sd[p + ".bias"], training=train, momentum=momentum, eps=1e-5)


def rcu(x, sd, p, train):
    """src/s3od/model.py:334-345 (bn=True): x + BN2(conv2(relu(BN1(conv1(relu(x))))))."""
    out = F.relu(x)
    out = F.conv2d(out, sd[p + "conv1.weight"], sd[p + "conv1.bias"], padding=1)
    out = _bn(out, sd, p + "bn1", train)
    out = F.relu(out)
    out = F.conv2d(out, sd[p + "conv2.weight"], sd[p + "conv2.bias"], padding=1)
    out = _bn(out, sd, p + "bn2", train)
    return out + x


def fusion(sd, r, train, x0, x1=None, size=None):
    """src/s3od/model.py:383-405: (+RCU1(skip)) → RCU2 → bilinear(align_corners=False) → 1x1."""
    p = f"seg_head.scratch.refinenet{r}."
    out = x0
    if x1 is not None:
        out = out + rcu(x1, sd, p + "resConfUnit1.", train)
    out = rcu(out, sd, p + "resConfUnit2.", train)
    if size is not None:
        out = F.interpolate(out, size=size, mode="bilinear", align_corners=False)
    else:
        out = F.interpolate(out, scale_factor=2, mode="bilinear", align_corners=False)
    return F.conv2d(out, sd[p + "out_conv.weight"], sd[p + "out_conv.bias"])


def dpt_head(taps, sd, ph, pw, train=False):
    """src/s3od/model.py:193-238 (+ _make_scratch :244-298, MultiMaskHead :455-467,
    classifier_head :185-191)."""
    h = "seg_head."
    feats = []
    for i, t in enumerate(taps):
        x = t.permute(0, 2, 1).reshape(t.shape[0], t.shape[-1], ph, pw)
        x = F.conv2d(x, sd[h + f"projects.{i}.weight"], sd[h + f"projects.{i}.bias"])
        if i == 0:
            x = F.conv_transpose2d(x, sd[h + "resize_layers.0.weight"], sd[h + "resize_layers.0.bias"], stride=4)
        elif i == 1:
            x = F.conv_transpose2d(x, sd[h + "resize_layers.1.weight"], sd[h + "resize_layers.1.bias"], stride=2)
        elif i == 3:
            x = F.conv2d(x, sd[h + "resize_layers.3.weight"], sd[h + "resize_layers.3.bias"], stride=2, padding=1)
        feats.append(x)
    rn = [F.conv2d(f, sd[h + f"scratch.layer{i + 1}_rn.weight"], None, padding=1) for i, f in enumerate(feats)]
    p4 = fusion(sd, 4, train, rn[3], size=rn[2].shape[2:])
    p3 = fusion(sd, 3, train, p4, rn[2], size=rn[1].shape[2:])
    p2 = fusion(sd, 2, train, p3, rn[1], size=rn[0].shape[2:])
    p1 = fusion(sd, 1, train, p2, rn[0])
    # classifier_head: AdaptiveAvgPool2d(1) → Linear → ReLU → Linear
    pooled = p1.mean(dim=(2, 3))
    iou = F.linear(F.relu(F.linear(pooled, sd[h + "classifier_head.2.weight"], sd[h + "classifier_head.2.bias"])),
                   sd[h + "classifier_head.4.weight"], sd[h + "classifier_head.4.bias"])
    m = h + "mask_head."
    f = F.conv2d(p1, sd[m + "output_conv1.weight"], sd[m + "output_conv1.bias"], padding=1)
    f = F.relu(F.conv_transpose2d(f, sd[m + "upsample_2x.0.weight"], sd[m + "upsample_2x.0.bias"], stride=2, padding=1))
    f = F.relu(F.conv2d(f, sd[m + "upsample_2x.2.weight"], sd[m + "upsample_2x.2.bias"], padding=1))
    # F.interpolate(size=(16ph,16pw), bilinear, antialias=True) is an exact identity here
    # (the feature is already 16*patch); kept explicit for fidelity.
    f = F.interpolate(f, size=(PATCH * ph, PATCH * pw), mode="bilinear", align_corners=False, antialias=True)
    masks = []
    n_masks = sum(1 for k in sd if k.startswith(m + "mask_heads.") and k.endswith(".0.weight"))
    for k in range(n_masks):
        g = F.relu(F.conv2d(f, sd[m + f"mask_heads.{k}.0.weight"], sd[m + f"mask_heads.{k}.0.bias"], padding=1))
        masks.append(F.conv2d(g, sd[m + f"mask_heads.{k}.2.weight"], sd[m + f"mask_heads.{k}.2.bias"]))
    return {"pred_masks": torch.cat(masks, dim=1), "pred_iou": iou, "features": p1}


def forward(x, sd, train=False, rope_rescale=None):
    """DPTSegmentation.forward, src/s3od/model.py:99-106."""
    ph, pw = x.shape[-2] // PATCH, x.shape[-1] // PATCH
    taps = encoder_taps(x, sd, rope_rescale if train else None)
    return dpt_head(taps, sd, ph, pw, train=train)


# ---------------------------------------------------------------- loss
def focal_loss(pred, target, alpha=0.25, gamma=2.0):
    """loss.py:126-143 with reduction='none' (pred is already sigmoid(logits): Quirk 3)."""
    bce = F.binary_cross_entropy_with_logits(pred, target, reduction="none")
    pt = torch.exp(-bce)
    return alpha * (1 - pt) ** gamma * bce


def iou_loss(pred, target, smooth=1e-6):
    """loss.py:79-99, reduction='none'."""
    pred = pred.reshape(pred.shape[0], -1)
    target = target.reshape(target.shape[0], -1)
    inter = (pred * target).sum(1)
    union = pred.sum(1) + target.sum(1) - inter
    return 1 - (inter + smooth) / (union + smooth)


def _gauss_window(ws=11, sigma=1.5):
    g = torch.exp(torch.tensor([-(x - ws // 2) ** 2 / float(2 * sigma ** 2) for x in range(ws)]))
    g = g / g.sum()
    return (g[:, None] @ g[None, :])[None, None]


def ssim_loss(img1, img2, ws=11):
    """loss.py:34-76 with reduction='none'."""
    w = _gauss_window(ws).to(device=img1.device, dtype=img1.dtype)
    mu1 = F.conv2d(img1, w, padding=ws // 2)
    mu2 = F.conv2d(img2, w, padding=ws // 2)
    mu1_sq, mu2_sq, mu12 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s1 = F.conv2d(img1 * img1, w, padding=ws // 2) - mu1_sq
    s2 = F.conv2d(img2 * img2, w, padding=ws // 2) - mu2_sq
    s12 = F.conv2d(img1 * img2, w, padding=ws // 2) - mu12
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    m = ((2 * mu12 + C1) * (2 * s12 + C2)) / ((mu1_sq + mu2_sq + C1) * (s1 + s2 + C2))
    return 1 - m.mean((1, 2, 3))


FOCAL_IOU = dict(components=[("focal_loss", 20.0, "focal"), ("iou_loss", 1.0, "iou")],
                 mse_weight=0.05, full_mask_lambda=0.1, decay_rate=0.2)
BCE_IOU_SSIM = dict(components=[("bce_loss", 30.0, "bce"), ("iou_loss", 0.5, "iou"), ("ssim_loss", 10.0, "ssim")],
                    mse_weight=0.05, full_mask_lambda=0.1, decay_rate=0.2)


def multi_mask_loss(outputs, masks, epoch=0, cfg=FOCAL_IOU):
    """loss.py:190-233 (MaskLossHandler.compute_multi_mask_losses) + :242-275 (aux MSE).
    Returns (loss, parts) with parts' tensors reduced by .mean() as LossModule.forward does."""
    logits = outputs["pred_masks"]
    B, M = logits.shape[:2]
    H, W = logits.shape[2:]
    tgt = masks.unsqueeze(1).expand(-1, M, -1, -1)
    lam = cfg["full_mask_lambda"] * math.exp(-cfg["decay_rate"] * epoch)
    p = torch.sigmoid(logits)
    pf = p.reshape(B * M, 1, H, W)
    tf = tgt.reshape(B * M, 1, H, W)
    with torch.no_grad():   # compute_iou :155-164 (squares form)
        inter = (tf * pf).reshape(B * M, 1, -1).sum(2)
        union = (tf ** 2).reshape(B * M, 1, -1).sum(2) + (pf ** 2).reshape(B * M, 1, -1).sum(2) - inter
        ious = ((inter + 1e-6) / (union + 1e-6)).mean(1).reshape(B, M)
    best = ious.argmax(dim=1)
    total = torch.zeros((), device=logits.device)
    parts = {"best_iou": ious.max(dim=1)[0].mean(), "gt_ious": ious}
    for name, w, kind in cfg["components"]:
        if kind == "focal":
            a = focal_loss(pf, tf).mean(dim=(1, 2, 3))
        elif kind == "bce":
            a = F.binary_cross_entropy(pf, tf, reduction="none").mean(dim=(1, 2, 3))
        elif kind == "iou":
            a = iou_loss(pf, tf)
        elif kind == "ssim":
            a = ssim_loss(pf, tf)
        a = a.reshape(B, M)
        b = a.gather(1, best.unsqueeze(1)).mean()
        total = total + w * (b + a.mean() * lam)
        parts[f"{name}_best"] = b
        parts[f"{name}_full"] = a
    mse = F.mse_loss(torch.sigmoid(outputs["pred_iou"]), ious)
    total = total + cfg["mse_weight"] * mse
    parts["mse_ious_loss"] = mse
    parts = {k: (v.mean() if v.dim() > 0 else v) for k, v in parts.items()}
    return total, parts, best, ious


def single_mask_loss(outputs, masks, cfg=FOCAL_IOU):
    """loss.py:166-188 (MaskLossHandler.compute_single_mask_loss, num_outputs=1): each mask criterion on
    the [B,H,W] maps, .mean(); no best-mask selection, no decay term, no aux MSE."""
    pred = torch.sigmoid(outputs["pred_masks"].squeeze(1))
    total = torch.zeros((), device=pred.device)
    parts = {}
    for name, w, kind in cfg["components"]:
        if kind == "focal":
            a = focal_loss(pred, masks).mean()
        elif kind == "bce":
            a = F.binary_cross_entropy(pred, masks, reduction="none").mean()
        elif kind == "iou":
            a = iou_loss(pred, masks).mean()
        else:
            raise RuntimeError("SSIMLoss fails on [B,H,W] maps in the reference")
        total = total + w * a
        parts[name] = a
    return total, parts


# ---------------------------------------------------------------- remove_background pieces
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def get_pad_info(h, w, image_size=1024):
    """src/s3od/utils.py:6-29."""
    aspect = w / h
    if aspect > 1:
        new_w = image_size
        new_h = int(new_w / aspect)
        return dict(height_pad=(image_size - new_h) // 2, width_pad=0, original_size=(h, w), resized_size=(new_h, new_w))
    new_h = image_size
    new_w = int(new_h * aspect)
    return dict(height_pad=0, width_pad=(image_size - new_w) // 2, original_size=(h, w), resized_size=(new_h, new_w))


def normalize(img_u8):
    """predictor.py:91-92: (x/255 - mean)/std in float64, then .float(); → [1,3,S,S]."""
    import numpy as np
    x = (img_u8.astype(np.float32) / 255.0 - np.array(IMAGENET_MEAN)) / np.array(IMAGENET_STD)
    return torch.from_numpy(x).permute(2, 0, 1).unsqueeze(0).float()


def postprocess(pred_masks_logits, pred_iou_logits, pad_info):
    """predictor.py:113-128: sigmoid, remove_padding (utils.py:32-37), antialias bilinear
    resize to the original size, argmax(sigmoid(iou))."""
    pm = torch.sigmoid(pred_masks_logits)
    ious = torch.sigmoid(pred_iou_logits).squeeze(0).numpy()
    m = pm.squeeze(0)
    if pad_info["height_pad"] > 0:
        m = m[:, pad_info["height_pad"]:-pad_info["height_pad"], :]
    if pad_info["width_pad"] > 0:
        m = m[:, :, pad_info["width_pad"]:-pad_info["width_pad"]]
    allm = F.interpolate(m.unsqueeze(0), size=pad_info["original_size"], mode="bilinear",
                         align_corners=False, antialias=True).squeeze(0).float().numpy()
    best = ious.argmax()
    return allm, ious, best
