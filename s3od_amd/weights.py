"""Parameter inventory, deterministic synthetic weights and checkpoint key mapping.

The reference network (``src/s3od/model.py:11-467`` + transformers ``DINOv3ViTModel``)
has 371 state-dict entries (323 parameters + 48 persistent BatchNorm buffers).  Real
weights (``okupyn/s3od``) are not available offline, so every parity fixture and every
benchmark uses the deterministic synthetic scheme below: each entry is drawn from its own
counter-based Philox stream keyed by (seed, crc32(name)), so the same 464 MB of fp32
weights can be regenerated bit-identically anywhere without committing them.

Canonical key layout = the reference's own ``model.state_dict()`` under transformers 5.x
(``encoder.model.layer.{i}.…``).  ``canonicalize_state_dict`` also accepts the
transformers 4.56/4.57 layout (``encoder.layer.{i}.…``, the published checkpoint's
layout: ``src/s3od/dinov3_config/config.json:29``) and Lightning ``model.``-prefixed keys
(``scripts/export_model.py:95-104``).
"""
from __future__ import annotations

import zlib
from collections import OrderedDict, namedtuple

import numpy as np

HIDDEN = 768
HEADS = 12
HEAD_DIM = 64
MLP = 3072
N_LAYERS = 12
N_REG = 4
PATCH = 16
TAPS = (2, 5, 8, 11)          # hidden_states indices, src/s3od/model.py:36-40
OUT_CH = (256, 512, 1024, 1024)  # src/s3od/model.py:45
FEAT = 256
N_MASKS = 3

# Encoder geometries of the two published model configs (synth_sod/.../config/model/{dinob,dinol}.yaml):
#   dinob: facebook/dinov3-vitb16-pretrain-lvd1689m (src/s3od/dinov3_config/config.json: hidden 768,
#          12 layers, 12 heads, intermediate 3072), taps [2,5,8,11] (MT/model.py:28-32);
#   dinol: facebook/dinov3-vitl16-pretrain-lvd1689m (transformers' DINOv3ViT-L/16 geometry: hidden 1024,
#          24 layers, 16 heads of 64, intermediate 4096, 4 registers, same RoPE / LayerScale / key_bias=False),
#          taps [4,11,17,23] (MT/model.py:28-32).  Its config file is not in the reference tree.
Variant = namedtuple("Variant", "hidden layers heads mlp taps")
VARIANTS = {
    "dinob": Variant(768, 12, 12, 3072, (2, 5, 8, 11)),
    "dinol": Variant(1024, 24, 16, 4096, (4, 11, 17, 23)),
}
ENCODER_VARIANT = {
    "dinov3_base": "dinob", "dinob": "dinob", "facebook/dinov3-vitb16-pretrain-lvd1689m": "dinob",
    "dinov3_large": "dinol", "dinol": "dinol", "facebook/dinov3-vitl16-pretrain-lvd1689m": "dinol",
}


def param_specs(variant: str = "dinob", n_masks: int = N_MASKS):
    """Ordered (name, shape, kind) for every state-dict entry of DPTSegmentation.

    kind drives the synthetic init: 'lin' (fan-in scaled normal), 'bias', 'ln_w', 'ln_b',
    'ls' (LayerScale), 'tok', 'zero', 'bn_w', 'bn_b', 'bn_rm', 'bn_rv', 'bn_nbt', 'convT'.
    """
    V = VARIANTS[variant]
    HIDDEN, MLP, N_LAYERS, N_MASKS = V.hidden, V.mlp, V.layers, n_masks
    s = []
    e = "encoder.embeddings."
    s += [(e + "cls_token", (1, 1, HIDDEN), "tok"),
          (e + "mask_token", (1, 1, HIDDEN), "zero"),
          (e + "register_tokens", (1, N_REG, HIDDEN), "tok"),
          (e + "patch_embeddings.weight", (HIDDEN, 3, PATCH, PATCH), "lin"),
          (e + "patch_embeddings.bias", (HIDDEN,), "bias")]
    for i in range(N_LAYERS):
        p = f"encoder.model.layer.{i}."
        s += [(p + "norm1.weight", (HIDDEN,), "ln_w"), (p + "norm1.bias", (HIDDEN,), "ln_b"),
              (p + "attention.k_proj.weight", (HIDDEN, HIDDEN), "lin"),
              (p + "attention.v_proj.weight", (HIDDEN, HIDDEN), "lin"),
              (p + "attention.v_proj.bias", (HIDDEN,), "bias"),
              (p + "attention.q_proj.weight", (HIDDEN, HIDDEN), "lin"),
              (p + "attention.q_proj.bias", (HIDDEN,), "bias"),
              (p + "attention.o_proj.weight", (HIDDEN, HIDDEN), "lin"),
              (p + "attention.o_proj.bias", (HIDDEN,), "bias"),
              (p + "layer_scale1.lambda1", (HIDDEN,), "ls"),
              (p + "norm2.weight", (HIDDEN,), "ln_w"), (p + "norm2.bias", (HIDDEN,), "ln_b"),
              (p + "mlp.up_proj.weight", (MLP, HIDDEN), "lin"),
              (p + "mlp.up_proj.bias", (MLP,), "bias"),
              (p + "mlp.down_proj.weight", (HIDDEN, MLP), "lin"),
              (p + "mlp.down_proj.bias", (HIDDEN,), "bias"),
              (p + "layer_scale2.lambda1", (HIDDEN,), "ls")]
    s += [("encoder.norm.weight", (HIDDEN,), "ln_w"), ("encoder.norm.bias", (HIDDEN,), "ln_b")]
    h = "seg_head."
    for i, c in enumerate(OUT_CH):
        s += [(h + f"projects.{i}.weight", (c, HIDDEN, 1, 1), "lin"),
              (h + f"projects.{i}.bias", (c,), "bias")]
    s += [(h + "resize_layers.0.weight", (256, 256, 4, 4), "convT4"),
          (h + "resize_layers.0.bias", (256,), "bias"),
          (h + "resize_layers.1.weight", (512, 512, 2, 2), "convT4"),
          (h + "resize_layers.1.bias", (512,), "bias"),
          (h + "resize_layers.3.weight", (1024, 1024, 3, 3), "lin"),
          (h + "resize_layers.3.bias", (1024,), "bias")]
    for i, c in enumerate(OUT_CH):
        s.append((h + f"scratch.layer{i + 1}_rn.weight", (FEAT, c, 3, 3), "lin"))
    for r in (1, 2, 3, 4):
        p = h + f"scratch.refinenet{r}."
        s += [(p + "out_conv.weight", (FEAT, FEAT, 1, 1), "lin"), (p + "out_conv.bias", (FEAT,), "bias")]
        for u in (1, 2):
            q = p + f"resConfUnit{u}."
            s += [(q + "conv1.weight", (FEAT, FEAT, 3, 3), "lin"), (q + "conv1.bias", (FEAT,), "bias"),
                  (q + "conv2.weight", (FEAT, FEAT, 3, 3), "lin"), (q + "conv2.bias", (FEAT,), "bias")]
            for b in ("bn1", "bn2"):
                s += [(q + f"{b}.weight", (FEAT,), "bn_w"), (q + f"{b}.bias", (FEAT,), "bn_b"),
                      (q + f"{b}.running_mean", (FEAT,), "bn_rm"),
                      (q + f"{b}.running_var", (FEAT,), "bn_rv"),
                      (q + f"{b}.num_batches_tracked", (), "bn_nbt")]
    m = h + "mask_head."
    s += [(m + "output_conv1.weight", (128, 256, 3, 3), "lin"), (m + "output_conv1.bias", (128,), "bias"),
          (m + "upsample_2x.0.weight", (128, 64, 4, 4), "convT2"), (m + "upsample_2x.0.bias", (64,), "bias"),
          (m + "upsample_2x.2.weight", (64, 64, 3, 3), "lin"), (m + "upsample_2x.2.bias", (64,), "bias")]
    for k in range(N_MASKS):
        s += [(m + f"mask_heads.{k}.0.weight", (32, 64, 3, 3), "lin"), (m + f"mask_heads.{k}.0.bias", (32,), "bias"),
              (m + f"mask_heads.{k}.2.weight", (1, 32, 1, 1), "head"), (m + f"mask_heads.{k}.2.bias", (1,), "bias")]
    s += [(h + "classifier_head.2.weight", (64, 256), "lin"), (h + "classifier_head.2.bias", (64,), "bias"),
          (h + "classifier_head.4.weight", (N_MASKS, 64), "lin"), (h + "classifier_head.4.bias", (N_MASKS,), "bias")]
    return s


def _rng(name: str, seed: int) -> np.random.Generator:
    key = (int(seed) << 32) | zlib.crc32(name.encode())
    return np.random.Generator(np.random.Philox(key=key))


def synthetic_tensor(name: str, shape, kind: str, seed: int = 0) -> np.ndarray:
    """One entry of the deterministic synthetic checkpoint (float32, or int64 for counters)."""
    if kind == "bn_nbt":
        return np.zeros((), dtype=np.int64)
    if kind == "zero":
        return np.zeros(shape, dtype=np.float32)
    g = _rng(name, seed)
    n = g.standard_normal(shape, dtype=np.float32)
    if kind == "lin":
        fan_in = int(np.prod(shape[1:]))
        return n * np.float32(1.0 / np.sqrt(fan_in))
    if kind.startswith("convT"):
        # ConvTranspose2d weight [Cin, Cout, k, k]; each output sees Cin*(k/s)^2 taps.
        s_ = int(kind[-1])
        fan_in = shape[0] * (shape[2] * shape[3]) // (s_ * s_)
        return n * np.float32(1.0 / np.sqrt(fan_in))
    if kind == "head":
        # last 1x1 conv of each mask head: spread the logits so masks are not all ~0.5
        return n * np.float32(8.0 / np.sqrt(shape[1]))
    if kind == "bias":
        return n * np.float32(0.02)
    if kind in ("ln_w", "bn_w"):
        return np.float32(1.0) + np.float32(0.1) * n
    if kind in ("ln_b", "bn_b"):
        return np.float32(0.05) * n
    if kind == "ls":
        return np.float32(0.7) + np.float32(0.1) * n
    if kind == "tok":
        return np.float32(0.5) * n
    if kind == "bn_rm":
        return np.float32(0.1) * n
    if kind == "bn_rv":
        return (np.float32(1.0) + np.float32(0.25) * np.tanh(n)).astype(np.float32)
    raise ValueError(kind)


def synthetic_state_dict(seed: int = 0, variant: str = "dinob", n_masks: int = N_MASKS) -> "OrderedDict[str, np.ndarray]":
    return OrderedDict((n, synthetic_tensor(n, sh, k, seed)) for n, sh, k in param_specs(variant, n_masks))


def canonicalize_state_dict(sd):
    """Map any accepted checkpoint layout onto the canonical key set.

    Accepts: canonical keys; transformers-4.x encoder keys (``encoder.layer.{i}``); a
    Lightning checkpoint's ``model.`` prefix; a wrapping ``{"state_dict": ...}``.
    Non-persistent ``inv_freq`` is dropped.  Returns a new dict (values untouched).
    """
    if isinstance(sd, dict) and "state_dict" in sd and not any(k.startswith("encoder.") for k in sd):
        sd = sd["state_dict"]
    out = OrderedDict()
    for k, v in sd.items():
        if k.startswith("model."):
            k = k[len("model."):]
        if k.startswith("encoder.layer."):
            k = "encoder.model.layer." + k[len("encoder.layer."):]
        if k.endswith("rope_embeddings.inv_freq"):
            continue
        out[k] = v
    return out


def to_transformers4_layout(sd):
    """Inverse of the 5.x rename (``encoder.model.layer`` -> ``encoder.layer``)."""
    return OrderedDict(("encoder.layer." + k[len("encoder.model.layer."):] if k.startswith("encoder.model.layer.") else k, v)
                       for k, v in sd.items())
