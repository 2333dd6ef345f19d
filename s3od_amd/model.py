"""Drop-in ``DPTSegmentation`` (reference: src/s3od/model.py:89-106 and the training copy
synth_sod/src/synth_sod/model_training/model.py:84-101, instantiated by Hydra
``_target_`` at lightning_module.py:157).

Same constructor kwargs, same ``.encoder`` / ``.seg_head`` sub-modules (AdamW param groups,
lightning_module.py:185-188), same state_dict keys (371 entries, canonical = transformers 5.x
layout; the 4.x ``encoder.layer.{i}`` layout and Lightning ``model.`` prefixes are accepted
by ``load_state_dict``), same output dict {"pred_masks", "pred_iou", "features"}.

The arithmetic runs in libs3od_hip.so through ``engine.DPTEngine``; this module holds the
fp32 parameters (masters) and wires PyTorch autograd to the native backward.
"""
from __future__ import annotations

import random

import numpy as np
import torch
import torch.nn as nn

from .weights import param_specs, synthetic_state_dict, canonicalize_state_dict

_ENCODERS = {"dinov3_base", "facebook/dinov3-vitb16-pretrain-lvd1689m", "dinob"}


def _container():
    return nn.Module()


class _Tree(nn.Module):
    pass


def _build_tree(root: nn.Module, specs):
    for name, shape, kind in specs:
        parts = name.split(".")
        mod = root
        for p in parts[:-1]:
            if p not in mod._modules:
                mod.add_module(p, _Tree())
            mod = mod._modules[p]
        leaf = parts[-1]
        if kind.startswith("bn_") and kind not in ("bn_w", "bn_b"):
            dt = torch.int64 if kind == "bn_nbt" else torch.float32
            mod.register_buffer(leaf, torch.zeros(shape, dtype=dt))
        else:
            mod.register_parameter(leaf, nn.Parameter(torch.zeros(shape, dtype=torch.float32)))


class DPTSegmentation(nn.Module):
    """DINOv3 ViT-B/16 + DPT head + 3-way MultiMaskHead on MI355X HIP kernels."""

    def __init__(self, num_classes=1, num_outputs=3, encoder_name="dinov3_base", features=256, out_channels=None,
                 use_bn=True, use_clstoken=False, compute_dtype="bf16", init_seed=0, **kwargs):
        super().__init__()
        if num_classes != 1 or num_outputs != 3 or features != 256 or not use_bn or use_clstoken:
            raise NotImplementedError("only the published S3OD configuration (dinob, 3 masks, 256 features, BN) is built")
        if out_channels not in (None, [256, 512, 1024, 1024], (256, 512, 1024, 1024)):
            raise NotImplementedError("out_channels must be [256, 512, 1024, 1024]")
        if encoder_name not in _ENCODERS:
            raise NotImplementedError(f"encoder {encoder_name!r}: only ViT-B/16 (dinov3_base) is built")
        self.patch_size = 16
        self.encoder_name = encoder_name
        self.use_flux_features = False
        self.compute_dtype = compute_dtype
        _build_tree(self, param_specs())
        if init_seed is not None:
            sd = synthetic_state_dict(init_seed)
            with torch.no_grad():
                own = self.state_dict(keep_vars=True)
                for k, v in sd.items():
                    own[k].copy_(torch.from_numpy(np.asarray(v)))
        self._engine = None
        self._rope_rescale = None   # train-mode RoPE rescale override (parity tests)

    # ---------------------------------------------------------------- state dict
    def load_state_dict(self, state_dict, strict=True, assign=False):
        return super().load_state_dict(canonicalize_state_dict(state_dict), strict=strict, assign=assign)

    # ---------------------------------------------------------------- engine
    def engine(self):
        from .engine import DPTEngine
        dev = next(self.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError("DPTSegmentation runs on the MI355X HIP kernels only: move the model to a GPU (model.cuda())")
        params = dict(self.named_parameters())
        bufs = dict(self.named_buffers())
        e = self._engine
        if e is None or e.p.keys() != params.keys() or any(e.p[k] is not v for k, v in params.items()) or \
                any(e.buf[k] is not v for k, v in bufs.items()):
            e = DPTEngine(params, bufs, self.compute_dtype)
            self._engine = e
        if e.cdt != self.compute_dtype:
            e.set_dtype(self.compute_dtype)
        return e

    def sample_rope_rescale(self):
        """tf:…/modeling_dinov3_vit.py:124-150 with pos_embed_rescale=2.0: exp(U(-ln 2, ln 2))."""
        if self._rope_rescale is not None:
            return float(self._rope_rescale)
        r = np.log(2.0)
        return float(torch.empty(1).uniform_(-r, r).exp().item())

    def forward(self, x):
        eng = self.engine()
        if self.training and torch.is_grad_enabled():
            from .autograd import dpt_train_forward
            return dpt_train_forward(self, eng, x)
        with torch.no_grad():
            rescale = self.sample_rope_rescale() if self.training else None
            return eng.forward(x, train=self.training, rope_rescale=rescale)
