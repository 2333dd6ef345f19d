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

from .weights import param_specs, synthetic_state_dict, canonicalize_state_dict, ENCODER_VARIANT, VARIANTS


def _container():
    return nn.Module()


class _Tree(nn.Module):
    """Plain container; numeric children are indexable like the reference's ModuleList/Sequential."""

    def __getitem__(self, i):
        return self._modules[str(i)]


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
    """DINOv3 ViT-B/16 (dinob) or ViT-L/16 (dinol) + DPT head + MultiMaskHead on MI355X HIP kernels."""

    def __init__(self, num_classes=1, num_outputs=3, encoder_name="dinov3_base", features=256, out_channels=None,
                 use_bn=True, use_clstoken=False, compute_dtype="bf16", init_seed=0, **kwargs):
        super().__init__()
        if num_classes != 1 or features != 256 or not use_bn or use_clstoken:
            raise NotImplementedError("only the published S3OD head configuration (1 class, 256 features, BN, "
                                      "no cls-token readout) is built")
        if num_outputs not in (1, 3):
            raise NotImplementedError(f"num_outputs={num_outputs}: the fused mask-head kernels are built for 1 (dinol) or 3 (dinob)")
        if out_channels not in (None, [256, 512, 1024, 1024], (256, 512, 1024, 1024)):
            raise NotImplementedError("out_channels must be [256, 512, 1024, 1024]")
        if encoder_name not in ENCODER_VARIANT:
            raise NotImplementedError(f"encoder {encoder_name!r}: ViT-B/16 (dinob) and ViT-L/16 (dinol) are built")
        self.patch_size = 16
        self.encoder_name = encoder_name
        self.variant = ENCODER_VARIANT[encoder_name]
        self.num_outputs = int(num_outputs)
        self.use_flux_features = False
        self.compute_dtype = compute_dtype
        _build_tree(self, param_specs(self.variant, self.num_outputs))
        if init_seed is not None:
            sd = synthetic_state_dict(init_seed, self.variant, self.num_outputs)
            with torch.no_grad():
                own = self.state_dict(keep_vars=True)
                for k, v in sd.items():
                    own[k].copy_(torch.from_numpy(np.asarray(v)))
        self._engine = None
        self._rope_rescale = None   # train-mode RoPE rescale override (parity tests)
        self._anchor = None
        self._flat = None           # flat fp32 gradient buffer (see _grad_views)
        self.grad_ready_callback = None   # fn(range_name, flat_slice) for bucketed all-reduce

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
            e = DPTEngine(params, bufs, self.compute_dtype, self.variant, self.num_outputs)
            self._engine = e
        if e.cdt != self.compute_dtype:
            e.set_dtype(self.compute_dtype)
        return e

    # ---------------------------------------------------------------- gradients
    def grad_layout(self):
        """Flat gradient order: reference order with q/k/v weights and the three mask heads'
        weights/biases made adjacent (they are produced by single fused kernels), encoder first.
        Returns (list of (name, numel, shape), dict range_name -> (start, end))."""
        nm = self.num_outputs
        specs = [(n, sh) for n, sh, k in param_specs(self.variant, nm) if not (k.startswith("bn_") and k not in ("bn_w", "bn_b"))]
        shapes = dict(specs)
        unused = set(self.unused_parameter_names())
        order = []
        done = set()
        for n, sh in specs:
            if n in done or n in unused:
                continue
            if n.endswith("attention.k_proj.weight") or n.endswith("attention.v_proj.weight"):
                continue
            if n.endswith("attention.q_proj.weight"):
                base = n[: -len("q_proj.weight")]
                grp = [base + "q_proj.weight", base + "k_proj.weight", base + "v_proj.weight"]
            elif ".mask_heads." in n:
                m = "seg_head.mask_head.mask_heads."
                grp = [m + f"{k}.{a}.{b}" for a, b in (("0", "weight"), ("0", "bias"), ("2", "weight"), ("2", "bias"))
                       for k in range(nm)]
                grp = [g for g in grp if g not in done]
            else:
                grp = [n]
            for g in grp:
                order.append(g); done.add(g)
        layout, ranges, off = [], {}, 0
        for n in order:
            numel = int(np.prod(shapes[n])) if shapes[n] else 1
            layout.append((n, off, numel, shapes[n]))
            key = "seg_head" if n.startswith("seg_head") else (
                "layer" + n.split(".")[3] if n.startswith("encoder.model.layer.") else "embeddings")
            a, b = ranges.get(key, (off, off))
            ranges[key] = (min(a, off), off + numel)
            off += numel
        return layout, ranges, off

    def unused_parameter_names(self):
        """Parameters the reference's forward never reaches (grad stays None): encoder layers at and
        after the last tap (dinob: layer 11; dinol: layer 23), the final norm, mask_token and
        refinenet4.resConfUnit1."""
        last = max(VARIANTS[self.variant].taps)
        specs = param_specs(self.variant, self.num_outputs)
        names = [n for n, sh, k in specs if n.startswith("encoder.model.layer.") and int(n.split(".")[3]) >= last]
        names += ["encoder.norm.weight", "encoder.norm.bias", "encoder.embeddings.mask_token"]
        names += [n for n, sh, k in specs if n.startswith("seg_head.scratch.refinenet4.resConfUnit1.")
                  and not (k.startswith("bn_") and k not in ("bn_w", "bn_b"))]
        return names

    def zero_grad(self, set_to_none: bool = True):
        """set_to_none=False zeroes the flat gradient buffer with one memset."""
        if not set_to_none and self._flat is not None:
            self._flat["buf"].zero_()
            for p in self.parameters():
                if p.grad is not None and not (self._flat["buf"].data_ptr() <= p.grad.data_ptr() <
                                               self._flat["buf"].data_ptr() + 4 * self._flat["buf"].numel()):
                    p.grad.zero_()
            return
        super().zero_grad(set_to_none=set_to_none)

    def _autograd_anchor(self):
        dev = next(self.parameters()).device
        if self._anchor is None or self._anchor.device != dev:
            self._anchor = torch.zeros((), device=dev, requires_grad=True)
        return self._anchor

    def _grad_views(self):
        """Make every reachable parameter's .grad a view of one flat fp32 buffer (zero-filled
        where .grad was None) and return name -> grad view, plus the fused views the kernels use."""
        params = dict(self.named_parameters())
        dev = next(iter(params.values())).device
        if self._flat is None or self._flat["buf"].device != dev:
            layout, ranges, total = self.grad_layout()
            self._flat = {"layout": layout, "ranges": ranges, "buf": torch.zeros(total, dtype=torch.float32, device=dev)}
        fl = self._flat
        buf = fl["buf"]
        G = {"_flat": buf}
        # after zero_grad(set_to_none=True) every .grad is None: ONE memset of the flat buffer
        # instead of a fill kernel per parameter (~220 launches per step)
        all_none = all(params[n].grad is None for n, _, _, _ in fl["layout"])
        if all_none:
            buf.zero_()
        for n, off, numel, shape in fl["layout"]:
            p = params[n]
            v = buf[off:off + numel].view(shape)
            g = p.grad
            if g is None:
                if not all_none:
                    v.zero_()
                p.grad = v
            elif g.data_ptr() != v.data_ptr():
                v.copy_(g)
                p.grad = v
            G[n] = v
        pos = {n: off for n, off, numel, shape in fl["layout"]}
        V, nm = VARIANTS[self.variant], self.num_outputs
        for i in range(max(V.taps)):
            q = f"encoder.model.layer.{i}.attention."
            o = pos[q + "q_proj.weight"]
            G[f"qkv_w{i}"] = buf[o:o + 3 * V.hidden * V.hidden]
        m = "seg_head.mask_head.mask_heads."
        for key, n, cnt in (("heads1_w", "0.0.weight", 32 * nm * 64 * 9), ("heads1_b", "0.0.bias", 32 * nm),
                            ("heads2_w", "0.2.weight", 32 * nm), ("heads2_b", "0.2.bias", nm)):
            o = pos[m + n]
            G[key] = buf[o:o + cnt]
        return G

    def _grad_ready_hook(self, name):
        cb = self.grad_ready_callback
        if cb is not None and self._flat is not None and name in self._flat["ranges"]:
            a, b = self._flat["ranges"][name]
            cb(name, self._flat["buf"][a:b])

    def _after_backward(self):
        cb = getattr(self, "grad_finish_callback", None)
        if cb is not None:
            cb()

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
