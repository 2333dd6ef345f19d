"""Native executor of the S3OD hot path: DINOv3 ViT-B/16 encoder + DPT decoder + mask heads.

Every arithmetic op runs in libs3od_hip.so (gfx950 HIP kernels); PyTorch only provides
device memory (caching allocator), streams and the autograd / nn.Module surface.

Layouts: tokens [B, Ntok, 768] (fp32 residual stream); q/k/v [B*12, Ntok, 64]; decoder
activations NHWC [B, H, W, C]; compute dtype T = bf16 (fast) or f32 (strict parity).
Parameters stay fp32 in the reference's state_dict layout; ``prepare()`` repacks them into
kernel layouts ([Cout][KH][KW][Cin], fused QKV [2304][768]) in T.

Reference structure: src/s3od/model.py:62-467 and tf:models/dinov3_vit/modeling_dinov3_vit.py.
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass, field

import torch

from ._lib import lib, stream, F32, BF16, NREP
from .weights import OUT_CH, VARIANTS

NREG = 4
ACT_NONE, ACT_RELU, ACT_GELU, ACT_GELU_BWD, ACT_RELU_BWD = 0, 1, 2, 3, 4
# bf16 training: the up-projection saves gelu'(v) (one erf for both outputs) and the down dgrad multiplies by it;
# the f32 strict path keeps the pre-activation and the exact erf GELU' (ACT_GELU_BWD)
ACT_GELU_SG, ACT_MUL = 5, 6


def _E(ref, n, dt, dev):
    return torch.empty(n, dtype=dt, device=dev)


@dataclass
class Ctx:
    """Tensors saved by a training forward for the native backward."""
    B: int = 0
    H: int = 0
    W: int = 0
    ph: int = 0
    pw: int = 0
    t: dict = field(default_factory=dict)


class DPTEngine:
    def __init__(self, params: dict, buffers: dict, compute_dtype: str = "bf16", variant: str = "dinob", n_masks: int = 3):
        """params / buffers: name -> fp32 CUDA tensor in the reference layout (canonical keys).
        variant: encoder geometry (weights.VARIANTS: dinob = ViT-B/16, dinol = ViT-L/16); n_masks: mask heads."""
        self.p = params
        self.buf = buffers
        c = VARIANTS[variant]
        self.D, self.H, self.MLP, self.taps = c.hidden, c.heads, c.mlp, c.taps
        self.last = max(c.taps)      # layers >= last (and the final norm) never reach the outputs
        self.nm = int(n_masks)
        self.set_dtype(compute_dtype)
        self.w = {}
        self._wkey = None
        self._zpool = {}       # persistent all-zero workspaces (the kernels that read them back leave them zero)
        self._nbt = []         # BatchNorm num_batches_tracked counters to bump once per forward
        self._slabs = {}       # hipStream_t -> split-K slab workspace (contents dead between calls)
        self._slab_need = {}   # shape key -> slab bytes the library asks for

    def zero_ws(self, key, n, dtype, dev):
        """Persistent workspace of >= n elements that is all zero between calls: every C-ABI entry given one
        (replicated column sums, BN statistics, split-K wgrad partials) clears what it reads back, so no
        memset is launched per call.  One buffer per key; all users run on one stream, in order."""
        t = self._zpool.get(key)
        if t is None or t.numel() < n or t.dtype != dtype or t.device != dev:
            t = torch.zeros(n, dtype=dtype, device=dev)
            self._zpool[key] = t
        return t

    def set_dtype(self, compute_dtype):
        assert compute_dtype in ("bf16", "f32")
        self.cdt = compute_dtype
        self.dt = BF16 if compute_dtype == "bf16" else F32
        self.tdt = torch.bfloat16 if compute_dtype == "bf16" else torch.float32
        self._wkey = None
        self._packs = None

    # ------------------------------------------------------------------ weights
    def _version_key(self):
        return (self.cdt, sum(int(v._version) for v in self.p.values()), id(self))

    def prepare(self, force=False):
        """Repack / cast all fp32 parameters into kernel layouts (cached until params change).

        The packed buffers are allocated once; every refresh (after each optimizer step) is two
        launches of ``s3od_repack_multi`` -- one for the compute-dtype weights, one for the fp32
        fused bias vectors -- instead of ~100 per-tensor repacks and torch copies."""
        key = self._version_key()
        if not force and key == self._wkey:
            return
        ptrs = tuple(v.data_ptr() for v in self.p.values())
        if getattr(self, "_packs", None) is None or self._packs["ptrs"] != ptrs or self._packs["dt"] != self.dt:
            self._build_packs(ptrs)
        L, st = lib(), stream()
        L.phase = "prepare"
        for dt, tab in self._packs["tabs"]:
            L("s3od_repack_multi", dt, tab["tab"], tab["ct"], tab["co"], tab["n"], self._REPACK_CHUNK, st)
        L.phase = None
        self._wkey = key

    _REPACK_CHUNK = 16384

    def _build_packs(self, ptrs):
        """Allocate the kernel-layout buffers and the device tables that fill them from the masters."""
        P, T = self.p, self.tdt
        dev = next(iter(P.values())).device
        D, MLP, nm = self.D, self.MLP, self.nm
        ents = {self.dt: [], F32: []}          # dtype -> [(src, dst, dst_offset, O, I, KHW)]
        w = {}

        def pack(name, O, I, KH=1, KW=1, dst=None, off=0):
            if dst is None:
                dst = torch.empty((O, KH, KW, I), dtype=T, device=dev)
            ents[self.dt].append((P[name], dst, off, O, I, KH * KW, 0, 0))
            return dst

        def pack_dgrad(name, O, I, dst, off, ld, KHW=9, mode=1):
            """[I][3][3][ld] transposed + tap-reversed copy (column off..off+O): the weight of the
            stride-1 3x3 conv's data gradient run as a forward conv (s3od_conv_dgrad's wT); mode 2: transposed
            without the tap reversal."""
            ents[self.dt].append((P[name], dst, off, O, I, KHW, mode, ld))

        def copy32(name, dst, off, n):
            ents[F32].append((P[name], dst, off, n, 1, 1, 0, 0))

        e = "encoder.embeddings."
        w["pe"] = pack(e + "patch_embeddings.weight", D, 3 * 16 * 16)
        for i in range(self.last):
            p = f"encoder.model.layer.{i}."
            qkv = torch.empty((3 * D, D), dtype=T, device=dev)
            for j, nme in enumerate(("q_proj", "k_proj", "v_proj")):
                pack(p + f"attention.{nme}.weight", D, D, dst=qkv, off=j * D * D)
            w[f"qkv{i}"] = qkv
            bq = torch.zeros(3 * D, dtype=torch.float32, device=dev)      # k_proj has no bias (key_bias=False)
            copy32(p + "attention.q_proj.bias", bq, 0, D)
            copy32(p + "attention.v_proj.bias", bq, 2 * D, D)
            w[f"bqkv{i}"] = bq
            w[f"o{i}"] = pack(p + "attention.o_proj.weight", D, D)
            w[f"up{i}"] = pack(p + "mlp.up_proj.weight", MLP, D)
            w[f"down{i}"] = pack(p + "mlp.down_proj.weight", D, MLP)
        h = "seg_head."
        for i, c in enumerate(OUT_CH):
            w[f"proj{i}"] = pack(h + f"projects.{i}.weight", c, D)
        w["rs0"] = pack(h + "resize_layers.0.weight", 256, 256, 4, 4)   # ConvT: [Cin_T][Cout_T] = conv view
        w["rs1"] = pack(h + "resize_layers.1.weight", 512, 512, 2, 2)
        w["rs3"] = pack(h + "resize_layers.3.weight", 1024, 1024, 3, 3)
        for i, c in enumerate(OUT_CH):
            w[f"rn{i + 1}"] = pack(h + f"scratch.layer{i + 1}_rn.weight", 256, c, 3, 3)
        for r in (1, 2, 3, 4):
            q = h + f"scratch.refinenet{r}."
            w[f"ref{r}.out"] = pack(q + "out_conv.weight", 256, 256)
            for u in (1, 2):
                for cv in (1, 2):
                    w[f"ref{r}.u{u}.c{cv}"] = pack(q + f"resConfUnit{u}.conv{cv}.weight", 256, 256, 3, 3)
        m = h + "mask_head."
        w["oc1"] = pack(m + "output_conv1.weight", 128, 256, 3, 3)
        w["up2x"] = pack(m + "upsample_2x.0.weight", 128, 64, 4, 4)     # ConvT [128][64][4][4]
        w["c64"] = pack(m + "upsample_2x.2.weight", 64, 64, 3, 3)
        heads = torch.empty((32 * nm, 3, 3, 64), dtype=T, device=dev)
        for k in range(nm):
            pack(m + f"mask_heads.{k}.0.weight", 32, 64, 3, 3, dst=heads, off=k * 32 * 9 * 64)
        w["heads1"] = heads
        if self.dt == BF16:       # data-gradient weights of the 3x3 s1 convs, run as forward convs (bf16 only)
            for r in (1, 2, 3, 4):
                q = h + f"scratch.refinenet{r}."
                for u in (1, 2):
                    for cv in (1, 2):
                        key = f"ref{r}.u{u}.c{cv}T"
                        w[key] = torch.empty((256, 3, 3, 256), dtype=T, device=dev)
                        pack_dgrad(q + f"resConfUnit{u}.conv{cv}.weight", 256, 256, w[key], 0, 256)
            for i, c in enumerate(OUT_CH):
                w[f"rn{i + 1}T"] = torch.empty((c, 3, 3, 256), dtype=T, device=dev)
                pack_dgrad(h + f"scratch.layer{i + 1}_rn.weight", 256, c, w[f"rn{i + 1}T"], 0, 256)
            w["oc1T"] = torch.empty((256, 3, 3, 128), dtype=T, device=dev)
            pack_dgrad(m + "output_conv1.weight", 128, 256, w["oc1T"], 0, 128)
            w["up2xT"] = torch.empty((64, 4, 4, 128), dtype=T, device=dev)       # ConvT sub-pixel kernel weight
            pack_dgrad(m + "upsample_2x.0.weight", 128, 64, w["up2xT"], 0, 128, KHW=16, mode=2)
            w["c64T"] = torch.empty((64, 3, 3, 64), dtype=T, device=dev)
            pack_dgrad(m + "upsample_2x.2.weight", 64, 64, w["c64T"], 0, 64)
            w["heads1T"] = torch.empty((64, 3, 3, 32 * nm), dtype=T, device=dev)
            for k in range(nm):
                pack_dgrad(m + f"mask_heads.{k}.0.weight", 32, 64, w["heads1T"], 32 * k, 32 * nm)
        for key, n, per in (("heads1_b", "0.bias", 32), ("heads2", "2.weight", 32), ("heads2_b", "2.bias", 1)):
            w[key] = torch.empty(per * nm, dtype=torch.float32, device=dev)
            for k in range(nm):
                copy32(m + f"mask_heads.{k}.{n}", w[key], k * per, per)
        tabs = []
        for dt, lst in ents.items():
            rows, ct, co = [], [], []
            for t, (src, dst, off, O, I, KHW, mode, ld) in enumerate(lst):
                rows.append([src.data_ptr(), dst.data_ptr(), O, I, KHW, off, mode, ld])
                for o in range(0, O * I * KHW, self._REPACK_CHUNK):
                    ct.append(t); co.append(o)
            tabs.append((dt, dict(tab=torch.tensor(rows, dtype=torch.int64, device=dev),
                                  ct=torch.tensor(ct, dtype=torch.int32, device=dev),
                                  co=torch.tensor(co, dtype=torch.int64, device=dev), n=len(ct))))
        self.w = w
        self._packs = {"ptrs": ptrs, "dt": self.dt, "tabs": tabs}

    # ------------------------------------------------------------------ helpers
    def _lin(self, x, w, M, N, K, out, bias=None, scale=None, shift=None, act=ACT_NONE, res1=None, res_f32=False,
             out_f32=False, pre=None, row_mode=0, P=0, prefix=0, ldx=None, ldo=None, ldr=None):
        lib()("s3od_linear_fwd", self.dt, M, N, K, x, ldx or K, w, bias, scale, shift, act,
              res1, ldr or N, None, 0, int(res_f32), out, ldo or N, int(out_f32), pre, N,
              row_mode, P, prefix, stream())

    def _conv(self, x, w, B, H, W, Cin, Cout, k, s, p, bias=None, scale=None, shift=None, act=ACT_NONE,
              relu_in=False, res1=None, res2=None, out=None, pre=None, stats=None, colsum=None):
        OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        if out is None:
            out = torch.empty((B, OH, OW, Cout), dtype=self.tdt, device=x.device)
        lib()("s3od_conv_fwd", self.dt, B, H, W, Cin, OH, OW, Cout, k, k, s, p, x, int(relu_in), w,
              bias, scale, shift, act, res1, res2, out, pre, stats, colsum, stream())
        return out

    def _convT(self, x, w, B, IH, IW, Cin_T, Cout_T, k, s, p, bias=None, act=ACT_NONE, out=None, wT=None):
        """ConvTranspose2d forward == conv dgrad with the conv-view weight (no flip); wT: the transposed copy
        [Cout_T][k][k][Cin_T] for the 4x4 s2 sub-pixel kernel (bf16)."""
        OH, OW = (IH - 1) * s - 2 * p + k, (IW - 1) * s - 2 * p + k
        if out is None:
            out = torch.empty((B, OH, OW, Cout_T), dtype=self.tdt, device=x.device)
        lib()("s3od_conv_dgrad", self.dt, B, OH, OW, Cout_T, IH, IW, Cin_T, k, k, s, p, x, w,
              bias, None, None, act, None, None, out, None, None, None, wT, stream())
        return out

    def _bilinear(self, x, B, IH, IW, OH, OW, C):
        y = torch.empty((B, OH, OW, C), dtype=self.tdt, device=x.device)
        lib()("s3od_bilinear_fwd", self.dt, x, y, B, IH, IW, OH, OW, C, stream())
        return y

    # ------------------------------------------------------------------ encoder
    def encoder_forward(self, x, train=False, rope_rescale=None, ctx=None):
        lib().phase = "encoder"
        L, P, W8, dt, T = lib(), self.p, self.w, self.dt, self.tdt
        D, H, MLP = self.D, self.H, self.MLP
        st = stream()
        B, _, Hh, Ww = x.shape
        ph, pw = Hh // 16, Ww // 16
        NP = ph * pw
        Nt = NP + 1 + NREG
        M = B * Nt
        dev = x.device
        cs = _E(None, (NP, 64), torch.float32, dev)
        sn = _E(None, (NP, 64), torch.float32, dev)
        L("s3od_rope_table", cs, sn, ph, pw, float(rope_rescale) if (train and rope_rescale) else -1.0, st)
        cols = _E(None, (B * NP, 768), T, dev)          # 3 x 16 x 16 patch pixels
        L("s3od_patch_im2col", dt, x, cols, B, Hh, Ww, st)
        xs = _E(None, (B, Nt, D), torch.float32, dev)
        e = "encoder.embeddings."
        self._lin(cols, W8["pe"], B * NP, D, 768, xs, bias=P[e + "patch_embeddings.bias"], out_f32=True,
                  row_mode=1, P=NP, prefix=1 + NREG)
        L("s3od_token_prefix", xs, P[e + "cls_token"], P[e + "register_tokens"], B, Nt, D, st)
        if ctx is not None:
            ctx.t.update(cols=cols, cos=cs, sin=sn)
        taps = []
        h1 = _E(None, (M, D), T, dev)
        q = _E(None, (B * H, Nt, 64), T, dev)
        k = torch.empty_like(q)
        v = torch.empty_like(q)
        o = _E(None, (M, D), T, dev)
        a = _E(None, (M, MLP), T, dev)
        for i in range(self.last):
            p = f"encoder.model.layer.{i}."
            if ctx is not None:   # fresh buffers per layer for the backward
                h1 = _E(None, (M, D), T, dev); q = _E(None, (B * H, Nt, 64), T, dev)
                k = torch.empty_like(q); v = torch.empty_like(q); o = _E(None, (M, D), T, dev)
                a = _E(None, (M, MLP), T, dev)
                mean1 = _E(None, (M,), torch.float32, dev); rstd1 = torch.empty_like(mean1)
                mean2 = torch.empty_like(mean1); rstd2 = torch.empty_like(mean1)
                lse = _E(None, (B * H, Nt), torch.float32, dev)
                u1 = _E(None, (M, D), T, dev); u2 = _E(None, (M, D), T, dev)
                hpre = _E(None, (M, MLP), T, dev); h2 = _E(None, (M, D), T, dev)
            else:
                mean1 = rstd1 = mean2 = rstd2 = _E(None, (M,), torch.float32, dev)
                lse = None; u1 = u2 = hpre = None
                h2 = h1
            L("s3od_layernorm_fwd", dt, xs, P[p + "norm1.weight"], P[p + "norm1.bias"], h1, mean1, rstd1, M, D, 1e-5, st)
            L("s3od_qkv_rope_fwd", dt, B, Nt, NP, H, h1, W8[f"qkv{i}"], W8[f"bqkv{i}"], cs, sn, q, k, v, st)
            L("s3od_attn_fwd", dt, q, k, v, o, lse, B, H, Nt, st)
            xm = _E(None, (B, Nt, D), torch.float32, dev)
            self._lin(o, W8[f"o{i}"], M, D, D, xm, bias=P[p + "attention.o_proj.bias"],
                      scale=P[p + "layer_scale1.lambda1"], res1=xs, res_f32=True, out_f32=True, pre=u1)
            L("s3od_layernorm_fwd", dt, xm, P[p + "norm2.weight"], P[p + "norm2.bias"], h2, mean2, rstd2, M, D, 1e-5, st)
            self._lin(h2, W8[f"up{i}"], M, MLP, D, a, bias=P[p + "mlp.up_proj.bias"],
                      act=ACT_GELU_SG if (hpre is not None and dt == BF16) else ACT_GELU, pre=hpre)
            xn = _E(None, (B, Nt, D), torch.float32, dev)
            self._lin(a, W8[f"down{i}"], M, D, MLP, xn, bias=P[p + "mlp.down_proj.bias"],
                      scale=P[p + "layer_scale2.lambda1"], res1=xm, res_f32=True, out_f32=True, pre=u2)
            if ctx is not None:
                ctx.t[f"L{i}"] = dict(x=xs, h1=h1, mean1=mean1, rstd1=rstd1, q=q, k=k, v=v, o=o, lse=lse, u1=u1,
                                      xm=xm, h2=h2, mean2=mean2, rstd2=rstd2, hpre=hpre, a=a, u2=u2)
            xs = xn
            if i + 1 in self.taps:
                tp = _E(None, (B, NP, D), T, dev)
                L("s3od_cast_tap", dt, xs, tp, B, Nt, NP, D, st)
                taps.append(tp)
        return taps, (B, ph, pw, Nt)

    # ------------------------------------------------------------------ decoder
    def _rcu(self, x, r, u, B, h, w, train, ctx, x0=None):
        """ResidualConvUnit (src/s3od/model.py:334-345) [+ x0 for the fusion add]."""
        P, W8 = self.p, self.w
        q = f"seg_head.scratch.refinenet{r}.resConfUnit{u}."
        tag = f"ref{r}.u{u}"
        if not train:
            st = stream()
            s1, t1 = self._bnfold(q + "bn1", st)
            s2, t2 = self._bnfold(q + "bn2", st)
            a1 = self._conv(x, W8[tag + ".c1"], B, h, w, 256, 256, 3, 1, 1, bias=P[q + "conv1.bias"], scale=s1, shift=t1,
                            act=ACT_RELU, relu_in=True)
            return self._conv(a1, W8[tag + ".c2"], B, h, w, 256, 256, 3, 1, 1, bias=P[q + "conv2.bias"], scale=s2,
                              shift=t2, res1=x, res2=x0)
        L, st, dev = lib(), stream(), x.device
        npix = B * h * w
        z1 = self._conv_bn_train(x, W8[tag + ".c1"], B, h, w, P[q + "conv1.bias"], relu_in=True)
        bn1 = self._bn_train(z1["stats"], npix, q + "bn1")
        a1 = torch.empty_like(z1["z"])
        L("s3od_affine_act", self.dt, z1["z"], bn1["scale"], bn1["shift"], 1, None, None, a1, a1.numel(), 256, st)
        z2 = self._conv_bn_train(a1, W8[tag + ".c2"], B, h, w, P[q + "conv2.bias"])
        bn2 = self._bn_train(z2["stats"], npix, q + "bn2")
        out = torch.empty_like(z2["z"])
        L("s3od_affine_act", self.dt, z2["z"], bn2["scale"], bn2["shift"], 0, x, x0, out, out.numel(), 256, st)
        if ctx is not None:   # train-mode BN under no_grad: batch statistics, nothing saved
            ctx.t[tag] = dict(x=x, z1=z1["z"], a1=a1, z2=z2["z"], bn1=bn1, bn2=bn2, h=h, w=w)
        return out

    def _conv_bn_train(self, x, wt, B, h, w, bias, relu_in=False):
        stats = self.zero_ws("bn_stats", NREP * 2 * 256, torch.float64, x.device)   # S3OD_NREP replicas, cleared by s3od_bn_finalize
        z = self._conv(x, wt, B, h, w, 256, 256, 3, 1, 1, bias=bias, relu_in=relu_in, stats=stats)
        return dict(z=z, stats=stats)

    def _bn_train(self, stats, npix, name):
        P, dev = self.p, stats.device
        d = {k: torch.empty(256, dtype=torch.float32, device=dev) for k in ("mean", "rstd", "scale", "shift")}
        lib()("s3od_bn_finalize", stats, npix, P[name + ".weight"], P[name + ".bias"], self.buf[name + ".running_mean"],
              self.buf[name + ".running_var"], 0.1, 1e-5, d["mean"], d["rstd"], d["scale"], d["shift"], 256, stream())
        nbt = self.buf.get(name + ".num_batches_tracked")
        if nbt is not None:
            self._nbt.append(nbt)      # bumped together at the end of the forward (one launch)
        return d

    def _bnfold(self, name, st):
        P = self.p
        s = torch.empty(256, dtype=torch.float32, device=P[name + ".weight"].device)
        t = torch.empty_like(s)
        lib()("s3od_bn_fold", P[name + ".weight"], P[name + ".bias"], self.buf[name + ".running_mean"],
              self.buf[name + ".running_var"], 1e-5, s, t, 256, st)
        return s, t

    def _fusion(self, r, x0, x1, B, h, w, oh, ow, train, ctx, pre_resize=None):
        """FeatureFusionBlock (src/s3od/model.py:383-405). out_conv (1x1, bias) runs before the
        bilinear resize: both are linear and bilinear weights sum to one, so the order commutes.
        pre_resize: a list that receives the tensor before the resize (the classifier's pooled input)."""
        P, W8 = self.p, self.w
        s = x0 if x1 is None else self._rcu(x1, r, 1, B, h, w, train, ctx, x0=x0)
        s = self._rcu(s, r, 2, B, h, w, train, ctx)
        q = f"seg_head.scratch.refinenet{r}."
        c = torch.empty_like(s)
        self._lin(s, W8[f"ref{r}.out"], B * h * w, 256, 256, c, bias=P[q + "out_conv.bias"])
        if ctx is not None:
            ctx.t[f"ref{r}"] = dict(s=s, h=h, w=w, oh=oh, ow=ow)
        if pre_resize is not None:
            pre_resize.append(c)
        return self._bilinear(c, B, h, w, oh, ow, 256)

    def decoder_forward(self, taps, B, ph, pw, train=False, ctx=None):
        lib().phase = "decoder"
        L, P, W8, dt = lib(), self.p, self.w, self.dt
        st = stream()
        h = "seg_head."
        dev = taps[0].device
        NP = ph * pw
        proj = []
        for i, c in enumerate(OUT_CH):
            y = torch.empty((B, ph, pw, c), dtype=self.tdt, device=dev)
            self._lin(taps[i], W8[f"proj{i}"], B * NP, c, self.D, y, bias=P[h + f"projects.{i}.bias"])
            proj.append(y)
        f0 = self._convT(proj[0], W8["rs0"], B, ph, pw, 256, 256, 4, 4, 0, bias=P[h + "resize_layers.0.bias"])
        f1 = self._convT(proj[1], W8["rs1"], B, ph, pw, 512, 512, 2, 2, 0, bias=P[h + "resize_layers.1.bias"])
        f2 = proj[2]
        f3 = self._conv(proj[3], W8["rs3"], B, ph, pw, 1024, 1024, 3, 2, 1, bias=P[h + "resize_layers.3.bias"])
        feats = [f0, f1, f2, f3]
        dims = [(f.shape[1], f.shape[2]) for f in feats]
        rn = [self._conv(f, W8[f"rn{i + 1}"], B, dims[i][0], dims[i][1], f.shape[3], 256, 3, 1, 1) for i, f in enumerate(feats)]
        if ctx is not None:
            ctx.t["dec"] = dict(taps=taps, proj=proj, feats=feats, rn=rn, dims=dims)
        p4 = self._fusion(4, rn[3], None, B, *dims[3], *dims[2], train, ctx)
        p3 = self._fusion(3, p4, rn[2], B, *dims[2], *dims[1], train, ctx)
        p2 = self._fusion(2, p3, rn[1], B, *dims[1], *dims[0], train, ctx)
        c1 = []
        p1 = self._fusion(1, p2, rn[0], B, *dims[0], 2 * dims[0][0], 2 * dims[0][1], train, ctx, pre_resize=c1)
        H1, W1 = p1.shape[1], p1.shape[2]
        # classifier head: AdaptiveAvgPool2d(1) -> Linear -> ReLU -> Linear.  The mean of p1 is taken over the
        # tensor BEFORE refinenet1's 2x bilinear resize (align_corners=False): every source pixel's weights over
        # the 4x outputs sum to 4 (edge rows / columns included: clamped taps add up to the same 2 per axis), so
        # mean(up2(c)) = mean(c) exactly in real arithmetic, read from a 4x smaller tensor (C5: 2.2 -> 0.55 GB)
        pooled = torch.empty((B, 256), dtype=torch.float32, device=dev)
        src, hw = (c1[0], dims[0][0] * dims[0][1]) if os.environ.get("S3OD_POOL_PRE", "1") != "0" else (p1, H1 * W1)
        part = torch.empty((B, -(-hw // 1024), 256), dtype=torch.float32, device=dev)   # per-1024-pixel partial sums
        L("s3od_avgpool", dt, src, pooled, part, B, hw, 256, st)
        hid = torch.empty((B, 64), dtype=torch.float32, device=dev)
        nm = self.nm
        iou = torch.empty((B, nm), dtype=torch.float32, device=dev)
        L("s3od_iou_head_fwd", pooled, P[h + "classifier_head.2.weight"], P[h + "classifier_head.2.bias"],
          P[h + "classifier_head.4.weight"], P[h + "classifier_head.4.bias"], hid, iou, B, nm, st)
        # mask head (src/s3od/model.py:455-467)
        m = h + "mask_head."
        oc1 = self._conv(p1, W8["oc1"], B, H1, W1, 256, 128, 3, 1, 1, bias=P[m + "output_conv1.bias"])
        up = self._convT(oc1, W8["up2x"], B, H1, W1, 128, 64, 4, 2, 1, bias=P[m + "upsample_2x.0.bias"], act=ACT_RELU,
                         wT=W8.get("up2xT"))
        HH, WW = up.shape[1], up.shape[2]
        c64 = self._conv(up, W8["c64"], B, HH, WW, 64, 64, 3, 1, 1, bias=P[m + "upsample_2x.2.bias"], act=ACT_RELU)
        # F.interpolate(size=(16ph,16pw), antialias=True) is an exact identity here (HH == 16*ph)
        assert HH == 16 * ph and WW == 16 * pw
        logits = torch.empty((B, nm, HH, WW), dtype=torch.float32, device=dev)
        hsave = torch.empty((B * HH * WW, 32 * nm), dtype=self.tdt, device=dev) if ctx is not None else None
        L("s3od_mask_heads_fwd", dt, B, HH, WW, nm, c64, W8["heads1"], W8["heads1_b"], W8["heads2"], W8["heads2_b"],
          logits, hsave, st)
        if ctx is not None:
            ctx.t["head"] = dict(p1=p1, pooled=pooled, hid=hid, oc1=oc1, up=up, c64=c64, hsave=hsave)
        lib().phase = None
        return {"pred_masks": logits, "pred_iou": iou, "features": p1.permute(0, 3, 1, 2)}

    # ------------------------------------------------------------------ full forward
    def _invalidate(self):
        """After a failed call: the persistent zero workspaces may hold partial sums of kernels whose
        clearing reader never ran, and BN counter bumps may be queued for a forward that did not finish.
        Drop both, so the next call allocates fresh zeros and bumps only its own counters."""
        self._zpool = {}
        self._nbt = []
        self._wg = DPTEngine._wg

    def forward(self, x, train=False, rope_rescale=None, ctx: Ctx | None = None):
        """x: [B,3,H,W] fp32 CUDA (normalised image).  Returns the reference output dict."""
        self._nbt = []
        try:
            return self._forward(x, train, rope_rescale, ctx)
        except BaseException:
            self._invalidate()
            raise

    def _forward(self, x, train, rope_rescale, ctx):
        if x.dtype != torch.float32:
            x = x.float()
        Hh, Ww = x.shape[2], x.shape[3]
        if Hh % 16 or Ww % 16:   # the stride-16 patch conv never reads the trailing rows / columns
            x = x[:, :, :16 * (Hh // 16), :16 * (Ww // 16)]
        x = x.contiguous()
        self.prepare()
        taps, (B, ph, pw, Nt) = self.encoder_forward(x, train, rope_rescale, ctx)
        if ctx is not None:
            ctx.B, ctx.H, ctx.W, ctx.ph, ctx.pw = B, x.shape[2], x.shape[3], ph, pw
        out = self.decoder_forward(taps, B, ph, pw, train, ctx)
        if self._nbt:
            torch._foreach_add_(self._nbt, 1)
            self._nbt = []
        return out

    # ================================================================== backward
    def _colsum(self, a, M, N, out, lda=None):
        """Bias gradient out += column sums of a [M, N]: two fixed-order passes through a caller-owned partial-sum
        buffer (the library's own size query; allocated on the calling stream, so the caching allocator orders its
        reuse behind this stream)."""
        key = ("colsum", M, N)
        nb = self._slab_need.get(key)
        if nb is None:
            n = ctypes.c_long(0)
            lib()("s3od_colsum_ws", M, N, ctypes.addressof(n))
            nb = self._slab_need[key] = int(n.value)
        ws = torch.empty(max(nb // 4, 1), dtype=torch.float32, device=out.device)
        lib()("s3od_colsum", self.dt, a, lda or N, M, N, out, ws, nb, stream())

    def _slab(self, entry, key, *args):
        """Caller-owned split-K slab workspace for a weight-gradient entry (the C ABI never allocates): sized by the
        library's own query (s3od_linear_wgrad_ws / s3od_conv_wgrad_ws; cached per shape), one buffer per stream --
        calls on one stream run in order, and the main and side streams both issue weight gradients.  Allocated
        under the stream that uses it, so the caching allocator orders any later reuse behind that stream."""
        nb = self._slab_need.get(key)
        if nb is None:
            n = ctypes.c_long(0)
            lib()(entry, *args, ctypes.addressof(n))
            nb = self._slab_need[key] = int(n.value)
        if nb == 0:
            return None, 0
        st = torch.cuda.current_stream()
        t = self._slabs.get(st.cuda_stream)
        if t is None or t.numel() * 4 < nb:
            t = self._slabs[st.cuda_stream] = torch.empty(nb // 4, dtype=torch.float32, device=st.device)
        return t, t.numel() * 4

    def _wgrad_lin(self, dy, x, Nout, Kin, rows, dw, lddy=None, ldx=None):
        slab, nb = self._slab("s3od_linear_wgrad_ws", ("lin", self.dt, Nout, Kin, rows), self.dt, Nout, Kin, rows, 0)
        lib()("s3od_linear_wgrad", self.dt, Nout, Kin, rows, dy, lddy or Nout, x, ldx or Kin, dw, 0, slab, nb, stream())

    def _dgrad_lin(self, dy, w, M, N, K, out, act=ACT_NONE, aux=None, out_f32=False, row_mode=0, P=0, prefix=0, ldaux=None,
                   colsum=None):
        lib()("s3od_linear_dgrad", self.dt, M, N, K, dy, K, w, act, aux, ldaux or N, out, N, int(out_f32),
              row_mode, P, prefix, colsum, stream())

    def _wgrad_conv(self, dy, x, B, H, W, Cin, OH, OW, Cout, k, s, p, dw, relu_x=False):
        # taps > 1: fp32 workspace in the GEMM's [Cout][tap][Cin] layout (contiguous split-K atomics), zero between calls
        ws = self.zero_ws("wgrad", Cout * k * k * Cin, torch.float32, dy.device) if k > 1 else None
        slab, nb = self._slab("s3od_conv_wgrad_ws", ("conv", self.dt, B, H, W, Cin, OH, OW, Cout, k, s, p),
                              self.dt, B, H, W, Cin, OH, OW, Cout, k, k, s, p, 0)
        lib()("s3od_conv_wgrad", self.dt, B, H, W, Cin, OH, OW, Cout, k, k, s, p, dy, x, int(relu_x), dw, ws, 0, slab, nb,
              stream())

    def _dgrad_conv(self, dy, w, B, H, W, Cin, OH, OW, Cout, k, s, p, act=ACT_NONE, res1=None, out=None, colsum=None,
                    wT=None):
        """dx [B,H,W,Cin] of a conv whose output grid is OH x OW with Cout channels (colsum: += column sums of dx;
        wT: the transposed tap-reversed weight of a 3x3 s1 conv -> the halo-tile kernel)."""
        if out is None:
            out = torch.empty((B, H, W, Cin), dtype=self.tdt, device=dy.device)
        lib()("s3od_conv_dgrad", self.dt, B, H, W, Cin, OH, OW, Cout, k, k, s, p, dy, w, None, None, None, act, res1,
              None, out, None, None, colsum, wT, stream())
        return out

    def _dgrad_conv_res(self, dy, w, B, H, W, C, act, res1, res2, wT=None):
        """3x3 s1 dgrad with RELU_BWD mask (res1 = the un-ReLU'd input) plus a residual gradient res2."""
        out = torch.empty((B, H, W, C), dtype=self.tdt, device=dy.device)
        lib()("s3od_conv_dgrad", self.dt, B, H, W, C, H, W, C, 3, 3, 1, 1, dy, w, None, None, None, act, res1,
              res2, out, None, None, None, wT, stream())
        return out

    def _rcu_bwd(self, d_out, r, u, B, ctx, G):
        """Backward of a train-mode ResidualConvUnit; returns d(input) (including the skip path)."""
        L, P, W8 = lib(), self.p, self.w
        st = stream()
        q = f"seg_head.scratch.refinenet{r}.resConfUnit{u}."
        tag = f"ref{r}.u{u}"
        c = ctx.t[tag]
        h, w = c["h"], c["w"]
        npix = B * h * w
        dev = d_out.device
        sums = self.zero_ws("bn_sums", NREP * 3 * 256, torch.float64, dev)   # S3OD_NREP replicas, zero between calls
        dz2 = torch.empty_like(d_out)
        L("s3od_bn_bwd", self.dt, d_out, c["z2"], None, c["bn2"]["mean"], c["bn2"]["rstd"], P[q + "bn2.weight"], sums, dz2,
          G[q + "bn2.weight"], G[q + "bn2.bias"], G[q + "conv2.bias"], npix, 256, st)
        self._wg(lambda: self._wgrad_conv(dz2, c["a1"], B, h, w, 256, h, w, 256, 3, 1, 1, G[q + "conv2.weight"]),
                 dz2, c["a1"])
        da1 = self._dgrad_conv(dz2, W8[tag + ".c2"], B, h, w, 256, h, w, 256, 3, 1, 1, wT=W8.get(tag + ".c2T"))
        dz1 = torch.empty_like(d_out)
        # ReLU mask recomputed from z1 and bn1's scale/shift (bit-identical to a1 > 0): a1 is not read
        L("s3od_bn_relu_bwd", self.dt, da1, c["z1"], c["bn1"]["scale"], c["bn1"]["shift"], c["bn1"]["mean"],
          c["bn1"]["rstd"], P[q + "bn1.weight"], sums, dz1,
          G[q + "bn1.weight"], G[q + "bn1.bias"], G[q + "conv1.bias"], npix, 256, st)
        self._wg(lambda: self._wgrad_conv(dz1, c["x"], B, h, w, 256, h, w, 256, 3, 1, 1, G[q + "conv1.weight"], relu_x=True),
                 dz1, c["x"])
        return self._dgrad_conv_res(dz1, W8[tag + ".c1"], B, h, w, 256, ACT_RELU_BWD, c["x"], d_out, wT=W8.get(tag + ".c1T"))

    def _fusion_bwd(self, r, d_p, B, ctx, G, bcast=None, two_inputs=True):
        """Backward of FeatureFusionBlock r. Returns (d_x0, d_x1) (d_x1 None for refinenet4)."""
        L, P, W8 = lib(), self.p, self.w
        c = ctx.t[f"ref{r}"]
        h, w, oh, ow = c["h"], c["w"], c["oh"], c["ow"]
        dev = d_p.device
        dc = torch.empty((B, h, w, 256), dtype=self.tdt, device=dev)
        L("s3od_bilinear_bwd", self.dt, d_p, bcast, dc, B, h, w, oh, ow, 256, stream())
        q = f"seg_head.scratch.refinenet{r}."
        npix = B * h * w
        self._colsum(dc, npix, 256, G[q + "out_conv.bias"])
        self._wg(lambda: self._wgrad_lin(dc, c["s"], 256, 256, npix, G[q + "out_conv.weight"]), dc, c["s"])
        ds2 = torch.empty_like(dc)
        self._dgrad_lin(dc, W8[f"ref{r}.out"], npix, 256, 256, ds2)
        ds = self._rcu_bwd(ds2, r, 2, B, ctx, G)
        if not two_inputs:
            return ds, None
        dx1 = self._rcu_bwd(ds, r, 1, B, ctx, G)
        return ds, dx1

    _wg = staticmethod(lambda fn, *ts: fn())     # weight-gradient runner (decoder_backward installs the side-stream one)

    def decoder_backward(self, ctx, d_logits, d_iou, G, d_feat=None):
        lib().phase = "decoder"
        L, P, W8, dt = lib(), self.p, self.w, self.dt
        st = stream()
        # weight gradients on the side stream (as in the encoder backward), concurrent with the data-gradient chain:
        # the decoder's many small-map convs (64^2, 32^2 at bs 16: a fraction of a round of tiles) and the wgrads'
        # tails then share the CUs.  Each wgrad only reads its operands; they are marked as used on the side stream
        # (record_stream), so the caching allocator keeps them until it has run.  S3OD_DEC_SIDE=0 (or
        # S3OD_BWD_SIDE=0): inline on the main stream.
        main = torch.cuda.current_stream(d_logits.device)
        side = (self._side_stream(d_logits.device) if os.environ.get("S3OD_BWD_SIDE", "1") != "0"
                and os.environ.get("S3OD_DEC_SIDE", "1") != "0" else None)
        self._dec_side = side

        def wg(fn, *ts):
            if side is None:
                return fn()
            e = torch.cuda.Event()
            e.record(main)
            side.wait_event(e)
            with torch.cuda.stream(side):
                fn()
            for t in ts:
                t.record_stream(side)
        self._wg = wg
        B, ph, pw = ctx.B, ctx.ph, ctx.pw
        hd = ctx.t["head"]
        h = "seg_head."
        m = h + "mask_head."
        dev = d_logits.device
        p1, c64, up, oc1 = hd["p1"], hd["c64"], hd["up"], hd["oc1"]
        H1, W1 = p1.shape[1], p1.shape[2]
        HH, WW = up.shape[1], up.shape[2]
        npx = B * HH * WW
        # ---- the mask heads (fused, N = 32 * n_masks)
        nm = self.nm
        dh = torch.empty((npx, 32 * nm), dtype=self.tdt, device=dev)
        L("s3od_mask_heads_bwd", dt, d_logits.contiguous(), hd["hsave"], W8["heads2"], dh, G["heads2_w"], G["heads2_b"],
          G["heads1_b"], B, HH * WW, nm, st)
        self._wg(lambda: self._wgrad_conv(dh, c64, B, HH, WW, 64, HH, WW, 32 * nm, 3, 1, 1, G["heads1_w"]), dh, c64)
        # (bias gradients are column sums fused into the epilogue that produces each gradient)
        d64 = self._dgrad_conv(dh, W8["heads1"], B, HH, WW, 64, HH, WW, 32 * nm, 3, 1, 1, act=ACT_RELU_BWD, res1=c64,
                               colsum=G[m + "upsample_2x.2.bias"], wT=W8.get("heads1T"))
        # ---- upsample_2x.2 conv 64->64 + ReLU
        self._wg(lambda: self._wgrad_conv(d64, up, B, HH, WW, 64, HH, WW, 64, 3, 1, 1, G[m + "upsample_2x.2.weight"]),
                 d64, up)
        dup = self._dgrad_conv(d64, W8["c64"], B, HH, WW, 64, HH, WW, 64, 3, 1, 1, act=ACT_RELU_BWD, res1=up,
                               colsum=G[m + "upsample_2x.0.bias"], wT=W8.get("c64T"))
        # ---- upsample_2x.0 ConvTranspose 128->64 k4 s2 p1 + ReLU (conv view: Y=oc1 grid, X=up grid)
        self._wg(lambda: self._wgrad_conv(oc1, dup, B, HH, WW, 64, H1, W1, 128, 4, 2, 1, G[m + "upsample_2x.0.weight"]),
                 oc1, dup)
        doc1 = self._conv(dup, W8["up2x"], B, HH, WW, 64, 128, 4, 2, 1, colsum=G[m + "output_conv1.bias"])
        # ---- output_conv1 3x3 256->128
        self._wg(lambda: self._wgrad_conv(doc1, p1, B, H1, W1, 256, H1, W1, 128, 3, 1, 1, G[m + "output_conv1.weight"]),
                 doc1, p1)
        dp1 = self._dgrad_conv(doc1, W8["oc1"], B, H1, W1, 256, H1, W1, 128, 3, 1, 1, wT=W8.get("oc1T"))
        if d_feat is not None:     # gradient of the returned features (= path_1, NCHW view)
            dp1.add_(d_feat.permute(0, 2, 3, 1).to(dp1.dtype))
        # ---- classifier head -> broadcast gradient onto path_1 (folded into the bilinear backward)
        dpix = torch.empty((B, 256), dtype=torch.float32, device=dev)
        L("s3od_iou_head_bwd", hd["pooled"], hd["hid"], P[h + "classifier_head.2.weight"], P[h + "classifier_head.4.weight"],
          d_iou.contiguous(), G[h + "classifier_head.2.weight"], G[h + "classifier_head.2.bias"],
          G[h + "classifier_head.4.weight"], G[h + "classifier_head.4.bias"], dpix, B, H1 * W1, nm, st)
        # ---- refinenets
        dp2, drn1 = self._fusion_bwd(1, dp1, B, ctx, G, bcast=dpix)
        dp3, drn2 = self._fusion_bwd(2, dp2, B, ctx, G)
        dp4, drn3 = self._fusion_bwd(3, dp3, B, ctx, G)
        drn4, _ = self._fusion_bwd(4, dp4, B, ctx, G, two_inputs=False)
        dec = ctx.t["dec"]
        feats, dims = dec["feats"], dec["dims"]
        drn = [drn1, drn2, drn3, drn4]
        dfeat = []
        # the feature gradient's column sums: resize_layers.{0,1,3}.bias; feature 2 is projects.2's output
        fbias = [h + "resize_layers.0.bias", h + "resize_layers.1.bias", h + "projects.2.bias", h + "resize_layers.3.bias"]
        for i, f in enumerate(feats):
            hh, ww = dims[i]
            C = f.shape[3]
            self._wg(lambda: self._wgrad_conv(drn[i], f, B, hh, ww, C, hh, ww, 256, 3, 1, 1, G[h + f"scratch.layer{i + 1}_rn.weight"]),
                     drn[i], f)
            dfeat.append(self._dgrad_conv(drn[i], W8[f"rn{i + 1}"], B, hh, ww, C, hh, ww, 256, 3, 1, 1, colsum=G[fbias[i]],
                                          wT=W8.get(f"rn{i + 1}T")))
        proj = dec["proj"]
        dproj = [None] * 4
        # resize0: ConvT 256 k4 s4 (conv view: Y = proj0 grid, X = f0 grid)
        self._wg(lambda: self._wgrad_conv(proj[0], dfeat[0], B, dims[0][0], dims[0][1], 256, ph, pw, 256, 4, 4, 0, G[h + "resize_layers.0.weight"]),
                 proj[0], dfeat[0])
        dproj[0] = self._conv(dfeat[0], W8["rs0"], B, dims[0][0], dims[0][1], 256, 256, 4, 4, 0, colsum=G[h + "projects.0.bias"])
        self._wg(lambda: self._wgrad_conv(proj[1], dfeat[1], B, dims[1][0], dims[1][1], 512, ph, pw, 512, 2, 2, 0, G[h + "resize_layers.1.weight"]),
                 proj[1], dfeat[1])
        dproj[1] = self._conv(dfeat[1], W8["rs1"], B, dims[1][0], dims[1][1], 512, 512, 2, 2, 0, colsum=G[h + "projects.1.bias"])
        dproj[2] = dfeat[2]
        self._wg(lambda: self._wgrad_conv(dfeat[3], proj[3], B, ph, pw, 1024, dims[3][0], dims[3][1], 1024, 3, 2, 1, G[h + "resize_layers.3.weight"]),
                 dfeat[3], proj[3])
        dproj[3] = self._dgrad_conv(dfeat[3], W8["rs3"], B, ph, pw, 1024, dims[3][0], dims[3][1], 1024, 3, 2, 1,
                                    colsum=G[h + "projects.3.bias"])
        # projects (1x1, bias) -> tap gradients
        NP = ph * pw
        dtaps = []
        for i, c in enumerate(OUT_CH):
            self._wg(lambda: self._wgrad_lin(dproj[i], dec["taps"][i], c, self.D, B * NP, G[h + f"projects.{i}.weight"]),
                     dproj[i], dec["taps"][i])
            dtaps.append((dproj[i], c))
        lib().phase = None
        return dtaps

    def encoder_backward(self, ctx, dtaps, G):
        lib().phase = "encoder"
        L, P, W8, dt, T = lib(), self.p, self.w, self.dt, self.tdt
        D, H, MLP = self.D, self.H, self.MLP
        st = stream()
        B, ph, pw = ctx.B, ctx.ph, ctx.pw
        NP = ph * pw
        Nt = NP + 1 + NREG
        M = B * Nt
        dev = dtaps[0][0].device
        # the first tap gradient writes the patch rows; only the prefix rows (cls + registers) need zeros
        dx = torch.empty((B, Nt, D), dtype=torch.float32, device=dev)
        dx[:, :1 + NREG].zero_()
        first_tap = True
        tap_of = {t: j for j, t in enumerate(self.taps)}
        # weight gradients run on a side stream, concurrently with the data-gradient chain on the main stream: each
        # wgrad only READS its two operands, so it may trail the chain; the chain waits for the reader's event before
        # it overwrites an operand buffer one layer later (in practice long done).  Two single-pipeline kernels then
        # share the CUs: one's store-bound epilogue / tail overlaps the other's MFMA main loop.
        main = torch.cuda.current_stream(dev)
        side = self._side_stream(dev) if os.environ.get("S3OD_BWD_SIDE", "1") != "0" else main   # (A/B: 0 = one stream)
        ev_free = {}                                   # buffer -> event after its last side-stream reader

        def on_side(fn, *bufs):
            e = torch.cuda.Event()
            e.record(main)
            side.wait_event(e)
            with torch.cuda.stream(side):
                fn()
            for b in bufs:
                f = torch.cuda.Event()
                f.record(side)
                ev_free[b] = f

        def claim(b):                                  # before the main stream overwrites buffer b
            f = ev_free.pop(b, None)
            if f is not None:
                main.wait_event(f)

        du = _E(None, (M, D), T, dev)
        du2 = _E(None, (M, D), T, dev)
        dhp = _E(None, (M, MLP), T, dev)
        dh = _E(None, (M, D), T, dev)
        dxm = _E(None, (B, Nt, D), torch.float32, dev)
        dxi = _E(None, (B, Nt, D), torch.float32, dev)
        dqkv = _E(None, (M, 3 * D), T, dev)
        delta = _E(None, (B * H, Nt), torch.float32, dev)
        qv_ws = self.zero_ws("qv", NREP * 2 * D, torch.float32, dev)     # S3OD_NREP replicas of the q/v bias partials
        red_ws = self.zero_ws("red", NREP * 2 * D, torch.float32, dev)   # same, for LayerNorm / LayerScale parameter grads
        red2_ws = self.zero_ws("red2", NREP * 2 * D, torch.float32, dev)  # the LayerScale half of the fused LN + LS backward
        ls_done = False       # the layer's layer_scale2 backward already ran inside the layer above's norm1 backward
        for i in reversed(range(self.last)):
            if i + 1 in tap_of:
                dp, c = dtaps[tap_of[i + 1]]
                # dx[prefix-skipped rows] += dproj @ W_proj   (in-place accumulate, fp32)
                self._dgrad_lin(dp, W8[f"proj{tap_of[i + 1]}"], B * NP, D, c, dx, aux=None if first_tap else dx,
                                out_f32=True, row_mode=1, P=NP, prefix=1 + NREG, ldaux=D)
                first_tap = False
            p = f"encoder.model.layer.{i}."
            s = ctx.t[f"L{i}"]
            # ---- MLP half
            if not ls_done:
                claim("du")
                L("s3od_layerscale_bwd", dt, dx, s["u2"], P[p + "layer_scale2.lambda1"], du, G[p + "layer_scale2.lambda1"],
                  G[p + "mlp.down_proj.bias"], red_ws, M, D, st)
            on_side(lambda: self._wgrad_lin(du, s["a"], D, MLP, M, G[p + "mlp.down_proj.weight"]), "du")
            claim("dhp")
            self._dgrad_lin(du, W8[f"down{i}"], M, MLP, D, dhp, act=ACT_MUL if dt == BF16 else ACT_GELU_BWD, aux=s["hpre"],
                            colsum=G[p + "mlp.up_proj.bias"])
            on_side(lambda: self._wgrad_lin(dhp, s["h2"], MLP, D, M, G[p + "mlp.up_proj.weight"]), "dhp")
            self._dgrad_lin(dhp, W8[f"up{i}"], M, D, MLP, dh)
            # norm2 backward fused with the attention half's layer_scale1 backward (which reads its dxm)
            claim("du2")
            L("s3od_layernorm_ls_bwd", dt, dh, s["xm"], s["mean2"], s["rstd2"], P[p + "norm2.weight"], dx, dxm,
              G[p + "norm2.weight"], G[p + "norm2.bias"], red_ws, s["u1"], P[p + "layer_scale1.lambda1"], du2,
              G[p + "layer_scale1.lambda1"], G[p + "attention.o_proj.bias"], red2_ws, M, D, st)
            # ---- attention half
            on_side(lambda: self._wgrad_lin(du2, s["o"], D, D, M, G[p + "attention.o_proj.weight"]), "du2")
            do = dh
            self._dgrad_lin(du2, W8[f"o{i}"], M, D, D, do)
            # attention backward with the inverse RoPE / q scale / q,v bias sums fused into its stores
            claim("dqkv")
            L("s3od_attn_bwd_qkv", dt, s["q"], s["k"], s["v"], s["o"], do, s["lse"], delta, ctx.t["cos"], ctx.t["sin"], NP,
              dqkv, G[p + "attention.q_proj.bias"], G[p + "attention.v_proj.bias"], qv_ws, B, H, Nt, st)
            on_side(lambda: self._wgrad_lin(dqkv, s["h1"], 3 * D, D, M, G[f"qkv_w{i}"]), "dqkv")
            dh1 = dh
            self._dgrad_lin(dqkv, W8[f"qkv{i}"], M, D, 3 * D, dh1)
            # norm1 backward, fused with layer i-1's layer_scale2 backward unless a tap gradient joins dx in between
            ls_done = i >= 1 and i not in tap_of
            if ls_done:
                q = f"encoder.model.layer.{i - 1}."
                claim("du")
                L("s3od_layernorm_ls_bwd", dt, dh1, s["x"], s["mean1"], s["rstd1"], P[p + "norm1.weight"], dxm, dxi,
                  G[p + "norm1.weight"], G[p + "norm1.bias"], red_ws, ctx.t[f"L{i - 1}"]["u2"], P[q + "layer_scale2.lambda1"],
                  du, G[q + "layer_scale2.lambda1"], G[q + "mlp.down_proj.bias"], red2_ws, M, D, st)
            else:
                L("s3od_layernorm_bwd", dt, dh1, s["x"], s["mean1"], s["rstd1"], P[p + "norm1.weight"], dxm, dxi,
                  G[p + "norm1.weight"], G[p + "norm1.bias"], red_ws, M, D, st)
            dx, dxi = dxi, dx
            if self.grad_hook is not None:
                # the layer's gradients are final once both streams are past it: the hook (the DDP bucket all-reduce)
                # is issued from the side stream after it has joined the main stream
                on_side(lambda: self.grad_hook(f"layer{i}"))
        # ---- embeddings
        e = "encoder.embeddings."
        L("s3od_token_prefix_bwd", dx, G[e + "cls_token"], G[e + "register_tokens"], B, Nt, D, st)
        dpatch = _E(None, (B, NP, D), T, dev)
        L("s3od_cast_tap", dt, dx, dpatch, B, Nt, NP, D, st)
        self._colsum(dpatch, B * NP, D, G[e + "patch_embeddings.bias"])
        self._wgrad_lin(dpatch, ctx.t["cols"], D, 768, B * NP, G[e + "patch_embeddings.weight"])
        main.wait_stream(side)                         # every weight gradient is final on the main stream
        lib().phase = None
        if self.grad_hook is not None:
            self.grad_hook("embeddings")

    grad_hook = None

    def _side_stream(self, dev):
        st = getattr(self, "_side", None)
        if st is None or st.device != dev:
            st = self._side = torch.cuda.Stream(device=dev)
        return st

    def backward(self, ctx: Ctx, d_logits, d_iou, G, d_feat=None):
        """Accumulate parameter gradients into G (name -> fp32 tensor, reference layout; plus the
        fused views 'qkv_w{i}', 'heads1_w', 'heads1_b', 'heads2_w', 'heads2_b').  d_feat: optional
        gradient of the returned ``features`` (NCHW), added to path_1's."""
        try:
            dtaps = self.decoder_backward(ctx, d_logits, d_iou, G, d_feat=d_feat)
            self._wg = DPTEngine._wg
            if self.grad_hook is not None:
                side = self._dec_side
                if side is None:
                    self.grad_hook("seg_head")
                else:     # the decoder's gradients are final once both streams are past it: hook from the side stream
                    e = torch.cuda.Event()
                    e.record(torch.cuda.current_stream(d_logits.device))
                    side.wait_event(e)
                    with torch.cuda.stream(side):
                        self.grad_hook("seg_head")
            self.encoder_backward(ctx, dtaps, G)
        except BaseException:
            # side-stream weight gradients may still read ctx activations / workspaces and add into G: the main
            # stream waits for them before anything is freed (ctx, zero workspaces) or re-used by a retry
            side = getattr(self, "_side", None)
            if side is not None:
                torch.cuda.current_stream(side.device).wait_stream(side)
            self._wg = DPTEngine._wg
            self._invalidate()
            raise
