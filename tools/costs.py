"""Algorithmic cost of each C-ABI call (measurement only: bench.py's roofline / per-class table).

``cost(name, args) -> (kind, amount)`` with kind "mfma" (FLOPs) or "hbm" (bytes), computed from
the call's own arguments (include/s3od_hip.h), i.e. the work the reference's op REQUIRES:

* GEMM-shaped entries: 2*M*N*K of the op they implement (a conv's dgrad / wgrad count the same
  2*B*OH*OW*Cout*Cin*KH*KW as its forward; ConvTranspose forward is a conv dgrad with the conv-view
  grid, so the same formula holds).  Attention forward 4*N^2*64 per (b,h) (QK^T + PV); backward
  SURVEY §8(d)'s convention (training = 3x forward, "flash recompute is not counted"): 2x forward =
  8*N^2*64 (dV = P^T dO, dP = dO V^T, dQ = dS K, dK = dS^T Q).  ``executed(name, args)`` gives what the
  kernels actually issue (14*N^2*64: S in the dK/dV pass, S and dP again in the dQ pass).
* memory-bound entries: mandatory bytes in + out at the storage dtype (each tensor touched once).
"""
from __future__ import annotations

F32, BF16 = 0, 1
D = 768


def _t(dt):
    return 2 if dt == BF16 else 4


def cost(name, a):
    n = name[len("s3od_"):]
    if n == "linear_fwd":
        dt, M, N, K = a[:4]
        return "mfma", 2.0 * M * N * K
    if n == "linear_dgrad":
        dt, M, N, K = a[:4]
        return "mfma", 2.0 * M * N * K
    if n == "linear_wgrad":
        dt, Nout, Kin, rows = a[:4]
        return "mfma", 2.0 * Nout * Kin * rows
    if n == "qkv_rope_fwd":
        dt, B, Nt, P = a[:4]
        return "mfma", 2.0 * B * Nt * D * 3 * D
    if n in ("conv_fwd", "conv_dgrad", "conv_wgrad"):
        dt, B, H, W, Cin, OH, OW, Cout, KH, KW = a[:10]
        return "mfma", 2.0 * B * OH * OW * Cout * Cin * KH * KW
    if n == "mask_heads_fwd":
        dt, B, H, W = a[:4]
        return "mfma", 2.0 * B * H * W * (96 * 64 * 9 + 96)
    if n == "attn_fwd":
        B, H, N = a[6:9]
        return "mfma", 4.0 * B * H * N * N * 64
    if n == "attn_bwd":
        B, H, N = a[11:14]
        return "mfma", 8.0 * B * H * N * N * 64
    if n == "attn_bwd_qkv":
        B, H, N = a[15:18]
        return "mfma", 8.0 * B * H * N * N * 64
    # ---- memory-bound
    if n == "layernorm_fwd":
        dt, M = a[0], a[7]
        return "hbm", M * D * (4 + _t(dt)) + 8.0 * M
    if n == "layernorm_bwd":
        dt, dres, M = a[0], a[6], a[11]
        return "hbm", M * D * (_t(dt) + 4 + 4 + (4 if dres is not None else 0)) + 8.0 * M
    if n == "layernorm_ls_bwd":       # the LayerNorm backward + the LayerScale backward's u read and du write
        dt, dres, M = a[0], a[6], a[17]
        return "hbm", M * D * (_t(dt) + 4 + 4 + (4 if dres is not None else 0) + 2 * _t(dt)) + 8.0 * M
    if n == "layerscale_bwd":
        dt, M = a[0], a[8]
        return "hbm", M * D * (4 + 2 * _t(dt))
    if n == "cast_tap":
        dt, B, Nt, P = a[0], a[3], a[4], a[5]
        return "hbm", B * P * D * (4 + _t(dt))
    if n == "bilinear_fwd" or n == "bilinear_bwd":
        dt = a[0]
        B, IH, IW, OH, OW, C = a[-7:-1]
        return "hbm", B * C * (IH * IW + OH * OW) * _t(dt)
    if n == "affine_act":
        dt, r1, r2, total = a[0], a[5], a[6], a[8]
        return "hbm", total * _t(dt) * (2 + (r1 is not None) + (r2 is not None))
    if n == "bn_bwd":
        dt, yrelu, npix, C = a[0], a[3], a[12], a[13]
        return "hbm", npix * C * _t(dt) * (3 + (yrelu is not None))
    if n == "bn_relu_bwd":   # dy, z read, dz written (the ReLU mask is recomputed from z)
        dt, npix, C = a[0], a[13], a[14]
        return "hbm", npix * C * _t(dt) * 3
    if n == "avgpool":
        dt, B, HW, C = a[0], a[4], a[5], a[6]
        return "hbm", B * HW * C * _t(dt)
    if n == "mask_heads_bwd":
        dt, B, HW = a[0], a[8], a[9]
        return "hbm", B * HW * (3 * 4 + 2 * 96 * _t(dt))
    if n == "mask_loss_fwd":
        B, M, HW = a[3], a[4], a[5]
        return "hbm", B * HW * 4 * (M + 1)
    if n == "mask_loss_bwd":
        B, M, HW = a[8], a[9], a[10]
        return "hbm", B * HW * 4 * (2 * M + 1)
    if n == "qkv_unrope":
        dt, B, Nt = a[0], a[10], a[11]
        return "hbm", 2.0 * 3 * B * Nt * D * _t(dt)
    if n == "colsum":
        dt, M, N = a[0], a[3], a[4]
        return "hbm", M * N * _t(dt)
    if n == "patch_im2col":
        dt, B, H, W = a[0], a[3], a[4], a[5]
        return "hbm", B * 3 * H * W * (4 + _t(dt))
    if n == "repack_weight":
        dt, O, I, KH, KW = a[0], a[3], a[4], a[5], a[6]
        return "hbm", O * I * KH * KW * (4 + _t(dt))
    if n == "adamw_step":
        sizes = a[1]
        total = int(sizes.sum()) if hasattr(sizes, "sum") else 0
        return "hbm", 28.0 * total      # read p, g, m, v; write p, m, v (fp32)
    return "other", 0.0


def executed(name, a):
    """MFMA FLOPs the kernels issue, where that differs from the algorithmic figure (else None)."""
    n = name[len("s3od_"):]
    if n == "attn_bwd":
        B, H, N = a[11:14]
        return 14.0 * B * H * N * N * 64
    if n == "attn_bwd_qkv":
        B, H, N = a[15:18]
        return 14.0 * B * H * N * N * 64
    return None


CLASS = {
    "linear_fwd": "ViT/1x1 linear fwd", "qkv_rope_fwd": "ViT/1x1 linear fwd", "linear_dgrad": "linear dgrad",
    "linear_wgrad": "linear wgrad", "conv_fwd": "conv fwd", "conv_dgrad": "conv dgrad + ConvT fwd",
    "conv_wgrad": "conv wgrad", "mask_heads_fwd": "conv fwd", "attn_fwd": "attention fwd", "attn_bwd": "attention bwd",
    "attn_bwd_qkv": "attention bwd",
}


def klass(name):
    return CLASS.get(name[len("s3od_"):], "memory-bound")
