"""Micro-benchmark of the HBM-bound backward kernels through the C ABI (dev tool, GPU box).
Run under `rocprofv3 --kernel-trace --stats` to split multi-kernel entry points."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd._lib import lib, stream, BF16  # noqa: E402
from tools.gemm_bench import timeit  # noqa: E402


def bn_bwd(npix=16 * 256 * 256, C=256, relu=True):
    dy = torch.randn(npix, C, device="cuda").bfloat16()
    z = torch.randn_like(dy)
    y = torch.randn_like(dy) if relu else None
    mean = torch.zeros(C, device="cuda"); rstd = torch.ones(C, device="cuda"); w = torch.ones(C, device="cuda")
    sums = torch.zeros(32 * 3 * C, dtype=torch.float64, device="cuda")
    dz = torch.empty_like(dy)
    dw, db, dcb = (torch.zeros(C, device="cuda") for _ in range(3))
    f = lambda: lib()("s3od_bn_bwd", BF16, dy, z, y, mean, rstd, w, sums, dz, dw, db, dcb, npix, C, stream())
    t = timeit(f)
    nbytes = npix * C * 2 * ((3 if relu else 2) * 2 + 1)
    print(f"bn_bwd npix={npix} C={C} relu={relu}: {t * 1e6:8.1f} us  {nbytes / t / 1e12:6.2f} TB/s (reduce+apply bytes)")


def bn_relu_bwd(npix=16 * 256 * 256, C=256):
    """BN + ReLU backward with the ReLU mask recomputed from z (s3od_bn_relu_bwd)."""
    dy = torch.randn(npix, C, device="cuda").bfloat16()
    z = torch.randn_like(dy)
    mean = torch.zeros(C, device="cuda"); rstd = torch.ones(C, device="cuda"); w = torch.ones(C, device="cuda")
    sc, sh = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
    sums = torch.zeros(32 * 3 * C, dtype=torch.float64, device="cuda")
    dz = torch.empty_like(dy)
    dw, db, dcb = (torch.zeros(C, device="cuda") for _ in range(3))
    f = lambda: lib()("s3od_bn_relu_bwd", BF16, dy, z, sc, sh, mean, rstd, w, sums, dz, dw, db, dcb, npix, C, stream())
    t = timeit(f)
    nbytes = npix * C * 2 * 5
    print(f"bn_relu_bwd npix={npix} C={C}: {t * 1e6:8.1f} us  {nbytes / t / 1e12:6.2f} TB/s (reduce+apply bytes)")


def unrope(B=16, N=4101):
    dq = torch.randn(B * 12, N, 64, device="cuda").bfloat16()
    dk, dv = torch.randn_like(dq), torch.randn_like(dq)
    cs = torch.randn(N - 5, 64, device="cuda"); sn = torch.randn_like(cs)
    out = torch.empty(B * N, 2304, device="cuda", dtype=torch.bfloat16)
    bq, bv = torch.zeros(768, device="cuda"), torch.zeros(768, device="cuda")
    ws = torch.zeros(32 * 1536, device="cuda")
    f = lambda: lib()("s3od_qkv_unrope", BF16, dq, dk, dv, cs, sn, out, bq, bv, ws, B, N, N - 5, stream())
    t = timeit(f)
    nbytes = 2 * out.numel() * 2
    print(f"qkv_unrope B={B} N={N}: {t * 1e6:8.1f} us  {nbytes / t / 1e12:6.2f} TB/s")


def vit_bwd(M=16 * 4101, D=768):
    """LayerNorm backward (bf16 dy, f32 x / dres / dx) and LayerScale backward at the C3 shape;
    S3OD_LN_RPB / S3OD_LS_RPB select rows per block."""
    dy = torch.randn(M, D, device="cuda").bfloat16()
    x = torch.randn(M, D, device="cuda"); dres = torch.randn_like(x); dx = torch.empty_like(x)
    mean = x.mean(1); rstd = torch.ones(M, device="cuda"); w = torch.ones(D, device="cuda")
    dw, db = torch.zeros(D, device="cuda"), torch.zeros(D, device="cuda")
    ws = torch.zeros(32 * 2 * D, device="cuda")
    t = timeit(lambda: lib()("s3od_layernorm_bwd", BF16, dy, x, mean, rstd, w, dres, dx, dw, db, ws, M, D, stream()))
    nb = M * D * (2 + 4 + 4 + 4)
    print(f"layernorm_bwd M={M} D={D}: {t * 1e6:8.1f} us  {nb / t / 1e12:6.2f} TB/s")
    u = torch.randn(M, D, device="cuda").bfloat16(); du = torch.empty_like(u)
    t = timeit(lambda: lib()("s3od_layerscale_bwd", BF16, x, u, w, du, dw, db, ws, M, D, stream()))
    nb = M * D * (4 + 2 + 2)
    print(f"layerscale_bwd M={M} D={D}: {t * 1e6:8.1f} us  {nb / t / 1e12:6.2f} TB/s")


def copy(n=1 << 28):
    a = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    b = torch.empty_like(a)
    t = timeit(lambda: b.copy_(a))
    print(f"torch copy {n * 2 / 1e6:.0f} MB: {t * 1e6:8.1f} us  {2 * n * 2 / t / 1e12:6.2f} TB/s")


if __name__ == "__main__":
    if sys.argv[1:] == ["bn"]:
        for npix in (16 * 256 * 256, 16 * 128 * 128, 16 * 64 * 64):
            bn_bwd(npix, relu=False)
            bn_relu_bwd(npix)
        sys.exit(0)
    if sys.argv[1:] == ["vit"]:
        vit_bwd()
        sys.exit(0)
    copy()
    bn_bwd(relu=True)
    bn_bwd(relu=False)
    unrope()
