"""GEMM / conv micro-benchmark through the C ABI (dev tool).  python tools/gemm_bench.py"""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd._lib import lib, stream, BF16  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e-3


def lin(M, N, K, out_f32=False):
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    o = torch.empty(M, N, device="cuda", dtype=torch.float32 if out_f32 else torch.bfloat16)
    b = torch.randn(N, device="cuda")
    f = lambda: lib()("s3od_linear_fwd", BF16, M, N, K, x, K, w, b, None, None, 0, None, N, None, 0, 0, o, N, int(out_f32),
                      None, N, 0, 0, 0, stream())
    t = timeit(f)
    print(f"linear fwd M={M} N={N} K={K}: {t * 1e6:8.1f} us  {2 * M * N * K / t / 1e12:7.1f} TF/s")


def dgrad(M, N, K):
    dy = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(K, N, device="cuda").bfloat16()
    o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    f = lambda: lib()("s3od_linear_dgrad", BF16, M, N, K, dy, K, w, 0, None, N, o, N, 0, 0, 0, 0, None, stream())
    t = timeit(f)
    print(f"linear dgrad M={M} N={N} K={K}: {t * 1e6:8.1f} us  {2 * M * N * K / t / 1e12:7.1f} TF/s")


def wgrad(Nout, Kin, rows):
    dy = torch.randn(rows, Nout, device="cuda").bfloat16()
    x = torch.randn(rows, Kin, device="cuda").bfloat16()
    dw = torch.zeros(Nout, Kin, device="cuda")
    f = lambda: lib()("s3od_linear_wgrad", BF16, Nout, Kin, rows, dy, Nout, x, Kin, dw, 0, stream())
    t = timeit(f)
    print(f"linear wgrad N={Nout} K={Kin} rows={rows}: {t * 1e6:8.1f} us  {2 * Nout * Kin * rows / t / 1e12:7.1f} TF/s")


def conv(B, H, W, Cin, Cout, k=3):
    x = torch.randn(B, H, W, Cin, device="cuda").bfloat16()
    w = torch.randn(Cout, k, k, Cin, device="cuda").bfloat16()
    o = torch.empty(B, H, W, Cout, device="cuda", dtype=torch.bfloat16)
    f = lambda: lib()("s3od_conv_fwd", BF16, B, H, W, Cin, H, W, Cout, k, k, 1, k // 2, x, 0, w, None, None, None, 0, None,
                      None, o, None, None, None, stream())
    t = timeit(f, 10)
    fl = 2 * B * H * W * Cin * Cout * k * k
    print(f"conv fwd B={B} {H}x{W} {Cin}->{Cout} k{k}: {t * 1e6:8.1f} us  {fl / t / 1e12:7.1f} TF/s")


def attn(B, N):
    q = torch.randn(B * 12, N, 64, device="cuda").bfloat16()
    k, v = torch.randn_like(q), torch.randn_like(q)
    o = torch.empty(B, N, 768, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B * 12, N, device="cuda")
    f = lambda: lib()("s3od_attn_fwd", BF16, q, k, v, o, lse, B, 12, N, stream())
    t = timeit(f, 10)
    print(f"attn fwd B={B} N={N}: {t * 1e6:8.1f} us  {4 * B * 12 * N * N * 64 / t / 1e12:7.1f} TF/s")


def attn_bwd(B, N):
    q = torch.randn(B * 12, N, 64, device="cuda").bfloat16() * 0.3
    k, v = torch.randn_like(q), torch.randn_like(q)
    o = torch.empty(B, N, 768, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B * 12, N, device="cuda")
    lib()("s3od_attn_fwd", BF16, q, k, v, o, lse, B, 12, N, stream())
    do = torch.randn_like(o)
    delta = torch.empty_like(lse)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(q), torch.empty_like(q)
    f = lambda: lib()("s3od_attn_bwd", BF16, q, k, v, o, do, lse, delta, dq, dk, dv, B, 12, N, stream())
    t = timeit(f, 10)
    print(f"attn bwd B={B} N={N}: {t * 1e6:8.1f} us  {10 * B * 12 * N * N * 64 / t / 1e12:7.1f} TF/s (5 GEMMs; 4 algorithmic)")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "attn":
        attn(16, 4101)
        attn_bwd(16, 4101)
        sys.exit(0)
    M = 16 * 4101
    lin(4096, 4096, 4096)
    lin(M, 2304, 768)
    lin(M, 3072, 768)
    lin(M, 768, 3072, out_f32=True)
    dgrad(M, 768, 3072)
    dgrad(M, 3072, 768)
    wgrad(2304, 768, M)
    wgrad(768, 3072, M)
    conv(16, 256, 256, 256, 256)
    conv(16, 1024, 1024, 64, 64)
    attn(16, 4101)
