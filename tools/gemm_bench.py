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
    tb = timeit(lambda: torch.matmul(x, w.t()))
    print(f"linear fwd M={M} N={N} K={K}: {t * 1e6:8.1f} us  {2 * M * N * K / t / 1e12:7.1f} TF/s"
          f"   (hipBLASLt torch.matmul yardstick {2 * M * N * K / tb / 1e12:7.1f} TF/s)")


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
    f = lambda: lib()("s3od_linear_wgrad", BF16, Nout, Kin, rows, dy, Nout, x, Kin, dw, 0, None, 0, stream())
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


def check():
    """Numerics of linear fwd / dgrad / wgrad through the active tile config vs torch fp32."""
    torch.manual_seed(0)
    for (M, N, K) in ((2 * 4101 + 7, 2304, 768), (4101, 768, 3072), (300, 128, 64)):
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = torch.randn(N, K, device="cuda").bfloat16()
        b = torch.randn(N, device="cuda")
        o = torch.empty(M, N, device="cuda", dtype=torch.float32)
        lib()("s3od_linear_fwd", BF16, M, N, K, x, K, w, b, None, None, 0, None, N, None, 0, 0, o, N, 1,
              None, N, 0, 0, 0, stream())
        ref = x.float() @ w.float().t() + b
        e1 = ((o - ref).norm() / ref.norm()).item()
        dy = torch.randn(M, N, device="cuda").bfloat16()
        dx = torch.empty(M, K, device="cuda", dtype=torch.float32)
        lib()("s3od_linear_dgrad", BF16, M, K, N, dy, N, w, 0, None, K, dx, K, 1, 0, 0, 0, None, stream())
        rd = dy.float() @ w.float()
        e2 = ((dx - rd).norm() / rd.norm()).item()
        dw = torch.zeros(N, K, device="cuda")
        lib()("s3od_linear_wgrad", BF16, N, K, M, dy, N, x, K, dw, 0, None, 0, stream())
        rw = dy.float().t() @ x.float()
        e3 = ((dw - rw).norm() / rw.norm()).item()
        torch.cuda.synchronize()
        ok = max(e1, e2, e3) < 1e-5
        print(f"check M={M} N={N} K={K}: fwd {e1:.2e} dgrad {e2:.2e} wgrad {e3:.2e} {'OK' if ok else 'FAIL'}")
        assert ok


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "check":
        check()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "ksweep":
        for K in (64, 128, 256, 768, 1536, 3072):
            lin(65536, 2304, K)
        for K in (64, 768):
            lin(65536, 256, K)
            lin(4096, 2304, K)
        sys.exit(0)
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
