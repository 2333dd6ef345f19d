"""Time the fused LayerNorm + LayerScale backward (s3od_layernorm_ls_bwd) against the unfused pair at the bs-16
1024^2 shape (M = 65616 tokens, D = 768, bf16), alternating rounds in one process (dev tool).

    python tools/ln_bench.py
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd._lib import lib, stream, BF16  # noqa: E402


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e-3


def main():
    M, D = 65616, 768
    L, st = lib(), stream()
    x = torch.randn(M, D, device="cuda")
    w = torch.randn(D, device="cuda")
    mean, rstd = x.mean(1), torch.rsqrt(x.var(1, unbiased=False) + 1e-5)
    dy = torch.randn(M, D, device="cuda").bfloat16()
    dres = torch.randn(M, D, device="cuda")
    u = torch.randn(M, D, device="cuda").bfloat16()
    lam = torch.rand(D, device="cuda")
    ws, ws2 = torch.zeros(32 * 2 * D, device="cuda"), torch.zeros(32 * 2 * D, device="cuda")
    dx = torch.empty(M, D, device="cuda")
    du = torch.empty(M, D, device="cuda", dtype=torch.bfloat16)
    g = [torch.zeros(D, device="cuda") for _ in range(4)]
    fused = lambda: L("s3od_layernorm_ls_bwd", BF16, dy, x, mean, rstd, w, dres, dx, g[0], g[1], ws, u, lam, du, g[2], g[3],
                      ws2, M, D, st)
    ln = lambda: L("s3od_layernorm_bwd", BF16, dy, x, mean, rstd, w, dres, dx, g[0], g[1], ws, M, D, st)
    ls = lambda: L("s3od_layerscale_bwd", BF16, dx, u, lam, du, g[2], g[3], ws2, M, D, st)
    for rnd in range(3):
        tf, tl, ts = timeit(fused), timeit(ln), timeit(ls)
        print(f"round {rnd}: fused {tf * 1e6:7.1f} us ({M * D * 18 / tf / 1e9:6.0f} GB/s) | layernorm_bwd {tl * 1e6:7.1f} us "
              f"({M * D * 14 / tl / 1e9:6.0f} GB/s) + layerscale_bwd {ts * 1e6:7.1f} us ({M * D * 8 / ts / 1e9:6.0f} GB/s) = "
              f"{(tl + ts) * 1e6:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
