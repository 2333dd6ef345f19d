"""Measurement of north_star's "fused LayerNorm+QKV projection" (dev tool): the build's unfused pair
(s3od_layernorm_fwd writing the bf16 LN output + s3od_qkv_rope_fwd on the ping-pong kernel) vs the prototype
(s3od_layernorm_fwd statistics only + s3od_ln_qkv_rope_fwd: the LN applied in a register-staged A loader of the
128x128 GEMM), bs 16 x 4101 tokens x 768, interleaved rounds in one process; q/k/v compared.

    python tools/ln_qkv_bench.py
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
    B, Nt, P, H = 16, 4101, 4096, 12
    D, M = 64 * H, B * Nt
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(M, D, device="cuda", generator=g)
    lw = 1 + 0.1 * torch.randn(D, device="cuda", generator=g)
    lb = 0.1 * torch.randn(D, device="cuda", generator=g)
    wq = (torch.randn(3 * D, D, device="cuda", generator=g) * 0.03).bfloat16()
    bq = 0.1 * torch.randn(3 * D, device="cuda", generator=g)
    cs = torch.randn(P, 64, device="cuda", generator=g)
    sn = torch.randn(P, 64, device="cuda", generator=g)
    y = torch.empty(M, D, device="cuda", dtype=torch.bfloat16)
    mean, rstd = torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
    outs = {}
    for tag in ("unfused", "fused"):
        outs[tag] = [torch.empty(B * H, Nt, 64, device="cuda", dtype=torch.bfloat16) for _ in range(3)]

    def unfused():
        q, k, v = outs["unfused"]
        lib()("s3od_layernorm_fwd", BF16, x, lw, lb, y, mean, rstd, M, D, 1e-6, stream())
        lib()("s3od_qkv_rope_fwd", BF16, B, Nt, P, H, y, wq, bq, cs, sn, q, k, v, stream())

    def ln_only():
        lib()("s3od_layernorm_fwd", BF16, x, lw, lb, y, mean, rstd, M, D, 1e-6, stream())

    def stats_only():
        lib()("s3od_layernorm_fwd", BF16, x, lw, lb, None, mean, rstd, M, D, 1e-6, stream())

    def fused():
        q, k, v = outs["fused"]
        lib()("s3od_layernorm_fwd", BF16, x, lw, lb, None, mean, rstd, M, D, 1e-6, stream())
        lib()("s3od_ln_qkv_rope_fwd", BF16, B, Nt, P, H, x, mean, rstd, lw, lb, wq, bq, cs, sn, q, k, v, stream())

    def fused_gemm():
        q, k, v = outs["fused"]
        lib()("s3od_ln_qkv_rope_fwd", BF16, B, Nt, P, H, x, mean, rstd, lw, lb, wq, bq, cs, sn, q, k, v, stream())

    def qkv_gemm():
        q, k, v = outs["unfused"]
        lib()("s3od_qkv_rope_fwd", BF16, B, Nt, P, H, y, wq, bq, cs, sn, q, k, v, stream())

    for rnd in range(3):
        t = {n: timeit(f) for n, f in (("unfused", unfused), ("fused", fused), ("ln_fwd", ln_only),
                                       ("ln_stats", stats_only), ("qkv_gemm_pp", qkv_gemm), ("ln_qkv_gemm", fused_gemm))}
        print(f"round {rnd}: " + "  ".join(f"{n} {v * 1e6:7.1f} us" for n, v in t.items()), flush=True)
    unfused(); fused()
    torch.cuda.synchronize()
    for i, n in enumerate("qkv"):
        a, b = outs["fused"][i].float(), outs["unfused"][i].float()
        print(f"{n}: max |fused - unfused| / max|unfused| = {float((a - b).abs().max() / b.abs().max()):.3e}")


if __name__ == "__main__":
    main()
