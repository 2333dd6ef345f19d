"""Run one GEMM-engine op through the C ABI `reps` times (dev tool for rocprofv3 --pmc passes and kernel traces).

    python tools/gemm_probe.py OP M N K [reps]
      OP: fwd (plain bf16 out) | gelu (ACT_GELU_SG pair, the up-projection) | dgrad (bf16 out) | wgrad (M=Nout, N=Kin,
          K=rows) | conv (3x3 s1, M = B*H*W with H=W=sqrt(M/16), N = Cout, K = Cin) | convw (its weight gradient)
"""
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd._lib import lib, stream, BF16  # noqa: E402


def r(*s):
    return torch.rand(*s, device="cuda").mul_(2).sub_(1).bfloat16()


def main():
    op = sys.argv[1]
    M, N, K = (int(a) for a in sys.argv[2:5])
    reps = int(sys.argv[5]) if len(sys.argv) > 5 else 20
    L, st = lib(), stream()
    if op in ("fwd", "gelu"):
        x, w = r(M, K), r(N, K)
        o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        pre = torch.empty_like(o) if op == "gelu" else None
        act = 5 if op == "gelu" else 0
        f = lambda: L("s3od_linear_fwd", BF16, M, N, K, x, K, w, None, None, None, act, None, N, None, 0, 0, o, N, 0,
                      pre, N, 0, 0, 0, st)
    elif op == "dgrad":
        dy, w = r(M, K), r(K, N)
        o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        f = lambda: L("s3od_linear_dgrad", BF16, M, N, K, dy, K, w, 0, None, N, o, N, 0, 0, 0, 0, None, st)
    elif op == "wgrad":
        dy, x = r(K, M), r(K, N)
        dw = torch.zeros(M, N, device="cuda")
        f = lambda: L("s3od_linear_wgrad", BF16, M, N, K, dy, M, x, N, dw, 0, None, 0, st)
    elif op in ("conv", "convw"):
        B = 16
        hh = int(math.isqrt(M // B))
        x = r(B, hh, hh, K)
        if op == "conv":
            wp = r(N, 3, 3, K)
            o = torch.empty(B, hh, hh, N, device="cuda", dtype=torch.bfloat16)
            f = lambda: L("s3od_conv_fwd", BF16, B, hh, hh, K, hh, hh, N, 3, 3, 1, 1, x, 0, wp, None, None, None, 0, None,
                          None, o, None, None, None, st)
        else:
            dy = r(B, hh, hh, N)
            dw = torch.zeros(N, K, 3, 3, device="cuda")
            ws = torch.zeros(N * 9 * K, device="cuda")
            f = lambda: L("s3od_conv_wgrad", BF16, B, hh, hh, K, hh, hh, N, 3, 3, 1, 1, dy, x, 0, dw, ws, 0, None, 0, st)
    else:
        raise SystemExit(f"unknown op {op}")
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
