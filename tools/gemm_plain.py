"""Plain bf16 GEMMs through s3od_linear_fwd (no bias / activation, bf16 out) at cube sizes, to compare the ping-pong
main loop with hipBLASLt (dev tool, GPU box):  CFGS=5,6 python tools/gemm_plain.py [sizes...]   (CFGS: S3OD_GEMM_CFG
values to run in turn; 5 = the 8-wave ping-pong kernel, 6 = the 4-wave kernel of gemm_q.hip)"""
import os
os.environ.setdefault("S3OD_AB", "1")
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd._lib import lib, stream, BF16  # noqa: E402
from tools.lin_sweep import timeit  # noqa: E402


def run(M, N, K, rnd=True):
    g = torch.Generator(device="cuda").manual_seed(0)
    mk = (lambda *s: (torch.rand(*s, device="cuda", generator=g) * 2 - 1).bfloat16()) if rnd else \
        (lambda *s: torch.zeros(*s, device="cuda", dtype=torch.bfloat16))
    x, w = mk(M, K), mk(N, K)
    for c in os.environ.get("CFGS", "5").split(","):
        os.environ["S3OD_GEMM_CFG"] = c
        one(M, N, K, x, w, rnd, c)


def one(M, N, K, x, w, rnd, c):
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    f = lambda: lib()("s3od_linear_fwd", BF16, M, N, K, x, K, w, None, None, None, 0, None, N, None, 0, 0, out, N, 0,
                      None, N, 0, 0, 0, stream())
    t = timeit(f, 10)
    ref = (x[:256].float() @ w.float().t())
    err = float((out[:256].float() - ref).norm() / max(ref.norm(), 1e-30))
    print(f"cfg {c} M{M} N{N} K{K} {'rand' if rnd else 'zero'}: {t * 1e6:8.1f} us {2.0 * M * N * K / t / 1e12:7.1f} TF/s  "
          f"(hipBLASLt {hip(x, w, out)})  rel {err:.1e}", flush=True)


def hip(x, w, out):
    f = lambda: torch.matmul(x, w.t(), out=out)
    t = timeit(f, 10)
    return f"{2.0 * x.shape[0] * w.shape[0] * x.shape[1] / t / 1e12:6.1f} TF/s"


def kfit(M=65536, N=3072):
    """time vs K at fixed M, N: the intercept is the per-launch fixed cost (prologue / epilogue / tail), the slope the
    main-loop rate; S3OD_EPI_PROBE=1 rows skip the epilogue stores"""
    g = torch.Generator(device="cuda").manual_seed(0)
    for c in os.environ.get("CFGS", "5").split(","):
        os.environ["S3OD_GEMM_CFG"] = c
        for probe in ("0", "1"):
            os.environ["S3OD_EPI_PROBE"] = probe
            pts = []
            for K in (256, 768, 1536, 3072, 6144):
                x = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).bfloat16()
                w = (torch.rand(N, K, device="cuda", generator=g) * 2 - 1).bfloat16()
                out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
                f = lambda: lib()("s3od_linear_fwd", BF16, M, N, K, x, K, w, None, None, None, 0, None, N, None, 0, 0, out,
                                  N, 0, None, N, 0, 0, 0, stream())
                t = timeit(f, 10) * 1e6
                th = timeit(lambda: torch.matmul(x, w.t(), out=out), 10) * 1e6 if probe == "0" else 0.0
                pts.append((K, t, th))
            n = len(pts)
            for idx in (1, 2):
                mk = sum(p[0] for p in pts) / n; mt = sum(p[idx] for p in pts) / n
                b = sum((p[0] - mk) * (p[idx] - mt) for p in pts) / sum((p[0] - mk) ** 2 for p in pts)
                a = mt - b * mk
                who = f"cfg {c} probe {probe}" if idx == 1 else "hipBLASLt"
                if idx == 2 and probe == "1":
                    continue
                print(f"M{M} N{N} {who:18s}: " + " ".join(f"K{p[0]}:{p[idx]:.1f}" for p in pts) +
                      f" | fixed {a:.1f} us, {b * 64:.2f} us per 64-K ({2.0 * M * N * 64 / (b * 64) / 1e6:.0f} TF/s)", flush=True)
        os.environ["S3OD_EPI_PROBE"] = "0"


if __name__ == "__main__":
    if sys.argv[1:2] == ["kfit"]:
        kfit()
        kfit(65536, 768)
        sys.exit(0)
    sizes = [int(s) for s in sys.argv[1:]] or [4096, 8192]
    for s in sizes:
        run(s, s, s, True)
    run(65536, 768, 3072, True)
    run(65536, 3072, 768, True)
