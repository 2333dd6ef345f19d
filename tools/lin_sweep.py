"""Time the ViT linear GEMMs of the bs=16 1024^2 training step with their REAL epilogues, through the
C ABI, for the tile config selected by S3OD_GEMM_CFG (dev tool; run once per config).

    S3OD_GEMM_CFG=4 python tools/lin_sweep.py
"""
import os
os.environ.setdefault("S3OD_AB", "1")   # knobs toggled per call (csrc/common.hpp S3OD_KNOB)
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd._lib import lib, stream, BF16  # noqa: E402

M, D, F = int(os.environ.get("LIN_M", 65616)), 768, 3072   # LIN_M: row count (tail studies)
ACT_GELU, ACT_GELU_BWD = 2, 3


def timeit(fn, n=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e-3


def r(*s, dt=torch.bfloat16):
    return torch.randn(*s, device="cuda").to(dt)


def fwd(name, N, K, act=0, res_f32=False, out_f32=False, pre=False, scale=False):
    x, w, b = r(M, K), r(N, K), r(N, dt=torch.float32)
    out = torch.empty(M, N, device="cuda", dtype=torch.float32 if out_f32 else torch.bfloat16)
    res = r(M, N, dt=torch.float32) if res_f32 else None
    pr = torch.empty(M, N, device="cuda", dtype=torch.bfloat16) if pre else None
    sc = r(N, dt=torch.float32) if scale else None
    f = lambda: lib()("s3od_linear_fwd", BF16, M, N, K, x, K, w, b, sc, None, act, res, N, None, 0, int(res_f32), out, N,
                      int(out_f32), pr, N, 0, 0, 0, stream())
    report(name, 2.0 * M * N * K, timeit(f))


def dgrad(name, N, K, act=0, out_f32=False, aux=False):
    dy, w = r(M, K), r(K, N)
    out = torch.empty(M, N, device="cuda", dtype=torch.float32 if out_f32 else torch.bfloat16)
    ax = r(M, N) if aux else None
    f = lambda: lib()("s3od_linear_dgrad", BF16, M, N, K, dy, K, w, act, ax, N, out, N, int(out_f32), 0, 0, 0, None, stream())
    report(name, 2.0 * M * N * K, timeit(f))


def wgrad(name, Nout, Kin):
    dy, x = r(M, Nout), r(M, Kin)
    dw = torch.zeros(Nout, Kin, device="cuda")
    f = lambda: lib()("s3od_linear_wgrad", BF16, Nout, Kin, M, dy, Nout, x, Kin, dw, 0, None, 0, stream())
    report(name, 2.0 * M * Nout * Kin, timeit(f))


def qkv():
    B, Nt, P = 16, 4101, 4096
    x, w, b = r(B * Nt, D), r(3 * D, D), r(3 * D, dt=torch.float32)
    cs, sn = r(P, 64, dt=torch.float32), r(P, 64, dt=torch.float32)
    q, k, v = (torch.empty(B * 12, Nt, 64, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    f = lambda: lib()("s3od_qkv_rope_fwd", BF16, B, Nt, P, 12, x, w, b, cs, sn, q, k, v, stream())
    report("qkv_rope fwd N2304 K768", 2.0 * B * Nt * 3 * D * D, timeit(f))


def conv(name, B, H, Cin, Cout, k=3, act=0):
    x, w, b = r(B, H, H, Cin), r(Cout, k, k, Cin), r(Cout, dt=torch.float32)
    out = torch.empty(B, H, H, Cout, device="cuda", dtype=torch.bfloat16)
    f = lambda: lib()("s3od_conv_fwd", BF16, B, H, H, Cin, H, H, Cout, k, k, 1, k // 2, x, 0, w, b, None, None, act, None, None,
                      out, None, None, None, stream())
    report(name, 2.0 * B * H * H * Cout * Cin * k * k, timeit(f))


def dgrad_conv(name, B, H, Cin, Cout, k=3):
    dy, w, wT = r(B, H, H, Cout), r(Cout, k, k, Cin), r(Cin, k, k, Cout)
    out = torch.empty(B, H, H, Cin, device="cuda", dtype=torch.bfloat16)
    f = lambda: lib()("s3od_conv_dgrad", BF16, B, H, H, Cin, H, H, Cout, k, k, 1, k // 2, dy, w, None, None, None, 0, None,
                      None, out, None, None, None, wT, stream())
    report(name, 2.0 * B * H * H * Cout * Cin * k * k, timeit(f))


def wgrad_conv(name, B, H, Cin, Cout):
    dy, x = r(B, H, H, Cout), r(B, H, H, Cin)
    dw = torch.zeros(Cout * 9 * Cin, device="cuda")
    ws = torch.zeros(Cout * 9 * Cin, device="cuda")
    f = lambda: lib()("s3od_conv_wgrad", BF16, B, H, H, Cin, H, H, Cout, 3, 3, 1, 1, dy, x, 0, dw, ws, 0, None, 0, stream())
    report(name, 2.0 * B * H * H * Cout * Cin * 9, timeit(f))


def heads(name, B, H):
    feat, w1 = r(B, H, H, 64), r(96, 3, 3, 64)
    b1, w2, b2 = r(96, dt=torch.float32), r(3, 32, dt=torch.float32), r(3, dt=torch.float32)
    logits = torch.empty(B, 3, H, H, device="cuda")
    hsave = torch.empty(B * H * H, 96, device="cuda", dtype=torch.bfloat16)
    f = lambda: lib()("s3od_mask_heads_fwd", BF16, B, H, H, 3, feat, w1, b1, w2, b2, logits, hsave, stream())
    report(name, 2.0 * B * H * H * 96 * 576, timeit(f))


def report(name, fl, t):
    tag = os.environ.get('S3OD_GEMM_CFG', 'def')
    print(f"cfg {tag:>3} {name:40s} {t * 1e6:8.1f} us {fl / t / 1e12:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    if os.environ.get("SWEEP") == "ab":
        # same-process A/B of a per-call knob: KNOB=<env name>, positional values (e.g. S3OD_PP_DMA 0 1)
        knob = os.environ["KNOB"]
        for rnd in range(2):
            for val in sys.argv[1:]:
                os.environ[knob] = val
                print(f"--- {knob}={val} round {rnd}", flush=True)
                qkv()
                fwd("o_proj fwd N768 K768 (res f32, out f32, pre)", D, D, res_f32=True, out_f32=True, pre=True, scale=True)
                fwd("up fwd N3072 K768 (GELU, gelu' saved)", F, D, act=5, pre=True)
                fwd("down fwd N768 K3072 (res f32, out f32, pre)", D, F, res_f32=True, out_f32=True, pre=True, scale=True)
                dgrad("up dgrad N768 K3072", D, F)
                dgrad("qkv dgrad N768 K2304", D, 3 * D)
                wgrad("wgrad 3072x768", F, D)
                wgrad("wgrad 768x3072", D, F)
                wgrad("wgrad 2304x768", 3 * D, D)
                conv("conv fwd 256->256 3x3 @256^2 bs16", 16, 256, 256, 256)
                wgrad_conv("conv wgrad 256x(3x3x256) @256^2 bs16", 16, 256, 256, 256)
        sys.exit(0)
    if os.environ.get("SWEEP") == "tail":
        # cost of the 80-row M tail: the fwd / dgrad shapes at 65536 rows (whole panels), 65616 (+ tail launch) and
        # the tail alone (80 rows; S3OD_GEMM_CFG selects its config)
        ms = [int(v) for v in os.environ.get("TAIL_MS", "65536,65616,80").split(",")] * 2
        for m in ms:
            M = m
            print(f"--- M={m}", flush=True)
            fwd("o_proj fwd N768 K768 (res f32, out f32, pre)", D, D, res_f32=True, out_f32=True, pre=True, scale=True)
            fwd("up fwd N3072 K768 (GELU, gelu' saved)", F, D, act=5, pre=True)
            fwd("down fwd N768 K3072 (res f32, out f32, pre)", D, F, res_f32=True, out_f32=True, pre=True, scale=True)
            dgrad("up dgrad N768 K3072", D, F)
            dgrad("down dgrad N3072 K768 (gelu')", F, D, act=6, aux=True)
            dgrad("qkv dgrad N768 K2304", D, 3 * D)
            dgrad("o_proj dgrad N768 K768", D, D)
        sys.exit(0)
    if os.environ.get("SWEEP") == "conv256":
        for hh in (256, 128, 64):
            conv(f"conv fwd 256->256 3x3 @{hh}^2 bs16", 16, hh, 256, 256)
            dgrad_conv(f"conv dgrad 256<-256 3x3 @{hh}^2 bs16", 16, hh, 256, 256)
        sys.exit(0)
    if os.environ.get("SWEEP") == "conv64":
        conv("conv fwd 64->64 3x3 @1024^2 bs16 relu", 16, 1024, 64, 64, act=1)
        heads("mask heads fwd 64->96 (+relu+1x1) @1024^2 bs16", 16, 1024)
        wgrad_conv("conv wgrad 64x(3x3x64) @1024^2 bs16", 16, 1024, 64, 64)
        wgrad_conv("conv wgrad 96x(3x3x64) @1024^2 bs16", 16, 1024, 64, 96)
        wgrad_conv("conv wgrad 256x(3x3x256) @256^2 bs16", 16, 256, 256, 256)
        wgrad_conv("conv wgrad 128x(3x3x256) @512^2 bs16", 16, 512, 256, 128)
        sys.exit(0)
    if os.environ.get("SWEEP") == "gelu":
        # the MLP's GELU pair: pre-activation saved + GELU' in the down dgrad, vs gelu'(v) saved + a multiply
        fwd("up fwd N3072 K768 (GELU, pre saved)", 3072, 768, act=ACT_GELU, pre=True)
        fwd("up fwd N3072 K768 (GELU, gelu' saved)", 3072, 768, act=5, pre=True)
        dgrad("down dgrad N3072 K768 (GELU')", 3072, 768, act=ACT_GELU_BWD, aux=True)
        dgrad("down dgrad N3072 K768 (x saved gelu')", 3072, 768, act=6, aux=True)
        wgrad_conv("conv wgrad 256x(3x3x256) @128^2 bs16", 16, 128, 256, 256)
        wgrad_conv("conv wgrad 256x(3x3x1024) @64^2 bs16", 16, 64, 1024, 256)
        wgrad_conv("conv wgrad 256x(3x3x256) @64^2 bs16", 16, 64, 256, 256)
        dgrad_conv("conv dgrad 64<-64 3x3 @1024^2 bs16", 16, 1024, 64, 64)
        dgrad_conv("conv dgrad 64<-96 3x3 @1024^2 bs16", 16, 1024, 64, 96)
        sys.exit(0)
    qkv()
    fwd("o_proj fwd N768 K768 (res f32, out f32, pre)", D, D, res_f32=True, out_f32=True, pre=True, scale=True)
    fwd("up fwd N3072 K768 (GELU, pre)", F, D, act=ACT_GELU, pre=True)
    fwd("down fwd N768 K3072 (res f32, out f32, pre)", D, F, res_f32=True, out_f32=True, pre=True, scale=True)
    dgrad("down dgrad N3072 K768 (GELU')", F, D, act=ACT_GELU_BWD, aux=True)
    dgrad("up dgrad N768 K3072", D, F)
    dgrad("qkv dgrad N768 K2304", D, 3 * D)
    dgrad("o dgrad N768 K768", D, D)
    wgrad("wgrad 3072x768", F, D)
    wgrad("wgrad 768x3072", D, F)
    wgrad("wgrad 2304x768", 3 * D, D)
    wgrad("wgrad 768x768", D, D)
    conv("conv fwd 256->256 3x3 @256^2 bs16", 16, 256, 256, 256)
    conv("conv fwd 64->64 3x3 @1024^2 bs16 relu", 16, 1024, 64, 64, act=1)
    conv("conv fwd 256->128 3x3 @512^2 bs16", 16, 512, 256, 128)
    # hipBLASLt yardstick (not used by the product): plain bf16 matmul, bf16 out
    for (N, K) in ((F, D), (D, F), (3 * D, D), (D, D)):
        a, bb = r(M, K), r(K, N)
        report(f"hipBLASLt torch.matmul N{N} K{K}", 2.0 * M * N * K, timeit(lambda: torch.matmul(a, bb)))
