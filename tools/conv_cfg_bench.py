"""Time the 256-channel 3x3 decoder convs of the bs-16 1024^2 training step (RCU fwd with relu_in + BN sums,
layer1_rn, output_conv1 and the data gradients run as forward convs) for the GEMM tile config that
S3OD_GEMM_CFG selects (dev tool; one process per config, the knob is read once); positional arguments are
S3OD_CONV_PP values to alternate (read per call).

    S3OD_GEMM_CFG=5 python tools/conv_cfg_bench.py
    python tools/conv_cfg_bench.py 0 1 0 1
"""
import os
os.environ.setdefault("S3OD_AB", "1")   # knobs toggled per call (csrc/common.hpp S3OD_KNOB)
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd._lib import lib, stream, BF16  # noqa: E402


def timeit(fn, n=8):
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


def conv(tag, B, hh, Cin, Cout, relu_in=0, stats=False, bias=True):
    g = torch.Generator(device="cuda").manual_seed(hh + Cin)
    x = torch.randn(B, hh, hh, Cin, device="cuda", generator=g).bfloat16()
    wp = (torch.randn(Cout, 3, 3, Cin, device="cuda", generator=g) * 0.02).bfloat16()
    b = torch.randn(Cout, device="cuda", generator=g) * 0.1 if bias else None
    st = torch.zeros(32 * 2 * Cout, device="cuda", dtype=torch.float64) if stats else None
    o = torch.empty(B, hh, hh, Cout, device="cuda", dtype=torch.bfloat16)
    f = lambda: lib()("s3od_conv_fwd", BF16, B, hh, hh, Cin, hh, hh, Cout, 3, 3, 1, 1, x, relu_in, wp, b, None, None, 0,
                      None, None, o, None, st, None, stream())
    t = timeit(f)
    fl = 2.0 * B * hh * hh * Cin * Cout * 9
    ref = torch.nn.functional.conv2d(x[:1].permute(0, 3, 1, 2).float().clamp_min(0 if relu_in else -1e30),
                                     wp.float().permute(0, 3, 1, 2), b, padding=1).permute(0, 2, 3, 1)
    err = float((o[:1].float() - ref).norm() / ref.norm())
    print(f"cfg={os.environ.get('S3OD_GEMM_CFG', 'def')} {tag:28s} {t * 1e6:8.1f} us {fl / t / 1e12:7.1f} TF/s  relL2 {err:.2e}",
          flush=True)


def main():
    B = 16
    knobs = sys.argv[1:] or [None]
    for kn in knobs:
        if kn is not None:
            os.environ["S3OD_CONV_PP"] = kn
            os.environ["S3OD_WGRAD_PP"] = kn
        print(f"S3OD_CONV_PP={kn}", flush=True)
        run(B)


def wgrad(tag, B, hh, Cin, Cout, relu=0):
    g = torch.Generator(device="cuda").manual_seed(hh + Cin + 1)
    dy = torch.randn(B, hh, hh, Cout, device="cuda", generator=g).bfloat16()
    x = torch.randn(B, hh, hh, Cin, device="cuda", generator=g).bfloat16()
    dw = torch.zeros(Cout, Cin, 3, 3, device="cuda")
    ws = torch.zeros(Cout * 9 * Cin, device="cuda")
    f = lambda: lib()("s3od_conv_wgrad", BF16, B, hh, hh, Cin, hh, hh, Cout, 3, 3, 1, 1, dy, x, relu, dw, ws, 0, None, 0, stream())
    t = timeit(f)
    fl = 2.0 * B * hh * hh * Cin * Cout * 9
    print(f"cfg={os.environ.get('S3OD_WGRAD_PP', 'def')} {tag:28s} {t * 1e6:8.1f} us {fl / t / 1e12:7.1f} TF/s", flush=True)


def run(B):
    if os.environ.get("WG"):
        wgrad("wgrad rcu 256^2 relu", B, 256, 256, 256, relu=1)
        wgrad("wgrad rcu 256^2", B, 256, 256, 256)
        wgrad("wgrad rcu 128^2", B, 128, 256, 256)
        wgrad("wgrad rn2 128^2 512", B, 128, 512, 256)
        wgrad("wgrad rcu 64^2", B, 64, 256, 256)
        wgrad("wgrad rn3 64^2 1024", B, 64, 1024, 256)
        return
    conv("rcu 256^2 relu_in+stats", B, 256, 256, 256, relu_in=1, stats=True)
    conv("rcu 256^2 stats", B, 256, 256, 256, stats=True)
    conv("rcu/dgrad 256^2 plain", B, 256, 256, 256, bias=False)
    conv("rcu 128^2 relu_in+stats", B, 128, 256, 256, relu_in=1, stats=True)
    conv("rn2 128^2 512->256", B, 128, 512, 256)
    conv("rcu 64^2 stats", B, 64, 256, 256, stats=True)
    conv("oc1 512^2 256->128", B, 512, 256, 128)
    conv("oc1 dgrad 512^2 128->256", B, 512, 128, 256, bias=False)


if __name__ == "__main__":
    main()
