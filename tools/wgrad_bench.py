"""A/B of the halo-tile 3x3 weight gradients at bs 16: the LDS-DMA kernel (default: producer-wave form) vs the
register-staged one (S3OD_WGRAD_DMA=0) and the 4-wave LDS-DMA form (p0 = S3OD_WGD_PROD=0), knobs read per call,
one process, interleaved rounds; results compared (dev tool).
Shapes: upsample_2x.2 (1024^2, 64 -> 64), output_conv1 (512^2, 256 -> 128, ReLU'd input), mask heads (1024^2, 64 -> 96).

    python tools/wgrad_bench.py            # A/B, every shape
    python tools/wgrad_bench.py pmc        # DMA kernel only, 1024^2 64 -> 64 and 512^2 256 -> 128, one round (profiling)
"""
import os
os.environ.setdefault("S3OD_AB", "1")   # knobs toggled per call (csrc/common.hpp S3OD_KNOB)
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd._lib import lib, stream, BF16  # noqa: E402


def timeit(fn, n=5):
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
    B = 16
    pmc = sys.argv[1:2] == ["pmc"]
    if sys.argv[1:2] == ["big"]:                  # the 256-channel RCU / layerK_rn weight gradients: ping-pong (DMA=0) vs LDS-DMA
        for (H, cin, cout, relu) in ((256, 256, 256, 0), (256, 256, 256, 1), (128, 256, 256, 0), (128, 512, 256, 0),
                                     (64, 256, 256, 0), (64, 1024, 256, 0)):
            dy = torch.randn(B, H, H, cout, device="cuda").bfloat16()
            x = torch.randn(B, H, H, cin, device="cuda").bfloat16()
            ws = torch.zeros(cout * 9 * cin, device="cuda")
            import ctypes
            nb = ctypes.c_long(0)
            os.environ["S3OD_WGRAD_DMA"] = "0"             # the ping-pong arm's slab size
            lib()("s3od_conv_wgrad_ws", BF16, B, H, H, cin, H, H, cout, 3, 3, 1, 1, 0, ctypes.addressof(nb))
            slab = torch.zeros(max(nb.value, 4) // 4, device="cuda")
            fl = 2.0 * B * H * H * cin * cout * 9
            res = {}
            for rnd in range(3):
                for knob in ("0", "1"):
                    os.environ["S3OD_WGRAD_DMA"] = knob
                    dw = torch.zeros(cout, cin, 3, 3, device="cuda")
                    f = lambda: lib()("s3od_conv_wgrad", BF16, B, H, H, cin, H, H, cout, 3, 3, 1, 1, dy, x, relu, dw, ws, 0, slab,
                                      nb.value, stream())
                    t = timeit(f)
                    dw.zero_(); f(); torch.cuda.synchronize(); res[knob] = dw.clone()
                    print(f"{H}^2 {cin}->{cout} relu {relu} round {rnd} DMA={knob}: {t * 1e6:8.1f} us {fl / t / 1e12:7.1f} TF/s", flush=True)
            a, b = res["1"], res["0"]
            print(f"   max |dma - pp| / max|pp| = {float((a - b).abs().max() / b.abs().max()):.3e}")
        os.environ.pop("S3OD_WGRAD_DMA", None)
        return
    if sys.argv[1:2] == ["xp"]:                   # experiment: A/B of a dev knob (argv[2], values argv[3:]) at 1024^2 64 -> 64
        H, cin, cout = 1024, 64, 64                # (XP_SHAPE=512: 512^2 256 -> 128 with the ReLU'd input)
        relu = 0
        if os.environ.get("XP_SHAPE") == "512":
            H, cin, cout, relu = 512, 256, 128, 1
        dy = torch.randn(B, H, H, cout, device="cuda").bfloat16()
        x = torch.randn(B, H, H, cin, device="cuda").bfloat16()
        ws = torch.zeros(cout * 9 * cin, device="cuda")
        dw = torch.zeros(cout, cin, 3, 3, device="cuda")
        for rnd in range(2):
            for xp in sys.argv[3:]:
                os.environ[sys.argv[2]] = xp
                t = timeit(lambda: lib()("s3od_conv_wgrad", BF16, B, H, H, cin, H, H, cout, 3, 3, 1, 1, dy, x, relu, dw, ws, 0, None, 0, stream()))
                print(f"{sys.argv[2]}={xp}: {t * 1e6:8.1f} us", flush=True)
        os.environ.pop(sys.argv[2])
        return
    shapes = ((1024, 64, 64, 0), (512, 256, 128, 0)) + (() if pmc else ((512, 256, 128, 1), (1024, 64, 96, 0)))
    if sys.argv[1:] == ["pmc", "1024"]:
        shapes = shapes[:1]
    for (H, cin, cout, relu) in shapes:
        g = torch.Generator(device="cuda").manual_seed(H + cin)
        dy = torch.randn(B, H, H, cout, device="cuda", generator=g).bfloat16()
        x = torch.randn(B, H, H, cin, device="cuda", generator=g).bfloat16()
        ws = torch.zeros(cout * 9 * cin, device="cuda")
        fl = 2.0 * B * H * H * cin * cout * 9
        res = {}
        for rnd in range(1 if pmc else 3):
            for knob in ("1",) if pmc else ("0", "1", "p0"):
                os.environ["S3OD_WGRAD_DMA"] = "0" if knob == "0" else "1"   # p0: the 4-wave LDS-DMA kernel
                os.environ["S3OD_WGD_PROD"] = "0" if knob == "p0" else "1"
                dw = torch.zeros(cout, cin, 3, 3, device="cuda")
                f = lambda: lib()("s3od_conv_wgrad", BF16, B, H, H, cin, H, H, cout, 3, 3, 1, 1, dy, x, relu, dw, ws, 0, None, 0, stream())
                t = timeit(f)
                dw.zero_()
                f()
                torch.cuda.synchronize()
                res[knob] = dw.clone()
                print(f"{H}^2 {cin}->{cout} relu {relu} round {rnd} DMA={knob}: {t * 1e6:8.1f} us {fl / t / 1e12:7.1f} TF/s", flush=True)
        if pmc:
            continue
        b = res["0"]
        for k in ("1", "p0"):
            a = res[k]
            print(f"{H}^2 {k}: max |dma - staged| / max|staged| = {float((a - b).abs().max() / b.abs().max()):.3e}")
    os.environ.pop("S3OD_WGD_PROD", None)
    if pmc:
        return
    # upsample_2x.0 (ConvTranspose2d(128, 64, 4, 2, 1)) in its conv view: dy 512^2 x 128, x 1024^2 x 64
    H = 512
    g = torch.Generator(device="cuda").manual_seed(7)
    dy = torch.randn(B, H, H, 128, device="cuda", generator=g).bfloat16()
    x = torch.randn(B, 2 * H, 2 * H, 64, device="cuda", generator=g).bfloat16()
    ws = torch.zeros(128 * 16 * 64, device="cuda")
    fl = 2.0 * B * H * H * 128 * 64 * 16
    res = {}
    for rnd in range(3):
        for knob in ("0", "1"):
            os.environ["S3OD_WGRAD_DMA"] = knob
            dw = torch.zeros(128, 64, 4, 4, device="cuda")
            f = lambda: lib()("s3od_conv_wgrad", BF16, B, 2 * H, 2 * H, 64, H, H, 128, 4, 4, 2, 1, dy, x, 0, dw, ws, 0, None, 0, stream())
            t = timeit(f)
            dw.zero_()
            f()
            torch.cuda.synchronize()
            res[knob] = dw.clone()
            print(f"convT wgrad 4x4 s2 round {rnd} DMA={knob}: {t * 1e6:8.1f} us {fl / t / 1e12:7.1f} TF/s", flush=True)
    a, b = res["1"], res["0"]
    print(f"convT wgrad: max |dma - gemm| / max|gemm| = {float((a - b).abs().max() / b.abs().max()):.3e}")
    os.environ.pop("S3OD_WGRAD_DMA", None)


if __name__ == "__main__":
    main()
