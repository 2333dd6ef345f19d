"""A/B of upsample_2x.0 = ConvTranspose2d(128, 64, 4, s2, p1) + bias + ReLU at bs 16 (512^2 -> 1024^2): the
register-weight sub-pixel kernel (default) vs the per-parity-class implicit GEMM (S3OD_CONVT_RW=0, read per
call), one process, interleaved rounds; outputs compared (dev tool).

    python tools/convT_bench.py [B] [H]
"""
import os
os.environ.setdefault("S3OD_AB", "1")   # knobs toggled per call (csrc/common.hpp S3OD_KNOB)
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd._lib import lib, stream, BF16  # noqa: E402


def timeit(fn, n=10):
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
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(B, H, H, 128, device="cuda", generator=g).bfloat16()
    wp = (torch.randn(128, 4, 4, 64, device="cuda", generator=g) * 0.03).bfloat16()
    bias = torch.randn(64, device="cuda", generator=g) * 0.1
    wT = wp.permute(3, 1, 2, 0).contiguous()                       # [64][4][4][128]
    fl = 2.0 * B * (2 * H) ** 2 * 64 * 4 * 128
    by = B * H * H * 128 * 2 + B * (2 * H) ** 2 * 64 * 2
    outs = {}
    for rnd in range(3):
        for knob in ("0", "1"):
            os.environ["S3OD_CONVT_RW"] = knob
            o = torch.empty(B, 2 * H, 2 * H, 64, device="cuda", dtype=torch.bfloat16)
            f = lambda: lib()("s3od_conv_dgrad", BF16, B, 2 * H, 2 * H, 64, H, H, 128, 4, 4, 2, 1, x, wp, bias, None, None, 1,
                              None, None, o, None, None, None, wT, stream())
            t = timeit(f)
            outs[knob] = o
            print(f"round {rnd} CONVT_RW={knob}: {t * 1e6:8.1f} us  {fl / t / 1e12:6.1f} TF/s  {by / t / 1e9:6.0f} GB/s", flush=True)
    os.environ.pop("S3OD_CONVT_RW", None)

    b = outs["0"].float()
    for k in ("1",):
        a = outs[k].float()
        print(f"{k}: max |rw - igemm| / max|igemm| = {float((a - b).abs().max() / b.abs().max()):.3e}")
    # its data gradient: Conv2d(64, 128, 4, s2, p1) of dy (2H x 2W x 64) + column sums
    dy = torch.randn(B, 2 * H, 2 * H, 64, device="cuda", generator=g).bfloat16()
    fl2 = 2.0 * B * H * H * 128 * 16 * 64
    by2 = B * (2 * H) ** 2 * 64 * 2 + B * H * H * 128 * 2
    res = {}
    for rnd in range(3):
        for knob in ("0", "1"):
            os.environ["S3OD_CONVT_RW"] = knob
            o = torch.empty(B, H, H, 128, device="cuda", dtype=torch.bfloat16)
            cs = torch.zeros(128, device="cuda")
            f = lambda: lib()("s3od_conv_fwd", BF16, B, 2 * H, 2 * H, 64, H, H, 128, 4, 4, 2, 1, dy, 0, wp, None, None, None, 0,
                              None, None, o, None, None, cs, stream())
            t = timeit(f)
            res[knob] = o
            print(f"dgrad round {rnd} CONVT_RW={knob}: {t * 1e6:8.1f} us  {fl2 / t / 1e12:6.1f} TF/s  {by2 / t / 1e9:6.0f} GB/s", flush=True)
    os.environ.pop("S3OD_CONVT_RW", None)
    a, b = res["1"].float(), res["0"].float()
    print(f"dgrad: max |rw - igemm| / max|igemm| = {float((a - b).abs().max() / b.abs().max()):.3e}")


if __name__ == "__main__":
    main()
