"""A/B of the full-resolution 64 -> 64 3x3 convs (upsample_2x.2 forward with bias + ReLU, and its data gradient
with the ReLU' mask and the bias column sums) at bs 16 x 1024^2: the register-weight kernel (default) vs the
implicit GEMM (S3OD_CONV_RW=0, read per call), in one process, interleaved rounds; outputs compared (dev tool).

    python tools/conv64_bench.py [B] [H]        (ARMS=RW_GB=0,RW_GB=2: other S3OD_ knobs as the arms)
"""
import os
os.environ.setdefault("S3OD_AB", "1")   # knobs toggled per call (csrc/common.hpp S3OD_KNOB)
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd._lib import lib, stream, BF16  # noqa: E402

ACT_RELU, ACT_RELU_BWD = 1, 4


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
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    W = H
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(B, H, W, 64, device="cuda", generator=g).bfloat16()
    w = (torch.randn(64, 3, 3, 64, device="cuda", generator=g) * 0.06).bfloat16()       # [Cout][3][3][Cin]
    wT = w.flip(1, 2).permute(3, 1, 2, 0).contiguous()                                 # [Cin][3][3][Cout]
    bias = torch.randn(64, device="cuda", generator=g) * 0.1
    res1 = torch.randn(B, H, W, 64, device="cuda", generator=g).bfloat16()
    dy96 = torch.randn(B, H, W, 96, device="cuda", generator=g).bfloat16()
    w96 = (torch.randn(96, 3, 3, 64, device="cuda", generator=g) * 0.06).bfloat16()    # heads conv [96][3][3][64]
    w96T = w96.flip(1, 2).permute(3, 1, 2, 0).contiguous()                             # [64][3][3][96]
    hw1 = (torch.randn(96, 3, 3, 64, device="cuda", generator=g) * 0.06).bfloat16()
    hb1 = torch.randn(96, device="cuda", generator=g) * 0.1
    hw2 = torch.randn(3, 32, device="cuda", generator=g) * 0.2
    hb2 = torch.randn(3, device="cuda", generator=g) * 0.1
    outs = {}
    fl = 2.0 * B * H * W * 64 * 64 * 9

    def fwd(o):
        lib()("s3od_conv_fwd", BF16, B, H, W, 64, H, W, 64, 3, 3, 1, 1, x, 0, w, bias, None, None, ACT_RELU, None, None,
              o, None, None, None, stream())

    def dgrad(o, cs):
        lib()("s3od_conv_dgrad", BF16, B, H, W, 64, H, W, 64, 3, 3, 1, 1, x, w, None, None, None, ACT_RELU_BWD, res1,
              None, o, None, None, cs, wT, stream())

    def dgrad96(o, cs):
        lib()("s3od_conv_dgrad", BF16, B, H, W, 64, H, W, 96, 3, 3, 1, 1, dy96, w96, None, None, None, ACT_RELU_BWD, res1,
              None, o, None, None, cs, w96T, stream())

    def heads(lg, hs):
        lib()("s3od_mask_heads_fwd", BF16, B, H, W, 3, x, hw1, hb1, hw2, hb2, lg, hs, stream())

    arms = os.environ.get("ARMS", "CONV_RW=0,CONV_RW=1").split(",")   # e.g. ARMS=RW_GB=0,RW_GB=2
    for rnd in range(3):
        for rw in arms:
            kn, val = rw.split("=")
            for a in arms:
                os.environ.pop("S3OD_" + a.split("=")[0], None)
            os.environ["S3OD_" + kn] = val
            of = torch.empty(B, H, W, 64, device="cuda", dtype=torch.bfloat16)
            od = torch.empty_like(of)
            cs = torch.zeros(64, device="cuda")
            tf = timeit(lambda: fwd(of))
            td = timeit(lambda: dgrad(od, cs))
            o96 = torch.empty_like(of)
            t96 = timeit(lambda: dgrad96(o96, cs))
            cs.zero_()
            dgrad(od, cs)
            cs96 = torch.zeros(64, device="cuda")
            dgrad96(o96, cs96)
            torch.cuda.synchronize()
            lgt = torch.empty(B, 3, H, W, device="cuda")
            hs = torch.empty(B * H * W, 96, device="cuda", dtype=torch.bfloat16)
            th = timeit(lambda: heads(lgt, hs))
            outs[rw] = (of, od, cs.clone(), o96, cs96, lgt, hs)
            by_f = B * H * W * 64 * 2 * 2
            by_d = B * H * W * 64 * 2 * 3
            print(f"round {rnd} {rw}: fwd {tf * 1e6:8.1f} us ({fl / tf / 1e12:6.1f} TF/s, {by_f / tf / 1e9:6.0f} GB/s) | "
                  f"dgrad {td * 1e6:8.1f} us ({fl / td / 1e12:6.1f} TF/s, {by_d / td / 1e9:6.0f} GB/s) | dgrad 64<-96 {t96 * 1e6:8.1f} us "
                  f"({fl * 1.5 / t96 / 1e12:6.1f} TF/s, {by_d * 3.5 / 3 / t96 / 1e9:6.0f} GB/s) | heads {th * 1e6:8.1f} us "
                  f"({fl * 1.5 / th / 1e12:6.1f} TF/s, {B * H * W * (128 + 192 + 12) / th / 1e9:6.0f} GB/s)", flush=True)
    for i, name in enumerate(("fwd", "dgrad", "colsum", "dgrad 64<-96", "colsum 64<-96", "head logits", "hsave")):
        a, b = outs[arms[0]][i].float(), outs[arms[-1]][i].float()
        print(f"{name}: max |rw - igemm| / max|igemm| = {float((a - b).abs().max() / b.abs().max().clamp_min(1e-9)):.3e}")


if __name__ == "__main__":
    main()
