"""A/B of the 256-channel 3x3 convs (the DPT ResidualConvUnits, bs 16) on the halo ping-pong kernel (default) vs the
implicit GEMM (S3OD_CONV_HPP=0, read per call), one process, interleaved rounds (dev tool).

    python tools/conv256_bench.py
"""
import os
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
    B, C = 16, 256
    for hh in (256, 128, 64):
        g = torch.Generator(device="cuda").manual_seed(hh)
        x = torch.randn(B, hh, hh, C, device="cuda", generator=g).bfloat16()
        wp = (torch.randn(C, 3, 3, C, device="cuda", generator=g) * 0.02).bfloat16()
        bias = torch.randn(C, device="cuda", generator=g) * 0.1
        stats = torch.zeros(2 * C, device="cuda", dtype=torch.float64)
        fl = 2.0 * B * hh * hh * C * C * 9
        res = {}
        for rnd in range(2):
            for knob in ("0", "1"):
                os.environ["S3OD_CONV_HPP"] = knob
                o = torch.empty(B, hh, hh, C, device="cuda", dtype=torch.bfloat16)
                f = lambda: lib()("s3od_conv_fwd", BF16, B, hh, hh, C, hh, hh, C, 3, 3, 1, 1, x, 1, wp, bias, None, None, 0,
                                  None, None, o, None, stats, None, stream())
                t = timeit(f)
                res[knob] = o
                print(f"{hh}^2 round {rnd} HPP={knob}: conv fwd (relu_in, bias, BN sums) {t * 1e6:8.1f} us {fl / t / 1e12:7.1f} TF/s",
                      flush=True)
        a, b = res["1"].float(), res["0"].float()
        print(f"{hh}^2: max |hpp - gemm| / max|gemm| = {float((a - b).abs().max() / b.abs().max()):.3e}")
    os.environ.pop("S3OD_CONV_HPP", None)


if __name__ == "__main__":
    main()
