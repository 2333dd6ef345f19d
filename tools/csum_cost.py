"""Cost of the fused bias-gradient column sums (fp32 atomics per workgroup / tile) in the conv data gradients:
the same call with and without `colsum` (dev tool, GPU box).

    python tools/csum_cost.py
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd._lib import lib, stream, BF16  # noqa: E402

ACT_RELU_BWD = 4


def t(f, n=10):
    f(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    B = 16
    for (H, C, co) in ((1024, 64, 64), (256, 256, 256), (128, 256, 256)):
        dy = torch.randn(B, H, H, co, device="cuda").bfloat16()
        w = (torch.randn(co, 3, 3, C, device="cuda") * 0.05).bfloat16()
        wT = w.flip(1, 2).permute(3, 1, 2, 0).contiguous()
        res1 = torch.randn(B, H, H, C, device="cuda").bfloat16()
        dx = torch.empty(B, H, H, C, device="cuda", dtype=torch.bfloat16)
        cs = torch.zeros(C, device="cuda")
        for r in range(3):
            for use in (True, False):
                f = lambda: lib()("s3od_conv_dgrad", BF16, B, H, H, C, H, H, co, 3, 3, 1, 1, dy, w, None, None, None,
                                  ACT_RELU_BWD, res1, None, dx, None, None, cs if use else None, wT, stream())
                print(f"{H}^2 {co}->{C} round {r} colsum {use}: {t(f):8.1f} us", flush=True)


if __name__ == "__main__":
    main()
