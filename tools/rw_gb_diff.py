"""Where the grouped-epilogue rw kernel (S3OD_RW_GB) differs from S3OD_RW_GB=0 (dev tool, GPU box): prints the
mismatching (b, y, x, channel) pattern of the masked 64-channel data gradient and the forward.

    python tools/rw_gb_diff.py [GB]
"""
import os
os.environ.setdefault("S3OD_AB", "1")
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd._lib import lib, stream, BF16  # noqa: E402

ACT_RELU, ACT_RELU_BWD = 1, 4


def main():
    gb = sys.argv[1] if len(sys.argv) > 1 else "4"
    for (B, H, W) in ((2, 40, 70), (1, 8, 32), (1, 16, 64)):
        g = torch.Generator(device="cuda").manual_seed(3)
        x = torch.randn(B, H, W, 64, device="cuda", generator=g).bfloat16()
        wp = (torch.randn(64, 3, 3, 64, device="cuda", generator=g) * 0.06).bfloat16()
        wT = wp.flip(1, 2).permute(3, 1, 2, 0).contiguous()
        res1 = torch.randn(B, H, W, 64, device="cuda", generator=g).bfloat16()
        bias = torch.randn(64, device="cuda", generator=g) * 0.1
        outs = {}
        os.environ["S3OD_RW_GB1"] = os.environ.get("GB1", "1")
        for k in ("0", gb):
            os.environ["S3OD_RW_GB"] = k
            dx = torch.full((B, H, W, 64), 7.0, device="cuda", dtype=torch.bfloat16)
            cs = torch.zeros(64, device="cuda")
            lib()("s3od_conv_dgrad", BF16, B, H, W, 64, H, W, 64, 3, 3, 1, 1, x, wp, None, None, None, ACT_RELU_BWD, res1,
                  None, dx, None, None, cs, wT, stream())
            of = torch.full((B, H, W, 64), 7.0, device="cuda", dtype=torch.bfloat16)
            lib()("s3od_conv_fwd", BF16, B, H, W, 64, H, W, 64, 3, 3, 1, 1, x, 0, wp, bias, None, None, ACT_RELU, None, None,
                  of, None, None, None, stream())
            o0 = torch.full((B, H, W, 64), 7.0, device="cuda", dtype=torch.bfloat16)
            lib()("s3od_conv_fwd", BF16, B, H, W, 64, H, W, 64, 3, 3, 1, 1, x, 0, wp, bias, None, None, 0, None, None,
                  o0, None, None, None, stream())
            torch.cuda.synchronize()
            outs[k] = (dx, of, o0, cs)
        for i, nm in enumerate(("dgrad", "fwd relu", "fwd plain")):
            a, b = outs[gb][i].float(), outs["0"][i].float()
            bad = (a != b).nonzero()
            print(f"B{B} H{H} W{W} {nm}: {bad.shape[0]} mismatches of {a.numel()}", flush=True)
            if bad.shape[0]:
                ys = sorted(set(bad[:, 1].tolist())); xs = sorted(set(bad[:, 2].tolist())); cs_ = sorted(set(bad[:, 3].tolist()))
                print("   rows", ys[:40], "\n   cols", xs[:70], "\n   chans", cs_[:64])
                for j in range(min(6, bad.shape[0])):
                    t = tuple(bad[j].tolist())
                    print("   ", t, float(a[t]), float(b[t]))
        print("colsum maxdiff", float((outs[gb][3] - outs["0"][3]).abs().max()))


if __name__ == "__main__":
    main()
