"""BatchNorm backward A/B between library builds on the GPU box (dev tool): s3od_bn_bwd and s3od_bn_relu_bwd at the
decoder's shapes (bs 16: 256 channels at 128^2 / 64^2, ...), builds loaded side by side (tools/lib_ab.py Lib), calls
alternating, HIP-event medians, and the relative difference of every output against the first build.

    python tools/bn_ab.py old_lib/libs3od_hip.so s3od_amd/libs3od_hip.so
"""
import os
import sys
from pathlib import Path

os.environ.setdefault("S3OD_AB", "1")
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd._lib import BF16, NREP, stream  # noqa: E402
from tools.lib_ab import Lib  # noqa: E402


def main():
    libs = [Lib(p) for p in sys.argv[1:]]
    g = torch.Generator(device="cuda").manual_seed(0)
    st = stream()
    for (B, H, C) in ((16, 256, 256), (16, 128, 256), (16, 64, 256)):
        npix = B * H * H
        dy = (torch.randn(npix, C, device="cuda", generator=g) * 0.1).bfloat16()
        z = torch.randn(npix, C, device="cuda", generator=g).bfloat16()
        mean = torch.randn(C, device="cuda", generator=g) * 0.1
        rstd = torch.rand(C, device="cuda", generator=g) + 0.5
        w = torch.randn(C, device="cuda", generator=g)
        scale = torch.randn(C, device="cuda", generator=g)
        shift = torch.randn(C, device="cuda", generator=g)
        sums = torch.zeros(NREP * 3 * C, dtype=torch.float64, device="cuda")
        res = []
        for L in libs:
            dz = torch.empty_like(dy)
            dw, db, dcb = (torch.zeros(C, device="cuda") for _ in range(3))
            f1 = lambda L=L, dz=dz, dw=dw, db=db, dcb=dcb: L("s3od_bn_bwd", BF16, dy, z, None, mean, rstd, w, sums, dz, dw, db, dcb, npix, C, st)
            f2 = lambda L=L, dz=dz, dw=dw, db=db, dcb=dcb: L("s3od_bn_relu_bwd", BF16, dy, z, scale, shift, mean, rstd, w, sums, dz, dw, db, dcb, npix, C, st)
            res.append(dict(L=L, fns=(f1, f2), dz=dz, t=([], [])))
        for r in range(7):
            for R in res:
                for i, f in enumerate(R["fns"]):
                    f(); torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(3):
                        f()
                    e1.record(); torch.cuda.synchronize()
                    R["t"][i].append(e0.elapsed_time(e1) / 3)
        outs = []
        for R in res:
            R["fns"][1](); torch.cuda.synchronize(); outs.append(R["dz"].clone())
        for k, R in enumerate(res):
            meds = [sorted(x)[len(x) // 2] * 1e3 for x in R["t"]]
            rel = float((outs[k].float() - outs[0].float()).norm() / outs[0].float().norm())
            print(f"npix {npix} C {C} lib{k}: bn_bwd {meds[0]:7.1f} us  bn_relu_bwd {meds[1]:7.1f} us  dz rel vs lib0 {rel:.1e}", flush=True)


if __name__ == "__main__":
    main()
