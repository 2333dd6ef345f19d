"""Linear weight-gradient configs for the small / mid outputs of the training step (dev tool, GPU box): for each
shape, the default dispatch vs S3OD_GEMM_CFG x split (slab workspace sized by s3od_linear_wgrad_ws), same process.

    python tools/wgrad_sweep.py
"""
import ctypes
import os
os.environ.setdefault("S3OD_AB", "1")
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd._lib import lib, stream, BF16  # noqa: E402


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


def main():
    shapes = [(768, 768, 65616), (1024, 768, 65536), (256, 256, 1048576)]
    for Nout, Kin, rows in shapes:
        dy = torch.randn(rows, Nout, device="cuda").bfloat16()
        x = torch.randn(rows, Kin, device="cuda").bfloat16()
        ref = None
        for cfg in ("def", "0", "1", "3", "5"):
            for split in (0, 8, 16, 28, 56):
                if cfg == "def" and split:
                    continue
                if cfg == "def":
                    os.environ.pop("S3OD_GEMM_CFG", None)
                else:
                    os.environ["S3OD_GEMM_CFG"] = cfg
                nb = ctypes.c_long(0)
                lib()("s3od_linear_wgrad_ws", BF16, Nout, Kin, rows, split, ctypes.addressof(nb))
                slab = torch.empty(max(1, nb.value // 4), device="cuda") if nb.value else None
                dw = torch.zeros(Nout, Kin, device="cuda")
                f = lambda: lib()("s3od_linear_wgrad", BF16, Nout, Kin, rows, dy, Nout, x, Kin, dw, split, slab,
                                  nb.value, stream())
                t = timeit(f)
                dw.zero_(); f(); torch.cuda.synchronize()
                if ref is None:
                    ref = dw.clone()
                err = float((dw - ref).abs().max() / ref.abs().max())
                print(f"{Nout}x{Kin} rows {rows} cfg {cfg:>3} split {split:2d} slab {nb.value / 2**20:7.1f} MiB: "
                      f"{t * 1e6:7.1f} us {2.0 * rows * Nout * Kin / t / 1e12:6.1f} TF/s  rel {err:.1e}", flush=True)
    os.environ.pop("S3OD_GEMM_CFG", None)


if __name__ == "__main__":
    main()
