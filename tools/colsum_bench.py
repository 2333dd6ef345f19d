"""Column sums (s3od_colsum: the fusion blocks' out_conv bias gradients, [npix][256] bf16) at the training step's
four sizes: the two-pass form (partial-sum workspace) vs the per-block fp32 atomics (S3OD_COLSUM_2P=0), alternating in
one process (dev tool).

    python tools/colsum_bench.py
"""
import ctypes
import os
os.environ.setdefault("S3OD_AB", "1")
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd._lib import lib, stream, BF16  # noqa: E402


def main():
    vals = sys.argv[1:] or ["1", "0"]
    for hw in (256, 128, 64, 32):
        M = 16 * hw * hw
        a = torch.randn(M, 256, device="cuda").bfloat16()
        ref = a.float().sum(0)
        for rnd in range(3):
            for v in vals:
                os.environ["S3OD_COLSUM_2P"] = v
                out = torch.zeros(256, device="cuda")
                nb = ctypes.c_long(0)
                lib()("s3od_colsum_ws", M, 256, ctypes.addressof(nb))
                ws = torch.empty(nb.value // 4, device="cuda")
                f = lambda: lib()("s3od_colsum", BF16, a, 256, M, 256, out, ws, nb.value, stream())
                f(); torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    f()
                e1.record(); torch.cuda.synchronize()
                t = e0.elapsed_time(e1) / 10 * 1e-3
                out.zero_(); f(); torch.cuda.synchronize()
                err = float((out - ref).abs().max() / ref.abs().max())
                print(f"{hw}^2 x16 round {rnd} 2P={v}: {t * 1e6:7.1f} us {M * 512 / t / 1e9:7.0f} GB/s rel {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
