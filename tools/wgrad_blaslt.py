"""hipBLASLt (torch.matmul) on the linear weight-gradient shapes, dW[Nout][Kin] = dY^T X over 65616 rows, beside the
engine's s3od_linear_wgrad (slab path) -- is the library faster on these plain GEMMs? (dev tool, GPU box)"""
import ctypes
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd._lib import lib, stream, BF16  # noqa: E402
from tools.lin_sweep import timeit  # noqa: E402

M = 65616
for Nout, Kin in ((3072, 768), (768, 3072), (2304, 768), (768, 768)):
    dy = torch.randn(M, Nout, device="cuda").bfloat16()
    x = torch.randn(M, Kin, device="cuda").bfloat16()
    fl = 2.0 * M * Nout * Kin
    o16 = torch.empty(Nout, Kin, device="cuda", dtype=torch.bfloat16)
    t16 = timeit(lambda: torch.matmul(dy.t(), x, out=o16), 10)
    try:
        o32 = torch.empty(Nout, Kin, device="cuda")
        t32 = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32, out=o32), 10)
        s32 = f"{t32 * 1e6:7.1f} us ({fl / t32 / 1e12:6.1f} TF/s)"
    except Exception as e:  # noqa: BLE001
        s32 = f"n/a ({type(e).__name__})"
    dw = torch.zeros(Nout, Kin, device="cuda")
    nb = ctypes.c_long(0)
    lib()("s3od_linear_wgrad_ws", BF16, Nout, Kin, M, 0, ctypes.addressof(nb))
    slab = torch.empty(max(nb.value, 4) // 4, device="cuda")
    tw = timeit(lambda: lib()("s3od_linear_wgrad", BF16, Nout, Kin, M, dy, Nout, x, Kin, dw, 0, slab, nb.value, stream()), 10)
    print(f"{Nout}x{Kin}: engine {tw * 1e6:7.1f} us ({fl / tw / 1e12:6.1f} TF/s) | hipBLASLt bf16 out {t16 * 1e6:7.1f} us "
          f"({fl / t16 / 1e12:6.1f} TF/s) | fp32 out {s32}", flush=True)
