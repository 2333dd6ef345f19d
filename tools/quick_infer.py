"""Quick inference timing (dev tool): python tools/quick_infer.py [B] [S] [dtype]"""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd.model import DPTSegmentation  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
S = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
dt = sys.argv[3] if len(sys.argv) > 3 else "bf16"
m = DPTSegmentation(compute_dtype=dt).cuda().eval()
x = torch.randn(B, 3, S, S, device="cuda")
with torch.no_grad():
    for _ in range(2):
        m(x)
    torch.cuda.synchronize()
    t = time.perf_counter()
    n = 5
    for _ in range(n):
        m(x)
    torch.cuda.synchronize()
    dt_ = (time.perf_counter() - t) / n
print(f"B={B} S={S} {dt}: {dt_ * 1e3:.1f} ms/batch, {B / dt_:.2f} img/s, {2.2768e12 * B / dt_ / 1e12 * (S / 1024) ** 2:.1f} TFLOP/s (approx)")
