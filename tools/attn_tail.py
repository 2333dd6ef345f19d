"""Attention forward time vs sequence length around a 128-query block boundary (dev tool, GPU box): N = 16384
(whole blocks) against the C5 N = 16389 (one extra, almost empty 128-query block per (b, h)), and the training
N = 4101 against 4096.  Shows what the partial last block costs.

    python tools/attn_tail.py
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd._lib import lib, stream, BF16  # noqa: E402


def t_fwd(B, N, H=12, n=5):
    q = (torch.randn(B * H, N, 64, device="cuda") * 0.18).bfloat16()
    k = torch.randn(B * H, N, 64, device="cuda").bfloat16()
    v = torch.randn(B * H, N, 64, device="cuda").bfloat16()
    o = torch.empty(B, N, H * 64, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B * H, N, device="cuda")
    f = lambda: lib()("s3od_attn_fwd", BF16, q, k, v, o, lse, B, H, N, stream())
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    for B, Ns in ((4, (16384, 16389, 16512)), (16, (4096, 4101, 4224))):
        for r in range(2):
            for N in Ns:
                ms = t_fwd(B, N)
                fl = 4.0 * B * 12 * N * N * 64
                print(f"B{B} N{N}: {ms * 1e3:8.1f} us  {fl / ms / 1e9:7.1f} TF/s  (blocks per (b,h) {-(-N // 128)})", flush=True)


if __name__ == "__main__":
    main()
