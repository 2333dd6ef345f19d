"""Time s3od_attn_fwd / s3od_attn_bwd at the bs16 1024^2 (N=4101) and bs4 2048^2 (N=16389) shapes for the
variant selected by the dev knobs in the environment (S3OD_ATTN_KS / S3OD_ATTN_QS), and save the outputs
so variants can be compared bit for bit (dev tool; one process per variant).

    S3OD_ATTN_KS=4 python tools/attn_sweep.py gpurun_out/attn_ks4.pt
"""
import os
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


def main(out_path):
    res = {}
    tag = f"bwd={os.environ.get('S3OD_ATTN_BWD', '32')} wk={os.environ.get('S3OD_ATTN_WK', '4')} wq={os.environ.get('S3OD_ATTN_WQ', '4')} prio={os.environ.get('S3OD_ATTN_PRIO', '0')} il={os.environ.get('S3OD_ATTN_IL', '0')}"
    for B, N in ((16, 4101), (4, 16389)):
        H = 12
        g = torch.Generator(device="cuda").manual_seed(B * N)
        r = lambda *s: (torch.randn(*s, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
        q, k, v = r(B * H, N, 64), r(B * H, N, 64), r(B * H, N, 64)
        q = (q.float() * 0.18).to(torch.bfloat16)
        o = torch.empty(B, N, H * 64, device="cuda", dtype=torch.bfloat16)
        lse = torch.empty(B * H, N, device="cuda")
        do = r(B, N, H * 64)
        dq, dk, dv = (torch.empty(B * H, N, 64, device="cuda", dtype=torch.bfloat16) for _ in range(3))
        delta = torch.empty(B * H, N, device="cuda")
        fwd = lambda: lib()("s3od_attn_fwd", BF16, q, k, v, o, lse, B, H, N, stream())
        bwd = lambda: lib()("s3od_attn_bwd", BF16, q, k, v, o, do, lse, delta, dq, dk, dv, B, H, N, stream())
        tf = timeit(fwd)
        tb = timeit(bwd)
        fl = 4.0 * B * H * N * N * 64
        print(f"{tag} B{B} N{N}: fwd {tf * 1e6:8.1f} us {fl / tf / 1e12:7.1f} TF/s | bwd {tb * 1e6:8.1f} us "
              f"{2.0 * fl / tb / 1e12:7.1f} TF/s (algorithmic 2x fwd, SURVEY 8d)", flush=True)
        res[N] = {"o": o.cpu(), "dq": dq.cpu(), "dk": dk.cpu(), "dv": dv.cpu(), "tf": tf, "tb": tb}
    torch.save(res, out_path)


if __name__ == "__main__":
    main(sys.argv[1])
