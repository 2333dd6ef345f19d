"""Run one linear GEMM shape through the C ABI `reps` times (dev tool for rocprofv3 --pmc passes).

    S3OD_GEMM_CFG=5 python tools/gemm_probe.py M N K [reps]
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd._lib import lib, stream, BF16  # noqa: E402

M, N, K = (int(a) for a in sys.argv[1:4])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
x = torch.rand(M, K, device="cuda").mul_(2).sub_(1).bfloat16()
w = torch.rand(N, K, device="cuda").mul_(2).sub_(1).bfloat16()
o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(reps):
    lib()("s3od_linear_fwd", BF16, M, N, K, x, K, w, None, None, None, 0, None, N, None, 0, 0, o, N, 0,
          None, N, 0, 0, 0, stream())
torch.cuda.synchronize()
print("done")
