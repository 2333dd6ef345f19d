"""8192^3 bf16 GEMM: the ping-pong kernel (s3od_linear_fwd) and hipBLASLt (torch.matmul), 5 launches each, for PMC
passes (dev tool; tools/pmc_cmd.sh <tag> 'igemm_pp|Cijk' tools/gemm_plain_probe.py)."""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd._lib import lib, stream, BF16  # noqa: E402

S = int(os.environ.get("GP_S", 8192))
g = torch.Generator(device="cuda").manual_seed(0)
x = (torch.rand(S, S, device="cuda", generator=g) * 2 - 1).bfloat16()
w = (torch.rand(S, S, device="cuda", generator=g) * 2 - 1).bfloat16()
out = torch.empty(S, S, device="cuda", dtype=torch.bfloat16)
for _ in range(5):
    lib()("s3od_linear_fwd", BF16, S, S, S, x, S, w, None, None, None, 0, None, S, None, 0, 0, out, S, 0, None, S, 0, 0, 0,
          stream())
    torch.matmul(x, w.t(), out=out)
torch.cuda.synchronize()
