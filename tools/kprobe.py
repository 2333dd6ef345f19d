"""Run a few representative kernels a handful of times (for rocprofv3 PMC passes)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from tools.gemm_bench import lin, attn, attn_bwd, dgrad, wgrad, conv  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "all"
M = 16 * 4101
if which in ("all", "attn"):
    attn(16, 4101)
    attn_bwd(16, 4101)
if which == "lin64":
    lin(65536, 2304, 64)
if which in ("all", "lin"):
    lin(M, 2304, 768)
if which in ("all", "conv"):
    conv(16, 256, 256, 256, 256)
if which in ("wgrad64", "conv64"):
    from s3od_amd._lib import lib, stream, BF16  # noqa: E402
    B, H, C = 16, 1024, 64
    dy = torch.randn(B, H, H, C, device="cuda").bfloat16()
    x = torch.randn(B, H, H, C, device="cuda").bfloat16()
    w = torch.randn(C, 3, 3, C, device="cuda").bfloat16()
    dw = torch.zeros(C * 9 * C, device="cuda")
    ws = torch.zeros(C * 9 * C, device="cuda")
    out = torch.empty_like(x)
    for _ in range(3):
        if which == "wgrad64":
            lib()("s3od_conv_wgrad", BF16, B, H, H, C, H, H, C, 3, 3, 1, 1, dy, x, 0, dw, ws, 0, None, 0, stream())
        else:
            lib()("s3od_conv_fwd", BF16, B, H, H, C, H, H, C, 3, 3, 1, 1, x, 0, w, None, None, None, 1, None, None, out,
                  None, None, None, stream())
    torch.cuda.synchronize()
