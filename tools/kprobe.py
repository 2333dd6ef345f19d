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
