"""hipBLASLt (torch.mm) vs the engine on the plain linear GEMMs of the ViT backward (dev tool, GPU box):
dx[M, N] = dy[M, K] . w[K, N] for the up-projection (N 768, K 3072), QKV (N 768, K 2304) and o_proj (N 768, K 768)
data gradients, plus the bias-only DPT projections x[M, 768] . W^T + b (N 1024 / 512 / 256)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd._lib import lib, stream, BF16  # noqa: E402
from tools.lin_sweep import timeit  # noqa: E402

M = 65616
g = torch.Generator(device="cuda").manual_seed(0)
for N, K in ((768, 3072), (768, 2304), (768, 768)):
    dy = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(K, N, device="cuda", generator=g) * K ** -0.5).bfloat16()
    a = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    b = torch.empty_like(a)
    te = timeit(lambda: lib()("s3od_linear_dgrad", BF16, M, N, K, dy, K, w, 0, None, N, a, N, 0, 0, 0, 0, None, stream()), 10)
    tb = timeit(lambda: torch.mm(dy, w, out=b), 10)
    ref = dy.float() @ w.float()
    ea = float((a.float() - ref).norm() / ref.norm()); eb = float((b.float() - ref).norm() / ref.norm())
    fl = 2.0 * M * N * K
    print(f"dgrad N{N} K{K}: engine {te * 1e6:7.1f} us ({fl / te / 1e12:6.1f} TF/s, rel {ea:.1e}) | hipBLASLt {tb * 1e6:7.1f} us "
          f"({fl / tb / 1e12:6.1f} TF/s, rel {eb:.1e})", flush=True)
M2 = 65536
x = torch.randn(M2, 768, device="cuda", generator=g).bfloat16()
for N in (1024, 512, 256):
    W = (torch.randn(N, 768, device="cuda", generator=g) * 768 ** -0.5).bfloat16()
    bias = torch.randn(N, device="cuda", generator=g)
    a = torch.empty(M2, N, device="cuda", dtype=torch.bfloat16)
    b = torch.empty_like(a)
    bb = bias.bfloat16()
    te = timeit(lambda: lib()("s3od_linear_fwd", BF16, M2, N, 768, x, 768, W, bias, None, None, 0, None, N, None, 0, 0, a, N, 0,
                              None, N, 0, 0, 0, stream()), 10)
    tb = timeit(lambda: torch.addmm(bb, x, W.t(), out=b), 10)
    fl = 2.0 * M2 * N * 768
    print(f"DPT proj N{N}: engine {te * 1e6:7.1f} us ({fl / te / 1e12:6.1f} TF/s) | hipBLASLt addmm {tb * 1e6:7.1f} us "
          f"({fl / tb / 1e12:6.1f} TF/s)", flush=True)
