"""GPU: s3od_colsum (bias gradients: out += column sums of a [M, N] matrix) -- the two-pass form through the
caller-owned partial-sum workspace against fp32 torch, bit-identical run to run (fixed summation order), and the
per-block fp32-atomic form (no workspace) within fp32 summation-order tolerance; ragged M, N > 2048 (two column
block groups)."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu
BF16 = 1


@pytest.mark.parametrize("M,N", [(16 * 64 * 64, 256), (1000, 256), (65616, 768), (4099, 4096), (37, 64)])
def test_colsum_two_pass(M, N):
    from s3od_amd._lib import lib, stream
    g = torch.Generator(device="cuda").manual_seed(M + N)
    a = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    base = torch.randn(N, device="cuda", generator=g)
    ref = base + a.float().sum(0)
    nb = ctypes.c_long(0)
    lib()("s3od_colsum_ws", M, N, ctypes.addressof(nb))
    assert nb.value > 0
    ws = torch.full((nb.value // 4,), float("nan"), device="cuda")          # dead contents: poisoned
    outs = []
    for _ in range(2):
        out = base.clone()
        lib()("s3od_colsum", BF16, a, N, M, N, out, ws, nb.value, stream())
        outs.append(out)
    atom = base.clone()
    lib()("s3od_colsum", BF16, a, N, M, N, atom, None, 0, stream())
    torch.cuda.synchronize()
    scale = float(a.float().abs().sum(0).max())
    assert torch.equal(outs[0], outs[1])
    assert float((outs[0] - ref).abs().max()) <= 1e-5 * scale
    assert float((atom - ref).abs().max()) <= 1e-5 * scale
