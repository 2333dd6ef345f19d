"""GPU parity of the hipBLASLt route of s3od_linear_dgrad (csrc/blaslt.hip): the plain bf16 data gradients (no
activation, no column sums, dense rows, optional accumulate into aux / in place) against fp32 torch on the same bf16
operands (rel-L2 <= 4e-3: one bf16 rounding) and against the engine's own kernels (S3OD_DGRAD_BLASLT=0, read per call
under S3OD_AB=1: same tolerance -- the two differ in K summation order only)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
BF16 = 1


def _lib():
    from s3od_amd._lib import lib, stream
    return lib(), stream()


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("M,N,K", [(16384 + 80, 768, 3072), (16384 + 80, 768, 2304), (4101, 768, 768), (1000, 256, 136)])
@pytest.mark.parametrize("accum", ["none", "inplace", "separate"])
def test_blaslt_dgrad(M, N, K, accum, monkeypatch):
    torch.manual_seed(M + N + K)
    L, s = _lib()
    dy = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(K, N, device="cuda") * K ** -0.5).bfloat16()
    base = torch.randn(M, N, device="cuda").bfloat16()
    outs = {}
    for route in ("1", "0"):
        monkeypatch.setenv("S3OD_DGRAD_BLASLT", route)
        dx = base.clone() if accum == "inplace" else torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        aux = dx if accum == "inplace" else (base if accum == "separate" else None)
        L("s3od_linear_dgrad", BF16, M, N, K, dy, K, w, 0, aux, N, dx, N, 0, 0, 0, 0, None, s)
        torch.cuda.synchronize()
        outs[route] = dx
    ref = dy.float() @ w.float() + (base.float() if accum != "none" else 0)
    assert rel(outs["1"].float(), ref) < 4e-3
    assert rel(outs["0"].float(), ref) < 4e-3
    assert rel(outs["1"].float(), outs["0"].float()) < 4e-3
    assert torch.isfinite(outs["1"].float()).all()
