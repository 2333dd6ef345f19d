"""GPU: s3od_bilinear_bwd (the backward of F.interpolate(bilinear, align_corners=False), src/s3od/model.py:395-403)
against torch autograd of the fp32 interpolate, on the exact-2x path (its own gather with all 16 candidate rows loaded
together) and on the generic path (a non-multiple size), odd sizes and the broadcast term included (bf16 tolerance)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,IH,IW,OH,OW,C,bc", [(2, 16, 16, 32, 32, 64, False), (2, 15, 13, 30, 26, 32, True),
                                               (1, 7, 9, 14, 18, 16, True), (2, 12, 10, 25, 17, 32, True)])
def test_bilinear_bwd_vs_torch_autograd(B, IH, IW, OH, OW, C, bc):
    from s3od_amd._lib import lib, stream, BF16
    g = torch.Generator(device="cuda").manual_seed(IH * 100 + IW)
    dy = torch.randn(B, OH, OW, C, device="cuda", generator=g).bfloat16()
    bcast = torch.randn(B, C, device="cuda", generator=g) if bc else None
    dx = torch.full((B, IH, IW, C), float("nan"), device="cuda", dtype=torch.bfloat16)
    lib()("s3od_bilinear_bwd", BF16, dy, bcast, dx, B, IH, IW, OH, OW, C, stream())
    torch.cuda.synchronize()
    x = torch.zeros(B, C, IH, IW, device="cuda", requires_grad=True)
    y = F.interpolate(x, size=(OH, OW), mode="bilinear", align_corners=False)
    gy = dy.float().permute(0, 3, 1, 2)
    if bc:
        gy = gy + bcast[:, :, None, None]
    y.backward(gy)
    ref = x.grad.permute(0, 2, 3, 1)
    got = dx.float()
    assert torch.isfinite(got).all()
    assert float((got - ref).norm() / ref.norm()) < 1e-2
