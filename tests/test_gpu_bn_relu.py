"""GPU: BatchNorm2d + ReLU backward with the ReLU mask recomputed from z (s3od_bn_relu_bwd) is
bit-identical to the backward that reads the stored activation y = relu(bn(z)) (s3od_bn_bwd with
y_relu), for both dtypes, on a ragged pixel count and with z placed so that many y sit at or next
to the ReLU threshold.  The forward y comes from s3od_affine_act, as in the engine's train-mode
ResidualConvUnit (src/s3od/model.py:334-345).  Also checked against an fp32 torch restatement of
the BatchNorm backward on the same inputs (rel-L2 <= 1e-5 f32 / 1e-2 bf16).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

C = 256


def _lib():
    from s3od_amd._lib import lib, stream
    return lib(), stream()


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_bn_relu_bwd_matches_stored_mask(dtype):
    L, st = _lib()
    torch.manual_seed(7)
    dt, code = (torch.float32, 0) if dtype == "f32" else (torch.bfloat16, 1)
    npix = 3 * 1000 + 17
    dev = "cuda"
    w = torch.rand(C, device=dev) + 0.5
    b = torch.randn(C, device=dev) * 0.3
    zf = torch.randn(npix, C, device=dev) * 1.7 + 0.2
    mean = zf.mean(0)
    var = zf.var(0, unbiased=False)
    rstd = (var + 1e-5).rsqrt()
    scale = (w * rstd).contiguous()
    shift = (b - mean * w * rstd).contiguous()
    # a quarter of the rows sit exactly on (or one ulp around) the ReLU threshold z = -shift/scale
    thr = -shift / scale
    zf[: npix // 4] = thr + torch.randint(-1, 2, (npix // 4, C), device=dev).float() * thr.abs() * 2 ** -20
    z = zf.to(dt).contiguous()
    y = torch.empty_like(z)
    L("s3od_affine_act", code, z, scale, shift, 1, None, None, y, y.numel(), C, st)
    dy = torch.randn(npix, C, device=dev).to(dt)

    outs = []
    for mode in ("stored", "recompute"):
        sums = torch.zeros(32 * 3 * C, dtype=torch.float64, device=dev)     # all zero on entry, left all zero
        dz = torch.empty_like(z)
        dw, db, dcb = (torch.zeros(C, device=dev) for _ in range(3))
        if mode == "stored":
            L("s3od_bn_bwd", code, dy, z, y, mean, rstd, w, sums, dz, dw, db, dcb, npix, C, st)
        else:
            L("s3od_bn_relu_bwd", code, dy, z, scale, shift, mean, rstd, w, sums, dz, dw, db, dcb, npix, C, st)
        torch.cuda.synchronize()
        assert int((sums != 0).sum()) == 0, "bn backward must leave its workspace all zero"
        outs.append((dz, dw, db, dcb))
    n_edge = int(((y[: npix // 4].float() == 0) & (z[: npix // 4].float() * scale + shift >= -1e-3)).sum())
    assert n_edge > 0
    for a, c in zip(*outs):
        assert torch.equal(a, c)

    # fp32 reference of the BatchNorm backward given the forward's statistics (mean, rstd):
    # dz = w*rstd*(dy' - mean(dy') - xhat*mean(dy'*xhat)), dy' = dy*(y > 0); dw = sum(dy'*xhat), db = sum(dy')
    dyp = dy.float() * (y.float() > 0)
    xh = (z.float() - mean) * rstd
    dz_ref = w * rstd * (dyp - dyp.mean(0) - xh * (dyp * xh).mean(0))
    tol = 1e-5 if dtype == "f32" else 1e-2
    dz, dw, db, _ = outs[1]
    for got, ref in ((dz.float(), dz_ref), (dw, (dyp * xh).sum(0)), (db, dyp.sum(0))):
        rel = float((got - ref).norm() / ref.norm())
        assert rel <= tol, rel
