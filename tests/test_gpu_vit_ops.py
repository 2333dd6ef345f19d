"""GPU: the fused LayerNorm + LayerScale backward (s3od_layernorm_ls_bwd, csrc/vit_ops.hip ln_bwd_kernel<..., LS>)
against the unfused pair it replaces (s3od_layernorm_bwd, then s3od_layerscale_bwd on its dx) and against fp32 torch
autograd of y = x + lam * u and LayerNorm (tf:modeling_dinov3_vit.py:419-445).  dx and du are the same arithmetic in
both paths (bit-identical); the parameter gradients differ only in fp32 summation order (rel 1e-5)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
F32, BF16 = 0, 1


@pytest.mark.parametrize("dtype", [BF16, F32])
def test_layernorm_ls_bwd_matches_pair(dtype):
    from s3od_amd._lib import lib, stream
    L, st = lib(), stream()
    torch.manual_seed(dtype)
    M, D = 2 * 4101, 768
    T = torch.bfloat16 if dtype == BF16 else torch.float32
    x = torch.randn(M, D, device="cuda")
    w, b = torch.randn(D, device="cuda"), torch.randn(D, device="cuda")
    mean, rstd = x.mean(1), torch.rsqrt(x.var(1, unbiased=False) + 1e-5)
    dy = torch.randn(M, D, device="cuda").to(T)
    dres = torch.randn(M, D, device="cuda")
    u = torch.randn(M, D, device="cuda").to(T)
    lam = torch.rand(D, device="cuda") + 0.1
    ws, ws2 = torch.zeros(32 * 2 * D, device="cuda"), torch.zeros(32 * 2 * D, device="cuda")
    out = {}
    for fused in (True, False):
        dx = torch.empty(M, D, device="cuda")
        du = torch.empty(M, D, device="cuda", dtype=T)
        g = [torch.zeros(D, device="cuda") for _ in range(4)]     # dw, db, dlam, dbias
        if fused:
            L("s3od_layernorm_ls_bwd", dtype, dy, x, mean, rstd, w, dres, dx, g[0], g[1], ws, u, lam, du, g[2], g[3], ws2,
              M, D, st)
        else:
            L("s3od_layernorm_bwd", dtype, dy, x, mean, rstd, w, dres, dx, g[0], g[1], ws, M, D, st)
            L("s3od_layerscale_bwd", dtype, dx, u, lam, du, g[2], g[3], ws2, M, D, st)
        torch.cuda.synchronize()
        out[fused] = (dx, du, g)
    assert torch.equal(out[True][0], out[False][0])
    assert torch.equal(out[True][1], out[False][1])
    for a, c in zip(out[True][2], out[False][2]):
        assert float((a - c).norm() / c.norm()) < 1e-5
    assert float(ws.abs().max()) == 0.0 and float(ws2.abs().max()) == 0.0
    # fp32 autograd reference of the same maths
    xr = x.clone().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    y = torch.nn.functional.layer_norm(xr, (D,), wr, br, 1e-5)
    gx, gw, gb = torch.autograd.grad(y, (xr, wr, br), dy.float())
    dx_ref = gx + dres
    dx, du, g = out[True]
    assert float((dx - dx_ref).norm() / dx_ref.norm()) < 1e-5
    assert float((g[0] - gw).norm() / gw.norm()) < 1e-4 and float((g[1] - gb).norm() / gb.norm()) < 1e-4
    assert float((g[2] - (dx_ref * u.float()).sum(0)).norm() / (dx_ref * u.float()).sum(0).norm()) < 1e-4
    assert float((g[3] - (dx_ref * lam).sum(0)).norm() / (dx_ref * lam).sum(0).norm()) < 1e-4
