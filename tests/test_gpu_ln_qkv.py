"""GPU: the LayerNorm-fused QKV+RoPE projection prototype (s3od_ln_qkv_rope_fwd: the LN applied in a
register-staged A loader; measured slower than the unfused pair and NOT used by the engine -- DESIGN §6)
equals the build's unfused path (s3od_layernorm_fwd + s3od_qkv_rope_fwd) on the same inputs, and the
statistics-only LayerNorm (y = nullptr) leaves the same mean / rstd.  Reference semantics:
tf:modeling_dinov3_vit.py:419-445 (norm1 -> q/k/v projections), RoPE on the patch tokens."""
import pytest
import torch

pytestmark = pytest.mark.gpu
BF16 = 1


def test_ln_qkv_fused_equals_unfused():
    from s3od_amd._lib import lib, stream
    B, Nt, P, H = 2, 37, 32, 12
    D, M = 64 * H, B * Nt
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(M, D, device="cuda", generator=g) * 2 + 0.5
    lw = 1 + 0.1 * torch.randn(D, device="cuda", generator=g)
    lb = 0.1 * torch.randn(D, device="cuda", generator=g)
    wq = (torch.randn(3 * D, D, device="cuda", generator=g) * 0.03).bfloat16()
    bq = 0.1 * torch.randn(3 * D, device="cuda", generator=g)
    cs = torch.randn(P, 64, device="cuda", generator=g)
    sn = torch.randn(P, 64, device="cuda", generator=g)
    y = torch.empty(M, D, device="cuda", dtype=torch.bfloat16)
    m1, r1, m2, r2 = (torch.empty(M, device="cuda") for _ in range(4))
    qa = [torch.empty(B * H, Nt, 64, device="cuda", dtype=torch.bfloat16) for _ in range(3)]
    qb = [torch.empty(B * H, Nt, 64, device="cuda", dtype=torch.bfloat16) for _ in range(3)]
    lib()("s3od_layernorm_fwd", BF16, x, lw, lb, y, m1, r1, M, D, 1e-6, stream())
    lib()("s3od_qkv_rope_fwd", BF16, B, Nt, P, H, y, wq, bq, cs, sn, *qa, stream())
    lib()("s3od_layernorm_fwd", BF16, x, lw, lb, None, m2, r2, M, D, 1e-6, stream())
    lib()("s3od_ln_qkv_rope_fwd", BF16, B, Nt, P, H, x, m2, r2, lw, lb, wq, bq, cs, sn, *qb, stream())
    torch.cuda.synchronize()
    assert torch.equal(m1, m2) and torch.equal(r1, r2)
    ref = torch.nn.functional.layer_norm(x, (D,), lw, lb, 1e-6)
    assert float((y.float() - ref).abs().max()) < 3e-2
    for a, b in zip(qa, qb):
        assert float((a.float() - b.float()).abs().max() / a.float().abs().max()) < 1e-2
