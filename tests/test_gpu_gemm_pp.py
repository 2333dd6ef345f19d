"""GPU parity of the 256x256 ping-pong GEMM kernel (gemm.hpp igemm_pp_kernel) through the C ABI.

The production ViT linears (M = 16 * 4101 = 65616 token rows) run on it; the model-level tests
reach it only at the full-size configurations, so this file pins the kernel itself at sizes that
exercise its paths: the M-tail launch (rows past the last 256-row panel go to a second, 128x128
launch), K tails (K % 64 != 0: zero-filled by the buffer range check), the epilogue variants the
engine uses (bias, LayerScale, fp32 residual, pre-activation store, GELU, GELU' dgrad, in-place
fp32 accumulate), QKV + RoPE with a token-row offset in the tail launch, and split-K wgrad.

Reference: fp32 torch on the same bf16 operands.  Tolerances: rel-L2 <= 1e-5 for fp32 outputs
(fp32 accumulation; only the summation order differs), <= 4e-3 for bf16 outputs (one bf16
rounding, 2^-9 relative), GELU paths <= 5e-3 (the branch-free bf16-mode erf is 1.5e-7 absolute).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

BF16, ACT_GELU, ACT_GELU_BWD = 1, 2, 3


def _lib():
    from s3od_amd._lib import lib, stream
    return lib(), stream()


def rel_l2(a, b):
    a = a.double(); b = b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def r(*s, dt=torch.bfloat16, scale=1.0):
    return (torch.randn(*s, device="cuda") * scale).to(dt)


@pytest.mark.parametrize("M,N,K", [(16384 + 80, 768, 768), (16384 + 80, 2304, 776), (16384, 1280, 3072),
                                   (17000, 768, 136)])
def test_pp_linear_fwd_residual_pre(M, N, K):
    """o_proj / down-projection form: out_f32 = (x w^T + b) * ls + res (fp32), pre (bf16) stored."""
    torch.manual_seed(M + N + K)
    L, s = _lib()
    x, w = r(M, K), r(N, K, scale=K ** -0.5)
    b, ls = r(N, dt=torch.float32), r(N, dt=torch.float32)
    res = r(M, N, dt=torch.float32)
    out = torch.empty(M, N, device="cuda")
    pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    L("s3od_linear_fwd", BF16, M, N, K, x, K, w, b, ls, None, 0, res, N, None, 0, 1, out, N, 1, pre, N, 0, 0, 0, s)
    ref_pre = x.float() @ w.float().t() + b
    ref = ref_pre * ls + res
    torch.cuda.synchronize()
    assert rel_l2(out, ref) < 1e-5
    assert rel_l2(pre.float(), ref_pre) < 4e-3


@pytest.mark.parametrize("M,N,K", [(16384 + 80, 3072, 768), (16384 + 80, 1792, 200)])
def test_pp_linear_fwd_gelu(M, N, K):
    """up-projection form: out = GELU(x w^T + b) in bf16, pre stored."""
    torch.manual_seed(M + N)
    L, s = _lib()
    x, w, b = r(M, K), r(N, K, scale=K ** -0.5), r(N, dt=torch.float32)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    L("s3od_linear_fwd", BF16, M, N, K, x, K, w, b, None, None, ACT_GELU, None, N, None, 0, 0, out, N, 0, pre, N, 0, 0, 0, s)
    ref_pre = x.float() @ w.float().t() + b
    ref = torch.nn.functional.gelu(ref_pre)
    torch.cuda.synchronize()
    assert rel_l2(pre.float(), ref_pre) < 4e-3
    assert rel_l2(out.float(), ref) < 5e-3


def test_pp_qkv_rope_tail():
    """QKV + RoPE + head split at 4 images of 4101 tokens (M tail of 4 * 4101 % 256 = 20 rows):
    the tail launch must address the global token rows."""
    torch.manual_seed(3)
    L, s = _lib()
    B, Nt, P, H = 4, 4101, 4096, 12
    D = 64 * H
    x, w, b = r(B * Nt, D), r(3 * D, D, scale=D ** -0.5), r(3 * D, dt=torch.float32)
    ang = torch.rand(P, 32, device="cuda") * 6.28
    cs = torch.cat([ang.cos(), ang.cos()], 1).contiguous()
    sn = torch.cat([ang.sin(), ang.sin()], 1).contiguous()
    q, k, v = (torch.empty(B * H, Nt, 64, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    L("s3od_qkv_rope_fwd", BF16, B, Nt, P, H, x, w, b, cs, sn, q, k, v, s)
    y = x.float() @ w.float().t() + b                              # [B*Nt, 3D]
    y = y.view(B, Nt, 3, H, 64).permute(2, 0, 3, 1, 4).reshape(3, B * H, Nt, 64)
    def rope(t):
        t = t.clone()
        pt = t[:, Nt - P:]
        rot = torch.cat([-pt[..., 32:], pt[..., :32]], -1)
        t[:, Nt - P:] = pt * cs + rot * sn
        return t
    QSCALE = 0.125 * 1.4426950408889634              # q pre-scaled by log2(e)/8 (common.hpp)
    torch.cuda.synchronize()
    assert rel_l2(q.float(), rope(y[0]) * QSCALE) < 4e-3
    assert rel_l2(k.float(), rope(y[1])) < 4e-3
    assert rel_l2(v.float(), y[2]) < 4e-3


@pytest.mark.parametrize("M,N,K", [(16384 + 80, 768, 3072), (16384 + 80, 768, 2304)])
def test_pp_linear_dgrad_accumulate(M, N, K):
    """up / qkv dgrad form: dx (fp32) += dy w, accumulated in place into the residual gradient."""
    torch.manual_seed(K)
    L, s = _lib()
    dy, w = r(M, K), r(K, N, scale=K ** -0.5)
    dx0 = r(M, N, dt=torch.float32)
    dx = dx0.clone()
    L("s3od_linear_dgrad", BF16, M, N, K, dy, K, w, 0, dx, N, dx, N, 1, 0, 0, 0, None, s)
    ref = dx0 + dy.float() @ w.float()
    torch.cuda.synchronize()
    assert rel_l2(dx, ref) < 1e-5


def test_pp_linear_dgrad_gelu_bwd():
    """down-projection dgrad form (GELU' by the saved pre-activation), bf16 out."""
    torch.manual_seed(7)
    L, s = _lib()
    M, N, K = 16384 + 80, 3072, 768
    dy, w, pre = r(M, K), r(K, N, scale=K ** -0.5), r(M, N)
    dx = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    L("s3od_linear_dgrad", BF16, M, N, K, dy, K, w, ACT_GELU_BWD, pre, N, dx, N, 0, 0, 0, 0, None, s)
    p = pre.float().requires_grad_(True)
    g = torch.autograd.grad(torch.nn.functional.gelu(p), p, dy.float() @ w.float())[0]
    torch.cuda.synchronize()
    assert rel_l2(dx.float(), g) < 5e-3


def _wgrad_slab(L, Nout, Kin, rows):
    """Caller-owned split-K slab sized by the library's own query (s3od_linear_wgrad_ws), poisoned with NaN: the
    kernel must overwrite every word it reads back."""
    import ctypes
    n = ctypes.c_long(0)
    L("s3od_linear_wgrad_ws", BF16, Nout, Kin, rows, 0, ctypes.addressof(n))
    return n.value, (torch.full((max(n.value, 4) // 4,), float("nan"), device="cuda") if n.value else None)


@pytest.mark.parametrize("slab", [False, True])
@pytest.mark.parametrize("Nout,Kin,rows", [(3072, 768, 16384 + 80), (768, 3072, 16384 + 80), (2304, 768, 20000)])
def test_pp_linear_wgrad_split(Nout, Kin, rows, slab):
    """split-K wgrad accumulating onto an existing gradient: fp32 atomics (no slab passed) and the per-split slabs in a
    caller-owned workspace + the reduce kernel (slab = True; the C ABI never allocates)."""
    torch.manual_seed(rows)
    L, s = _lib()
    dy, x = r(rows, Nout), r(rows, Kin)
    dw0 = r(Nout, Kin, dt=torch.float32)
    dw = dw0.clone()
    nb, ws = _wgrad_slab(L, Nout, Kin, rows) if slab else (0, None)
    if slab:
        assert nb > 0 and nb % (4 * Nout * Kin) == 0      # sp slabs of Nout x Kin fp32
    L("s3od_linear_wgrad", BF16, Nout, Kin, rows, dy, Nout, x, Kin, dw, 0, ws, nb, s)
    ref = dw0 + dy.float().t() @ x.float()
    torch.cuda.synchronize()
    assert rel_l2(dw, ref) < 1e-5


@pytest.mark.parametrize("M,N,K", [(16384 + 80, 3072, 768), (16384 + 80, 1792, 200)])
def test_pp_gelu_saved_derivative_pair(M, N, K):
    """bf16 training's MLP pair: the up-projection with act 5 (ACT_GELU_SG) writes GELU(v) to out and gelu'(v) to pre;
    the down-projection dgrad with act 6 (ACT_MUL) multiplies dy w by that saved derivative.  Against fp32 torch
    (gelu and its autograd derivative of the same pre-activation)."""
    torch.manual_seed(M + N + 1)
    L, s = _lib()
    x, w, b = r(M, K), r(N, K, scale=K ** -0.5), r(N, dt=torch.float32)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    gsave = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    L("s3od_linear_fwd", BF16, M, N, K, x, K, w, b, None, None, 5, None, N, None, 0, 0, out, N, 0, gsave, N, 0, 0, 0, s)
    ref_pre = (x.float() @ w.float().t() + b).requires_grad_(True)
    ref = torch.nn.functional.gelu(ref_pre)
    ref_g = torch.autograd.grad(ref.sum(), ref_pre)[0]
    torch.cuda.synchronize()
    assert rel_l2(out.float(), ref.detach()) < 5e-3
    assert rel_l2(gsave.float(), ref_g) < 5e-3
    Kd = 768
    dy, wd = r(M, Kd), r(Kd, N, scale=Kd ** -0.5)
    dx = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    L("s3od_linear_dgrad", BF16, M, N, Kd, dy, Kd, wd, 6, gsave, N, dx, N, 0, 0, 0, 0, None, s)
    torch.cuda.synchronize()
    assert rel_l2(dx.float(), (dy.float() @ wd.float()) * ref_g) < 6e-3


def test_pp_production_rows_65616():
    """The bs-16 1024^2 step's own row count, M = 16 * 4101 = 65616 (256 full 256-row panels x N tiles on the
    ping-pong kernel + an 80-row tail launch), for the ViT linears that select the ping-pong kernel there: QKV + RoPE
    (N 2304, K 768), the up-projection with the saved-gelu' pair (N 3072, K 768), the down-projection forward with
    LayerScale + fp32 residual (N 768, K 3072), the up-projection dgrad accumulated in place (N 768, K 3072) and the
    up-projection wgrad (3072 x 768 over 65616 rows).  The MLP hidden tensors are 403 MB each."""
    torch.manual_seed(65616)
    L, s = _lib()
    B, Nt, P, H = 16, 4101, 4096, 12
    D, F = 64 * H, 4 * 64 * H
    M = B * Nt
    x = r(M, D)
    # QKV + RoPE + head split
    w, b = r(3 * D, D, scale=D ** -0.5), r(3 * D, dt=torch.float32)
    ang = torch.rand(P, 32, device="cuda") * 6.28
    cs = torch.cat([ang.cos(), ang.cos()], 1).contiguous()
    sn = torch.cat([ang.sin(), ang.sin()], 1).contiguous()
    q, k, v = (torch.empty(B * H, Nt, 64, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    L("s3od_qkv_rope_fwd", BF16, B, Nt, P, H, x, w, b, cs, sn, q, k, v, s)
    y = (x.float() @ w.float().t() + b).view(B, Nt, 3, H, 64).permute(2, 0, 3, 1, 4).reshape(3, B * H, Nt, 64)
    pt = y[:2, :, Nt - P:]
    y[:2, :, Nt - P:] = pt * cs + torch.cat([-pt[..., 32:], pt[..., :32]], -1) * sn
    torch.cuda.synchronize()
    QSCALE = 0.125 * 1.4426950408889634
    assert rel_l2(q.float(), y[0] * QSCALE) < 4e-3
    assert rel_l2(k.float(), y[1]) < 4e-3 and rel_l2(v.float(), y[2]) < 4e-3
    del y, pt, q, k, v
    # up-projection: GELU(v) and gelu'(v)
    wu, bu = r(F, D, scale=D ** -0.5), r(F, dt=torch.float32)
    a = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
    gs = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
    L("s3od_linear_fwd", BF16, M, F, D, x, D, wu, bu, None, None, 5, None, F, None, 0, 0, a, F, 0, gs, F, 0, 0, 0, s)
    pre = (x.float() @ wu.float().t() + bu)
    ref = torch.nn.functional.gelu(pre)
    torch.cuda.synchronize()
    assert rel_l2(a.float(), ref) < 5e-3
    pre.requires_grad_(True)
    ref_g = torch.autograd.grad(torch.nn.functional.gelu(pre).sum(), pre)[0]
    assert rel_l2(gs.float(), ref_g) < 5e-3
    del pre, ref, ref_g, gs
    # down-projection forward: (a wd^T + bd) * ls + residual (fp32)
    wd, bd, ls = r(D, F, scale=F ** -0.5), r(D, dt=torch.float32), r(D, dt=torch.float32)
    res = r(M, D, dt=torch.float32)
    out = torch.empty(M, D, device="cuda")
    L("s3od_linear_fwd", BF16, M, D, F, a, F, wd, bd, ls, None, 0, res, D, None, 0, 1, out, D, 1, None, D, 0, 0, 0, s)
    torch.cuda.synchronize()
    assert rel_l2(out, (a.float() @ wd.float().t() + bd) * ls + res) < 1e-5
    # up-projection dgrad, accumulated in place into an fp32 gradient
    dh = r(M, F)
    dx0 = r(M, D, dt=torch.float32)
    dx = dx0.clone()
    L("s3od_linear_dgrad", BF16, M, D, F, dh, F, wu, 0, dx, D, dx, D, 1, 0, 0, 0, None, s)
    torch.cuda.synchronize()
    assert rel_l2(dx, dx0 + dh.float() @ wu.float()) < 1e-5
    # up-projection wgrad over all 65616 rows
    dw0 = r(F, D, dt=torch.float32)
    dw = dw0.clone()
    nb, slab = _wgrad_slab(L, F, D, M)
    L("s3od_linear_wgrad", BF16, F, D, M, dh, F, x, D, dw, 0, slab, nb, s)
    torch.cuda.synchronize()
    assert rel_l2(dw, dw0 + dh.float().t() @ x.float()) < 1e-5


def test_pp_tail_kernel_bit_identical(monkeypatch):
    """The M-tail launch on the skinny full-K kernel (tail_gemm_kernel: one wave per 16 x 16 block, operands from
    global memory) must equal the 128x128 tail launch (S3OD_TAIL_SKINNY=0) BIT FOR BIT -- same MFMA chain over K,
    same fragment layout -- which is what keeps outputs independent of the batch size (a row's position relative to
    the 256-row panels).  Forms: GELU'-multiplied dgrad with the bias column sums (B operand N-contiguous), the
    down-projection forward (bias, LayerScale, fp32 residual, pre; B K-contiguous), each over 65536 + 80 rows, plus
    the fp32-torch check of the tail rows."""
    torch.manual_seed(80)
    L, s = _lib()
    M, D, F = 65536 + 80, 768, 3072
    dy, w, g = r(M, D), r(D, F, scale=D ** -0.5), r(M, F)
    x, w2, b, ls = r(M, F), r(D, F, scale=F ** -0.5), r(D, dt=torch.float32), r(D, dt=torch.float32)
    res = r(M, D, dt=torch.float32)
    outs = {}
    for knob in ("1", "0"):
        monkeypatch.setenv("S3OD_TAIL_SKINNY", knob)
        dx = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
        cs = torch.zeros(F, device="cuda")
        L("s3od_linear_dgrad", BF16, M, F, D, dy, D, w, 6, g, F, dx, F, 0, 0, 0, 0, cs, s)
        out = torch.empty(M, D, device="cuda")
        pre = torch.empty(M, D, device="cuda", dtype=torch.bfloat16)
        L("s3od_linear_fwd", BF16, M, D, F, x, F, w2, b, ls, None, 0, res, D, None, 0, 1, out, D, 1, pre, D, 0, 0, 0, s)
        torch.cuda.synchronize()
        outs[knob] = (dx[-80:].clone(), cs, out[-80:].clone(), pre[-80:].clone())
        del dx, out, pre
    for a, c in zip(outs["1"][:1] + outs["1"][2:], outs["0"][:1] + outs["0"][2:]):
        assert torch.equal(a, c)
    assert rel_l2(outs["1"][1], outs["0"][1]) < 1e-5       # column sums: fp32 atomics, order may differ
    ref = (dy[-80:].float() @ w.float()) * g[-80:].float()
    assert rel_l2(outs["1"][0].float(), ref) < 4e-3
    p = x[-80:].float() @ w2.float().t() + b
    assert rel_l2(outs["1"][2], p * ls + res[-80:]) < 1e-5
    assert rel_l2(outs["1"][3].float(), p) < 4e-3
