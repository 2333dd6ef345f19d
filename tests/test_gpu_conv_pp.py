"""GPU: the 3x3 stride-1 convs on the 256x256 ping-pong kernel (csrc/gemm.hpp igemm_pp_kernel with the Conv3A
loader, selected by conv_pp_ok in csrc/gemm_ops.hip) -- the DPT ResidualConvUnit / layerK_rn convs
(src/s3od/model.py:223-226,334-345) and their data gradients run as forward convs of dy -- against fp32 PyTorch
convolutions of the same bf16 operands.  Shapes are chosen so the ping-pong path is the one selected (>= 256 pixel
tiles filling whole rounds, K >= 9 * 512 or >= 8 rounds), with ragged image sizes (partial rows, an M tail past the
last 256-row panel) and every epilogue the training step uses: ReLU'd input + bias + BN batch statistics (fp64,
S3OD_NREP replicas), residual adds, the ReLU' mask of the data gradient.  Each case also runs with the path switched
off (S3OD_CONV_PP=0, read per call) and the two results must agree to bf16 rounding.
Tolerance: max-abs <= 2e-2 of the output scale (bf16 output rounding); BN sums <= 2e-3 relative."""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
BF16 = 1
ACT_NONE, ACT_RELU_BWD = 0, 4
NREP = 32


def _close(a, b, tol=2e-2):
    a, b = a.float(), b.float()
    scale = b.abs().max().clamp_min(1e-6)
    err = float((a - b).abs().max() / scale)
    assert err <= tol, err


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def _run(knob, fn):
    os.environ["S3OD_CONV_PP"] = knob
    try:
        return fn()
    finally:
        os.environ.pop("S3OD_CONV_PP", None)


@pytest.mark.parametrize("relu_in,res", [(1, False), (0, True)])
def test_conv_fwd_pp_ragged(relu_in, res):
    """B=4, 61 x 269 (M = 65636: 256 full panels + a 100-row tail), Cin 512 -> 256."""
    from s3od_amd._lib import lib, stream
    B, H, W, Ci, Co = 4, 61, 269, 512, 256
    g = torch.Generator(device="cuda").manual_seed(11 + relu_in)
    x = torch.randn(B, Ci, H, W, device="cuda", generator=g).bfloat16()
    w = (torch.randn(Co, Ci, 3, 3, device="cuda", generator=g) * 0.02).bfloat16()
    bias = torch.randn(Co, device="cuda", generator=g) * 0.1
    r1 = torch.randn(B, Co, H, W, device="cuda", generator=g).bfloat16() if res else None
    r2 = torch.randn(B, Co, H, W, device="cuda", generator=g).bfloat16() if res else None
    xin = x.float().clamp_min(0) if relu_in else x.float()
    pre = F.conv2d(xin, w.float(), bias, padding=1)
    ref = pre + r1.float() + r2.float() if res else pre
    wp = w.permute(0, 2, 3, 1).contiguous()
    outs = {}
    for knob in ("1", "0"):
        out = torch.empty(B, H, W, Co, device="cuda", dtype=torch.bfloat16)
        stats = None if res else torch.zeros(NREP * 2 * Co, device="cuda", dtype=torch.float64)
        _run(knob, lambda: lib()("s3od_conv_fwd", BF16, B, H, W, Ci, H, W, Co, 3, 3, 1, 1, _nhwc(x), relu_in, wp, bias, None,
                                 None, ACT_NONE, _nhwc(r1) if res else None, _nhwc(r2) if res else None, out, None, stats,
                                 None, stream()))
        torch.cuda.synchronize()
        _close(out, _nhwc(ref))
        if stats is not None:
            st = stats.view(NREP, 2, Co).sum(0)
            s_ref, q_ref = pre.double().sum((0, 2, 3)), (pre.double() ** 2).sum((0, 2, 3))
            assert float(((st[0] - s_ref).abs().max() / pre.double().abs().sum((0, 2, 3)).max())) < 2e-3
            assert float(((st[1] - q_ref).abs().max() / q_ref.abs().max())) < 2e-3
        outs[knob] = out
    _close(outs["1"], outs["0"], tol=1.6e-2)


def test_conv_dgrad_as_forward_pp():
    """The data gradient of a 3x3 s1 conv 512 -> 256 (layer2_rn's shape) at 4 x 256 x 256: forward conv of dy with
    the transposed, tap-reversed weight on the ping-pong kernel (N = 512, 2048 tiles), plus the ReLU' mask of a
    saved activation and a residual gradient (the RCU conv1 data gradient's epilogue)."""
    from s3od_amd._lib import lib, stream
    B, H, W, Ci, Co = 4, 256, 256, 512, 256
    g = torch.Generator(device="cuda").manual_seed(5)
    dy = torch.randn(B, Co, H, W, device="cuda", generator=g).bfloat16()
    w = (torch.randn(Co, Ci, 3, 3, device="cuda", generator=g) * 0.02).bfloat16()
    act = torch.randn(B, Ci, H, W, device="cuda", generator=g).bfloat16()
    dres = torch.randn(B, Ci, H, W, device="cuda", generator=g).bfloat16()
    ref = F.conv_transpose2d(dy.float(), w.float(), padding=1) * (act.float() > 0) + dres.float()
    wp = w.permute(0, 2, 3, 1).contiguous()                     # [Co][3][3][Ci]
    wT = w.flip(2, 3).permute(1, 2, 3, 0).contiguous()          # [Ci][3][3][Co], taps reversed
    outs = {}
    for knob in ("1", "0"):
        dx = torch.empty(B, H, W, Ci, device="cuda", dtype=torch.bfloat16)
        _run(knob, lambda: lib()("s3od_conv_dgrad", BF16, B, H, W, Ci, H, W, Co, 3, 3, 1, 1, _nhwc(dy), wp, None, None, None,
                                 ACT_RELU_BWD, _nhwc(act), _nhwc(dres), dx, None, None, None, wT, stream()))
        torch.cuda.synchronize()
        _close(dx, _nhwc(ref))
        outs[knob] = dx
    _close(outs["1"], outs["0"], tol=1.6e-2)


@pytest.mark.parametrize("B,H,W,Ci,relu", [(2, 37, 128, 256, 0), (3, 20, 64, 512, 1), (16, 64, 64, 256, 1)])
def test_conv_wgrad_pp(B, H, W, Ci, relu):
    """3x3 s1 weight gradient of a 256-output-channel conv on the ping-pong kernel (Wgrad3B loader: one tap's 256 input
    channels per tile, pixels split over the grid, fp32 atomics into the GEMM-layout workspace, then the permute),
    accumulated onto an existing gradient, vs torch's conv2d_weight of the same bf16 operands (ReLU'd input when
    relu = 1: an RCU conv1); and vs the 128x128 implicit GEMM (S3OD_WGRAD_PP=0).  Odd H, several images per split.
    Whole-tile shapes (H % 8, W % 32) take the LDS-DMA kernel by default; S3OD_WGRAD_DMA=0 keeps them here."""
    from s3od_amd._lib import lib, stream
    Co = 256
    g = torch.Generator(device="cuda").manual_seed(B * H + Ci)
    dy = torch.randn(B, Co, H, W, device="cuda", generator=g).bfloat16()
    x = torch.randn(B, Ci, H, W, device="cuda", generator=g).bfloat16()
    xin = x.float().clamp_min(0) if relu else x.float()
    dw0 = torch.randn(Co, Ci, 3, 3, device="cuda", generator=g)
    ref = dw0 + torch.nn.grad.conv2d_weight(xin, (Co, Ci, 3, 3), dy.float(), padding=1)
    ws = torch.zeros(Co * 9 * Ci, device="cuda")
    import ctypes
    nb = ctypes.c_long(0)
    os.environ["S3OD_WGRAD_DMA"] = "0"
    lib()("s3od_conv_wgrad_ws", BF16, B, H, W, Ci, H, W, Co, 3, 3, 1, 1, 0, ctypes.addressof(nb))
    os.environ.pop("S3OD_WGRAD_DMA", None)
    # the caller-owned split-K slab (poisoned: every word read back must have been written)
    slab = torch.full((max(nb.value, 4) // 4,), float("nan"), device="cuda") if nb.value else None
    outs = {}
    for knob, sl in (("1", None), ("1", slab), ("0", None)):
        dw = dw0.clone()
        os.environ["S3OD_WGRAD_PP"] = knob
        os.environ["S3OD_WGRAD_DMA"] = "0"
        try:
            lib()("s3od_conv_wgrad", BF16, B, H, W, Ci, H, W, Co, 3, 3, 1, 1, _nhwc(dy), _nhwc(x), relu, dw, ws, 0, sl,
                  nb.value if sl is not None else 0, stream())
        finally:
            os.environ.pop("S3OD_WGRAD_PP", None)
            os.environ.pop("S3OD_WGRAD_DMA", None)
        torch.cuda.synchronize()
        err = float((dw - ref).norm() / (ref - dw0).norm())
        assert err < 1e-5, (knob, sl is not None, err)
        outs[knob, sl is not None] = dw
    assert float(ws.abs().max()) == 0.0          # the workspace is left all zero
    assert float((outs["1", False] - outs["0", False]).norm() / (ref - dw0).norm()) < 1e-5
