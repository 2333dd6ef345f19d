"""GPU: the bf16 full-resolution decoder convs -- upsample_2x.2 (64->64 + ReLU) and its stride-1 data gradient with
the ReLU' mask and bias column sums (register-weight kernel conv3x3_c64_rw_kernel), the mask heads (64->96, fused
ReLU + 1x1 + hsave), the 64<-96 data gradient, the halo-tile / LDS-DMA weight gradients, the ConvTranspose2d(128, 64,
4, 2, 1) sub-pixel kernel and its strided data / weight gradients -- against fp32 PyTorch convolutions of the same
bf16 operands (reference semantics: nn.Conv2d / ConvTranspose2d in src/s3od/model.py:437-467).  Ragged sizes exercise
partial tiles at the right and bottom edges.  The specialised kernels' implicit-GEMM fall-backs (f32, very large maps)
are checked too through the S3OD_CONVT_RW=0 / S3OD_WGRAD_DMA=0 test hooks (read per call).  Tolerance: bf16 output
rounding (max-abs <= 2e-2 of the output scale)."""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
BF16 = 1
ACT_RELU, ACT_RELU_BWD = 1, 4


def _close(a, b, tol=2e-2):
    a, b = a.float(), b.float()
    scale = b.abs().max().clamp_min(1e-6)
    assert float((a - b).abs().max() / scale) <= tol, float((a - b).abs().max() / scale)


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


@pytest.mark.parametrize("B,H,W", [(2, 37, 45), (1, 64, 96), (3, 16, 33)])
def test_conv_fwd_64_relu(B, H, W):
    from s3od_amd._lib import lib, stream
    g = torch.Generator(device="cuda").manual_seed(H * W)
    x = torch.randn(B, 64, H, W, device="cuda", generator=g).bfloat16()
    w = (torch.randn(64, 64, 3, 3, device="cuda", generator=g) * 0.06).bfloat16()
    bias = torch.randn(64, device="cuda", generator=g) * 0.1
    ref = F.relu(F.conv2d(x.float(), w.float(), bias, padding=1))
    out = torch.empty(B, H, W, 64, device="cuda", dtype=torch.bfloat16)
    wp = w.permute(0, 2, 3, 1).contiguous()                      # [Cout][3][3][Cin]
    lib()("s3od_conv_fwd", BF16, B, H, W, 64, H, W, 64, 3, 3, 1, 1, _nhwc(x), 0, wp, bias, None, None, ACT_RELU,
          None, None, out, None, None, None, stream())
    _close(out, _nhwc(ref))


@pytest.mark.parametrize("cout_fwd", [64, 96])
def test_conv_dgrad_relu_mask_and_colsum(cout_fwd):
    """dx = conv_transpose(dy, W) * (res1 > 0), colsum += sum over pixels of dx."""
    from s3od_amd._lib import lib, stream
    B, H, W = 2, 40, 70
    g = torch.Generator(device="cuda").manual_seed(cout_fwd)
    dy = torch.randn(B, cout_fwd, H, W, device="cuda", generator=g).bfloat16()
    w = (torch.randn(cout_fwd, 64, 3, 3, device="cuda", generator=g) * 0.06).bfloat16()   # conv [Cout][Cin][3][3]
    res1 = torch.randn(B, 64, H, W, device="cuda", generator=g).bfloat16()
    dx_ref = F.conv_transpose2d(dy.float(), w.float(), padding=1) * (res1.float() > 0)
    wp = w.permute(0, 2, 3, 1).contiguous()                                            # [Cout][3][3][Cin]
    wT = w.flip(2, 3).permute(1, 2, 3, 0).contiguous()                                 # [Cin][3][3][Cout], taps reversed
    dx = torch.empty(B, H, W, 64, device="cuda", dtype=torch.bfloat16)
    cs = torch.zeros(64, device="cuda")
    lib()("s3od_conv_dgrad", BF16, B, H, W, 64, H, W, cout_fwd, 3, 3, 1, 1, _nhwc(dy), wp, None, None, None, ACT_RELU_BWD,
          _nhwc(res1), None, dx, None, None, cs, wT, stream())
    _close(dx, _nhwc(dx_ref))
    # column sums are taken in fp32 before the bf16 rounding of dx: compare with the fp32 reference
    ref_cs = dx_ref.sum((0, 2, 3))
    tol = 2e-3 * dx_ref.abs().sum((0, 2, 3)).max()
    assert float((cs - ref_cs).abs().max()) <= float(tol), (float((cs - ref_cs).abs().max()), float(tol))


@pytest.mark.parametrize("gb", ["2"])
def test_rw_grouped_epilogue_bit_identical(gb):
    """The grouped epilogue (S3OD_RW_GB: each group's epilogue issued between the next group's MFMAs, the last group's
    carried into the next tile) runs the same MFMA chain per accumulator: forward outputs (bias + ReLU) bit-identical
    to S3OD_RW_GB=0.  The masked data gradients (64 and 96 input channels) run ungrouped whatever the knob (their
    grouped instances spilled): checked unchanged under it; column sums to fp32 summation order."""
    from s3od_amd._lib import lib, stream
    B, H, W = 3, 37, 70                                    # ragged: partial tiles, several tiles per workgroup
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(B, H, W, 64, device="cuda", generator=g).bfloat16()
    wp = (torch.randn(64, 3, 3, 64, device="cuda", generator=g) * 0.06).bfloat16()
    bias = torch.randn(64, device="cuda", generator=g) * 0.1
    res1 = torch.randn(B, H, W, 64, device="cuda", generator=g).bfloat16()
    dy96 = torch.randn(B, H, W, 96, device="cuda", generator=g).bfloat16()
    w96 = (torch.randn(96, 3, 3, 64, device="cuda", generator=g) * 0.06).bfloat16()
    w96T = w96.flip(1, 2).permute(3, 1, 2, 0).contiguous()
    wT = wp.flip(1, 2).permute(3, 1, 2, 0).contiguous()

    def run():
        of = torch.empty(B, H, W, 64, device="cuda", dtype=torch.bfloat16)
        lib()("s3od_conv_fwd", BF16, B, H, W, 64, H, W, 64, 3, 3, 1, 1, x, 0, wp, bias, None, None, ACT_RELU, None, None,
              of, None, None, None, stream())
        outs = [of]
        for co, d, ww, wt in ((64, x, wp, wT), (96, dy96, w96, w96T)):
            dx = torch.empty(B, H, W, 64, device="cuda", dtype=torch.bfloat16)
            cs = torch.zeros(64, device="cuda")
            lib()("s3od_conv_dgrad", BF16, B, H, W, 64, H, W, co, 3, 3, 1, 1, d, ww, None, None, None, ACT_RELU_BWD, res1,
                  None, dx, None, None, cs, wt, stream())
            outs += [dx, cs]
        torch.cuda.synchronize()
        return outs

    try:
        os.environ["S3OD_RW_GB"] = "0"
        ref = run()
        os.environ["S3OD_RW_GB"] = gb
        got = run()
    finally:
        os.environ.pop("S3OD_RW_GB", None)
    for i, (a, b) in enumerate(zip(got, ref)):
        if a.dtype == torch.bfloat16:
            assert torch.equal(a, b), i
        else:
            assert float((a - b).abs().max()) <= 1e-4 * float(b.abs().max()) + 1e-3, i


@pytest.mark.parametrize("B,H,W", [(2, 50, 41), (3, 37, 70)])
def test_mask_heads_grouped_bit_identical(B, H, W):
    """Mask heads with the grouped epilogue (S3OD_RW_HGB=2: logits stored two tiles later from LDS partial slots) vs
    the ungrouped kernel (S3OD_RW_HGB=0): logits and hsave bit-identical (same summation order)."""
    from s3od_amd._lib import lib, stream
    g = torch.Generator(device="cuda").manual_seed(B * H + W)
    feat = torch.randn(B, H, W, 64, device="cuda", generator=g).bfloat16()
    w1 = (torch.randn(96, 3, 3, 64, device="cuda", generator=g) * 0.06).bfloat16()
    b1 = torch.randn(96, device="cuda", generator=g) * 0.1
    w2 = torch.randn(3, 32, device="cuda", generator=g) * 0.2
    b2 = torch.randn(3, device="cuda", generator=g) * 0.1
    outs = []
    try:
        for hgb in ("0", "2"):
            os.environ["S3OD_RW_HGB"] = hgb
            logits = torch.full((B, 3, H, W), 7.0, device="cuda")
            hsave = torch.full((B * H * W, 96), 7.0, device="cuda", dtype=torch.bfloat16)
            lib()("s3od_mask_heads_fwd", BF16, B, H, W, 3, feat, w1, b1, w2, b2, logits, hsave, stream())
            torch.cuda.synchronize()
            outs.append((logits, hsave))
    finally:
        os.environ.pop("S3OD_RW_HGB", None)
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


def test_mask_heads_fwd_halo():
    from s3od_amd._lib import lib, stream
    B, H, W, NM = 2, 50, 41, 3
    g = torch.Generator(device="cuda").manual_seed(7)
    feat = torch.randn(B, 64, H, W, device="cuda", generator=g).bfloat16()
    w1 = (torch.randn(32 * NM, 64, 3, 3, device="cuda", generator=g) * 0.06).bfloat16()
    b1 = torch.randn(32 * NM, device="cuda", generator=g) * 0.1
    w2 = torch.randn(NM, 32, device="cuda", generator=g) * 0.2
    b2 = torch.randn(NM, device="cuda", generator=g) * 0.1
    h = F.relu(F.conv2d(feat.float(), w1.float(), b1, padding=1))                     # [B, 96, H, W]
    ref = torch.stack([(h[:, 32 * k:32 * k + 32] * w2[k].view(1, 32, 1, 1)).sum(1) + b2[k] for k in range(NM)], 1)
    logits = torch.empty(B, NM, H, W, device="cuda")
    hsave = torch.empty(B * H * W, 32 * NM, device="cuda", dtype=torch.bfloat16)
    lib()("s3od_mask_heads_fwd", BF16, B, H, W, NM, _nhwc(feat), w1.permute(0, 2, 3, 1).contiguous(), b1, w2.contiguous(),
          b2, logits, hsave, stream())
    _close(logits, ref, 3e-2)
    _close(hsave.view(B, H, W, 32 * NM), _nhwc(h))


@pytest.mark.parametrize("cout,B,H,W,relu", [(64, 2, 37, 45, False), (96, 1, 40, 70, False), (64, 3, 16, 33, True),
                                             (64, 2, 64, 96, False), (64, 3, 16, 64, True), (64, 1, 8, 32, True),
                                             (96, 2, 32, 64, True), (96, 1, 8, 32, False)])
def test_conv_wgrad_halo(cout, B, H, W, relu):
    """3x3 s1 weight gradient (halo-tile kernel for Cin 64 -> Cout 64 / 96) vs torch's conv2d_weight of
    the same bf16 operands, accumulated into an existing gradient (+=).  H % 8 == 0 and W % 32 == 0 with Cout 64
    take the LDS-DMA kernel (csrc/wgrad_dma.hip: every border case, one-tile images, several images per workgroup;
    Cout 96 as two 64-channel blocks, the second padded); the ragged shapes the register-staged one."""
    from s3od_amd._lib import lib, stream
    g = torch.Generator(device="cuda").manual_seed(cout + H)
    dy = torch.randn(B, cout, H, W, device="cuda", generator=g).bfloat16()
    x = torch.randn(B, 64, H, W, device="cuda", generator=g).bfloat16()
    xin = F.relu(x.float()) if relu else x.float()
    ref = torch.nn.grad.conv2d_weight(xin, (cout, 64, 3, 3), dy.float(), padding=1)
    dw0 = torch.randn(cout, 64, 3, 3, device="cuda", generator=g)
    dw = dw0.clone()
    ws = torch.zeros(cout * 9 * 64, device="cuda")                 # all zero on entry, left all zero
    lib()("s3od_conv_wgrad", BF16, B, H, W, 64, H, W, cout, 3, 3, 1, 1, _nhwc(dy), _nhwc(x), int(relu), dw, ws, 0, None, 0, stream())
    torch.cuda.synchronize()
    assert int((ws != 0).sum()) == 0, "conv_wgrad must leave its workspace all zero"
    got = dw - dw0
    assert float((got - ref).abs().max() / ref.abs().max()) < 2e-3, float((got - ref).abs().max() / ref.abs().max())


@pytest.mark.parametrize("cin,cout,B,H,W,relu", [(256, 256, 2, 20, 36, True), (128, 192, 1, 512, 520, True),
                                                  (256, 128, 1, 520, 512, False), (128, 128, 2, 512, 512, True),
                                                  (256, 256, 4, 64, 64, True), (512, 256, 2, 32, 64, False),
                                                  (1024, 256, 1, 16, 32, False)])
def test_conv_wgrad_halo_channel_blocks(cin, cout, B, H, W, relu):
    """The halo wgrad over 64-channel blocks of wider convs: the LDS-DMA kernel for every whole-tile shape (the RCU /
    layerK_rn / output_conv1 weight gradients, down to one-tile-per-image maps), the register-staged one from 512^2
    maps otherwise; the ragged small map takes the ping-pong / implicit GEMM (first case)."""
    from s3od_amd._lib import lib, stream
    g = torch.Generator(device="cuda").manual_seed(cin + cout)
    dy = torch.randn(B, cout, H, W, device="cuda", generator=g).bfloat16()
    x = torch.randn(B, cin, H, W, device="cuda", generator=g).bfloat16()
    xin = F.relu(x.float()) if relu else x.float()
    ref = torch.nn.grad.conv2d_weight(xin, (cout, cin, 3, 3), dy.float(), padding=1)
    dw = torch.zeros(cout, cin, 3, 3, device="cuda")
    ws = torch.zeros(cout * 9 * cin, device="cuda")                # all zero on entry, left all zero
    lib()("s3od_conv_wgrad", BF16, B, H, W, cin, H, W, cout, 3, 3, 1, 1, _nhwc(dy), _nhwc(x), int(relu), dw, ws, 0, None, 0, stream())
    torch.cuda.synchronize()
    assert int((ws != 0).sum()) == 0, "conv_wgrad must leave its workspace all zero"
    assert float((dw - ref).abs().max() / ref.abs().max()) < 2e-3, float((dw - ref).abs().max() / ref.abs().max())


@pytest.mark.parametrize("cin,cout,H,W", [(256, 256, 40, 70), (512, 256, 33, 20), (256, 128, 24, 40)])
def test_conv_dgrad_via_transposed_weight(cin, cout, H, W):
    """3x3 s1 data gradient run as a forward conv of dy with wT = the transposed, tap-reversed weight (the RCU /
    layerK_rn / output_conv1 path, bf16): ReLU' mask of res1, the residual gradient res2 and the bias column sums,
    vs fp32 conv_transpose2d of the same bf16 operands."""
    from s3od_amd._lib import lib, stream
    B = 2
    g = torch.Generator(device="cuda").manual_seed(cin + cout + H)
    dy = torch.randn(B, cout, H, W, device="cuda", generator=g).bfloat16()
    w = (torch.randn(cout, cin, 3, 3, device="cuda", generator=g) * (1.0 / (3 * cout ** 0.5))).bfloat16()
    res1 = torch.randn(B, cin, H, W, device="cuda", generator=g).bfloat16()
    res2 = torch.randn(B, cin, H, W, device="cuda", generator=g).bfloat16()
    dx_ref = F.conv_transpose2d(dy.float(), w.float(), padding=1) * (res1.float() > 0)
    ref = dx_ref + res2.float()
    wp = w.permute(0, 2, 3, 1).contiguous()                                            # [Cout][3][3][Cin]
    wT = w.flip(2, 3).permute(1, 2, 3, 0).contiguous()                                 # [Cin][3][3][Cout]
    dx = torch.empty(B, H, W, cin, device="cuda", dtype=torch.bfloat16)
    cs = torch.zeros(cin, device="cuda")
    lib()("s3od_conv_dgrad", BF16, B, H, W, cin, H, W, cout, 3, 3, 1, 1, _nhwc(dy), wp, None, None, None, ACT_RELU_BWD,
          _nhwc(res1), _nhwc(res2), dx, None, None, cs, wT, stream())
    _close(dx, _nhwc(ref))
    ref_cs = ref.sum((0, 2, 3))
    tol = 2e-3 * ref.abs().sum((0, 2, 3)).max()
    assert float((cs - ref_cs).abs().max()) <= float(tol), (float((cs - ref_cs).abs().max()), float(tol))


@pytest.mark.parametrize("B,H,W,relu", [(2, 19, 37, True), (1, 32, 48, False), (3, 8, 16, True), (1, 70, 9, True)])
def test_convT_4s2_register_weight(B, H, W, relu):
    """upsample_2x.0 = ConvTranspose2d(128, 64, 4, stride 2, pad 1) + bias (+ ReLU) on the register-weight sub-pixel
    kernel (csrc/gemm_ops.hip convT4s2_rw_kernel; reference module src/s3od/model.py:146-153) vs fp32
    conv_transpose2d of the same bf16 operands; ragged input maps exercise partial 8 x 16 tiles.  The generic
    per-parity-class implicit GEMM (S3OD_CONVT_RW=0, read per call) is checked against the same reference."""
    import os
    from s3od_amd._lib import lib, stream
    g = torch.Generator(device="cuda").manual_seed(B * H * W)
    x = torch.randn(B, 128, H, W, device="cuda", generator=g).bfloat16()
    w = (torch.randn(128, 64, 4, 4, device="cuda", generator=g) * 0.03).bfloat16()      # ConvT [Cin][Cout][4][4]
    bias = torch.randn(64, device="cuda", generator=g) * 0.1
    ref = F.conv_transpose2d(x.float(), w.float(), bias, stride=2, padding=1)
    if relu:
        ref = F.relu(ref)
    wp = w.permute(0, 2, 3, 1).contiguous()                                              # conv view [128][4][4][64]
    wT = w.permute(1, 2, 3, 0).contiguous()                                              # [64][4][4][128] (no flip)
    outs = []
    for knob in ("1", "0"):
        os.environ["S3OD_CONVT_RW"] = knob
        try:
            out = torch.full((B, 2 * H, 2 * W, 64), float("nan"), device="cuda", dtype=torch.bfloat16)
            lib()("s3od_conv_dgrad", BF16, B, 2 * H, 2 * W, 64, H, W, 128, 4, 4, 2, 1, _nhwc(x), wp, bias, None, None,
                  ACT_RELU if relu else 0, None, None, out, None, None, None, wT, stream())
            torch.cuda.synchronize()
        finally:
            os.environ.pop("S3OD_CONVT_RW", None)
        assert not torch.isnan(out.float()).any(), "every output pixel must be written"
        _close(out, _nhwc(ref))
        outs.append(out)


@pytest.mark.parametrize("B,H,W", [(2, 19, 37), (1, 32, 48), (3, 4, 16), (1, 70, 9)])
def test_conv_4s2_register_weight_colsum(B, H, W):
    """The data gradient of upsample_2x.0 = Conv2d(64, 128, 4, stride 2, pad 1) of dy with the conv-view weight
    [128][4][4][64], plus the column sums (output_conv1's bias gradient), on the register-weight strided kernel
    (csrc/gemm_ops.hip conv4s2_rw_kernel) and on the implicit GEMM (S3OD_CONVT_RW=0), vs fp32 conv2d of the same
    bf16 operands (H x W = the output grid; the input is 2H x 2W)."""
    import os
    from s3od_amd._lib import lib, stream
    g = torch.Generator(device="cuda").manual_seed(B + H * W)
    x = torch.randn(B, 64, 2 * H, 2 * W, device="cuda", generator=g).bfloat16()
    w = (torch.randn(128, 64, 4, 4, device="cuda", generator=g) * 0.03).bfloat16()
    ref = F.conv2d(x.float(), w.float(), stride=2, padding=1)                              # [B, 128, H, W]
    wp = w.permute(0, 2, 3, 1).contiguous()                                              # [128][4][4][64]
    for knob in ("1", "0"):
        os.environ["S3OD_CONVT_RW"] = knob
        try:
            out = torch.full((B, H, W, 128), float("nan"), device="cuda", dtype=torch.bfloat16)
            cs = torch.zeros(128, device="cuda")
            lib()("s3od_conv_fwd", BF16, B, 2 * H, 2 * W, 64, H, W, 128, 4, 4, 2, 1, _nhwc(x), 0, wp, None, None, None, 0,
                  None, None, out, None, None, cs, stream())
            torch.cuda.synchronize()
        finally:
            os.environ.pop("S3OD_CONVT_RW", None)
        assert not torch.isnan(out.float()).any(), "every output pixel must be written"
        _close(out, _nhwc(ref))
        ref_cs = ref.sum((0, 2, 3))
        tol = 2e-3 * ref.abs().sum((0, 2, 3)).max()
        assert float((cs - ref_cs).abs().max()) <= float(tol), (knob, float((cs - ref_cs).abs().max()), float(tol))


@pytest.mark.parametrize("B,H,W", [(2, 19, 37), (1, 32, 64), (1, 5, 70)])
def test_conv_4s2_wgrad(B, H, W):
    """Weight gradient of the conv view of upsample_2x.0 (4x4, stride 2, pad 1; dy 128 channels on H x W, x 64 channels
    on 2H x 2W) on the LDS-DMA register-accumulator kernel (conv4s2_wgrad_dma_kernel) and on the implicit GEMM
    (S3OD_WGRAD_DMA=0) vs torch's conv2d_weight of the same bf16 operands, accumulated into an existing gradient."""
    import os
    from s3od_amd._lib import lib, stream
    g = torch.Generator(device="cuda").manual_seed(H * W + B)
    dy = torch.randn(B, 128, H, W, device="cuda", generator=g).bfloat16()
    x = torch.randn(B, 64, 2 * H, 2 * W, device="cuda", generator=g).bfloat16()
    ref = torch.nn.grad.conv2d_weight(x.float(), (128, 64, 4, 4), dy.float(), stride=2, padding=1)
    for knob in ("1", "0"):
        os.environ["S3OD_WGRAD_DMA"] = knob
        try:
            dw0 = torch.randn(128, 64, 4, 4, device="cuda", generator=g)
            dw = dw0.clone()
            ws = torch.zeros(128 * 16 * 64, device="cuda")
            lib()("s3od_conv_wgrad", BF16, B, 2 * H, 2 * W, 64, H, W, 128, 4, 4, 2, 1, _nhwc(dy), _nhwc(x), 0, dw, ws, 0, None, 0,
                  stream())
            torch.cuda.synchronize()
        finally:
            os.environ.pop("S3OD_WGRAD_DMA", None)
        assert int((ws != 0).sum()) == 0, "conv_wgrad must leave its workspace all zero"
        got = dw - dw0
        assert float((got - ref).abs().max() / ref.abs().max()) < 2e-3, (knob, float((got - ref).abs().max() / ref.abs().max()))
