"""GPU: the halo ping-pong 3x3 convolution (csrc/gemm.hpp conv3x3_hpp_kernel, opt-in: S3OD_CONV_HPP; measured
slower than the implicit GEMM, see gemm_ops.hip) for bf16 3x3 s1 convs with Cin % 64 == 0 and Cout % 256 == 0 --
the DPT ResidualConvUnits and layerK_rn (src/s3od/model.py:334-345, 223-226) -- against fp32 PyTorch
convolutions of the same bf16 operands.  S3OD_CONV_HPP=2 forces the
kernel on maps smaller than its production threshold; ragged sizes exercise partial 8 x 32 tiles (RowMap mode
3), several channel chunks, two output-channel tiles, the ReLU'd input, the BN batch sums and the residual
epilogue.  Tolerance: bf16 output rounding (max-abs <= 2e-2 of the output scale); BN sums in fp64 vs fp32
sums of the fp32 reference, 2e-3 relative."""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
BF16 = 1
ACT_NONE, ACT_RELU = 0, 1


def _close(a, b, tol=2e-2):
    a, b = a.float(), b.float()
    scale = b.abs().max().clamp_min(1e-6)
    assert float((a - b).abs().max() / scale) <= tol, float((a - b).abs().max() / scale)


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


@pytest.mark.parametrize("B,H,W,cin,cout,relu_in", [(2, 37, 45, 256, 256, True), (1, 64, 96, 320, 512, False),
                                                     (3, 16, 33, 64, 256, True)])
def test_conv_hpp_fwd(B, H, W, cin, cout, relu_in):
    from s3od_amd._lib import lib, stream
    os.environ["S3OD_CONV_HPP"] = "2"
    try:
        g = torch.Generator(device="cuda").manual_seed(H * W + cin)
        x = torch.randn(B, cin, H, W, device="cuda", generator=g).bfloat16()
        w = (torch.randn(cout, cin, 3, 3, device="cuda", generator=g) * (1.0 / (3 * cin ** 0.5))).bfloat16()
        bias = torch.randn(cout, device="cuda", generator=g) * 0.1
        res = torch.randn(B, cout, H, W, device="cuda", generator=g).bfloat16()
        xin = F.relu(x.float()) if relu_in else x.float()
        pre = F.conv2d(xin, w.float(), bias, padding=1)
        ref = F.relu(pre) + res.float()
        out = torch.empty(B, H, W, cout, device="cuda", dtype=torch.bfloat16)
        stats = torch.zeros(2 * cout, device="cuda", dtype=torch.float64)
        wp = w.permute(0, 2, 3, 1).contiguous()                      # [Cout][3][3][Cin]
        lib()("s3od_conv_fwd", BF16, B, H, W, cin, H, W, cout, 3, 3, 1, 1, _nhwc(x), int(relu_in), wp, bias, None, None,
              ACT_RELU, _nhwc(res), None, out, None, stats, None, stream())
        torch.cuda.synchronize()
        _close(out, _nhwc(ref))
        s_ref = pre.sum((0, 2, 3)).double()
        q_ref = (pre * pre).sum((0, 2, 3)).double()
        assert float(((stats[:cout] - s_ref).abs().max() / pre.abs().sum((0, 2, 3)).max()).item()) < 2e-3
        assert float(((stats[cout:] - q_ref).abs().max() / q_ref.abs().max()).item()) < 2e-3
    finally:
        os.environ.pop("S3OD_CONV_HPP", None)


def test_conv_hpp_matches_gemm_path_at_256():
    """Production shape (bs 4 x 256^2 x 256 -> 256, above the tile threshold): the halo kernel (S3OD_CONV_HPP=1)
    vs the implicit GEMM (S3OD_CONV_HPP=0, the default) on the same operands."""
    from s3od_amd._lib import lib, stream
    B, H, W, C = 4, 256, 256, 256
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(B, H, W, C, device="cuda", generator=g).bfloat16()
    wp = (torch.randn(C, 3, 3, C, device="cuda", generator=g) * 0.02).bfloat16()
    bias = torch.randn(C, device="cuda", generator=g) * 0.1
    outs = []
    for knob in ("1", "0"):
        os.environ["S3OD_CONV_HPP"] = knob
        o = torch.empty(B, H, W, C, device="cuda", dtype=torch.bfloat16)
        lib()("s3od_conv_fwd", BF16, B, H, W, C, H, W, C, 3, 3, 1, 1, x, 1, wp, bias, None, None, ACT_NONE, None, None,
              o, None, None, None, stream())
        outs.append(o)
    os.environ.pop("S3OD_CONV_HPP", None)
    torch.cuda.synchronize()
    _close(outs[0], outs[1], 1e-2)
