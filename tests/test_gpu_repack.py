"""GPU: s3od_repack_multi, the per-step cast / re-layout of every fp32 master weight into the kernel layouts
(engine.py _build_packs), against torch re-layouts of the same tensors -- bit-identical (a plain round-to-nearest
cast).  Covers the vectorised plain-cast path (linears: KHW 1, mode 0, aligned), its scalar fallback (source or
destination not 16-B / 8-B aligned, a ragged chunk end), the conv layout [O][KH][KW][I] (mode 0), the transposed,
tap-reversed data-gradient layout with a column offset inside a wider destination (mode 1), the ConvTranspose
sub-pixel layout (mode 2), and the fp32 copies of the bias vectors."""
import pytest
import torch

pytestmark = pytest.mark.gpu

CHUNK = 16384


def _run(dtype, ents):
    from s3od_amd._lib import lib, stream
    rows, ct, co = [], [], []
    for t, (src, dst, off, O, I, KHW, mode, ld) in enumerate(ents):
        rows.append([src.data_ptr(), dst.data_ptr(), O, I, KHW, off, mode, ld])
        for o in range(0, O * I * KHW, CHUNK):
            ct.append(t); co.append(o)
    tab = torch.tensor(rows, dtype=torch.int64, device="cuda")
    ctt = torch.tensor(ct, dtype=torch.int32, device="cuda")
    cot = torch.tensor(co, dtype=torch.int64, device="cuda")
    lib()("s3od_repack_multi", dtype, tab, ctt, cot, len(ct), CHUNK, stream())
    torch.cuda.synchronize()


def test_repack_multi_layouts_bit_identical():
    from s3od_amd._lib import BF16, F32
    g = torch.Generator(device="cuda").manual_seed(5)
    r = lambda *s: torch.randn(*s, device="cuda", generator=g)
    lin = r(3072, 768)                                   # plain cast, aligned, several chunks
    flat = r(1 + 768 * 40 + 3)
    lin_u = flat[1:1 + 768 * 40].view(40, 768)           # source 4 B past a 16-B boundary: scalar path
    conv = r(256, 128, 3, 3)                             # mode 0 conv layout
    dg = r(64, 96, 3, 3)                                 # mode 1: [I][3][3][ld], column offset 32, ld 128
    ct_w = r(128, 64, 4, 4)                              # mode 2 (ConvT weight [Cin][Cout][4][4] as O=128, I=64)
    d_lin = torch.empty(3072, 768, dtype=torch.bfloat16, device="cuda")
    d_big = torch.zeros(1 + 40 * 768, dtype=torch.bfloat16, device="cuda")   # destination offset 1: unaligned
    d_conv = torch.empty(256, 3, 3, 128, dtype=torch.bfloat16, device="cuda")
    d_dg = torch.zeros(96, 3, 3, 128, dtype=torch.bfloat16, device="cuda")
    d_ct = torch.empty(64, 4, 4, 128, dtype=torch.bfloat16, device="cuda")
    _run(BF16, [(lin, d_lin, 0, 3072, 768, 1, 0, 0), (lin_u, d_big, 1, 40, 768, 1, 0, 0),
                (conv, d_conv, 0, 256, 128, 9, 0, 0), (dg, d_dg, 32, 64, 96, 9, 1, 128),
                (ct_w, d_ct, 0, 128, 64, 16, 2, 128)])
    assert torch.equal(d_lin, lin.bfloat16())
    assert torch.equal(d_big[1:].view(40, 768), lin_u.bfloat16()) and float(d_big[0]) == 0.0
    assert torch.equal(d_conv, conv.permute(0, 2, 3, 1).bfloat16())
    ref_dg = torch.zeros(96, 3, 3, 128, dtype=torch.bfloat16, device="cuda")
    ref_dg[..., 32:96] = dg.flip(2, 3).permute(1, 2, 3, 0).bfloat16()
    assert torch.equal(d_dg, ref_dg)
    assert torch.equal(d_ct, ct_w.permute(1, 2, 3, 0).bfloat16())
    # fp32 copies (bias vectors): aligned and at an odd offset
    b1, b2 = r(768), r(33)
    d32 = torch.full((1 + 768 + 33,), float("nan"), device="cuda")
    _run(F32, [(b1, d32, 0, 768, 1, 1, 0, 0), (b2, d32, 768, 33, 1, 1, 0, 0)])
    assert torch.equal(d32[:768], b1) and torch.equal(d32[768:801], b2)
