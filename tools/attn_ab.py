"""Attention A/B on the GPU box (dev tool): alternating rounds of two (or more) settings of a knob in ONE process,
HIP-event timing of s3od_attn_fwd and s3od_attn_bwd_qkv at the training shape (bs 16, N 4101) and the C5 shape
(bs 4, N 16389), plus the relative difference of every output against the first setting.

    python tools/attn_ab.py S3OD_ATTN_BWD_PP 1 0
"""
import os
os.environ.setdefault("S3OD_AB", "1")   # knobs toggled per call (csrc/common.hpp S3OD_KNOB)
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd._lib import lib, stream, BF16, NREP  # noqa: E402


def inputs(B, N, H=12, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    q = (torch.randn(B * H, N, 64, device="cuda", generator=g) * 0.18).bfloat16()   # pre-scaled q (log2e / 8 folded in)
    k = torch.randn(B * H, N, 64, device="cuda", generator=g).bfloat16()
    v = torch.randn(B * H, N, 64, device="cuda", generator=g).bfloat16()
    do = (torch.randn(B, N, H * 64, device="cuda", generator=g) * 0.1).bfloat16()
    P = N - 5
    cs = torch.rand(P, 64, device="cuda", generator=g)
    sn = torch.rand(P, 64, device="cuda", generator=g)
    return q, k, v, do, cs, sn, P


def run(B, N, knob, vals, rounds, H=12):
    q, k, v, do, cs, sn, P = inputs(B, N, H)
    o = torch.empty(B, N, H * 64, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B * H, N, device="cuda")
    delta = torch.empty(B * H, N, device="cuda")
    dqkv = torch.empty(B * N, 3 * H * 64, device="cuda", dtype=torch.bfloat16)
    dbq = torch.zeros(H * 64, device="cuda")
    dbv = torch.zeros(H * 64, device="cuda")
    ws = torch.zeros(NREP * 2 * H * 64, device="cuda")
    L, st = lib(), stream()
    fwd = lambda: L("s3od_attn_fwd", BF16, q, k, v, o, lse, B, H, N, st)
    bwd = lambda: L("s3od_attn_bwd_qkv", BF16, q, k, v, o, do, lse, delta, cs, sn, P, dqkv, dbq, dbv, ws, B, H, N, st)
    times = {x: {"fwd": [], "bwd": []} for x in vals}
    outs = {}
    for r in range(rounds):
        for x in vals:
            os.environ[knob] = x
            for name, fn in (("fwd", fwd), ("bwd", bwd)):
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                n = 3
                for _ in range(n):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[x][name].append(e0.elapsed_time(e1) / n)
            if r == 0:
                dbq.zero_(); dbv.zero_()
                fwd(); bwd()
                torch.cuda.synchronize()
                outs[x] = (o.clone(), lse.clone(), dqkv.clone(), dbq.clone(), dbv.clone())
    os.environ.pop(knob, None)
    fl = 4.0 * B * H * N * N * 64
    for x in vals:
        tf, tb = sorted(times[x]["fwd"]), sorted(times[x]["bwd"])
        print(f"B{B} N{N} {knob}={x}: fwd med {tf[len(tf) // 2] * 1e3:8.1f} us min {tf[0] * 1e3:8.1f} ({fl / tf[0] / 1e9:6.1f} TF/s) | "
              f"bwd med {tb[len(tb) // 2] * 1e3:8.1f} us min {tb[0] * 1e3:8.1f} ({2 * fl / tb[0] / 1e9:6.1f} TF/s alg)", flush=True)
    ref = outs[vals[0]]
    for x in vals[1:]:
        errs = []
        for nm, a, b in zip(("o", "lse", "dqkv", "dbq", "dbv"), outs[x], ref):
            a, b = a.float(), b.float()
            errs.append(f"{nm} {float((a - b).norm() / b.norm()):.2e}")
        print(f"   vs {knob}={vals[0]}: " + "  ".join(errs), "| finite", bool(torch.isfinite(outs[x][2].float()).all()), flush=True)


if __name__ == "__main__":
    knob, vals = sys.argv[1], sys.argv[2:]
    rounds = int(os.environ.get("AB_ROUNDS", 5))
    run(16, 4101, knob, vals, rounds)
    if not os.environ.get("AB_SMALL"):
        run(4, 16389, knob, vals, rounds)
