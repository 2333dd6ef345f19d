"""Block timeline of the ping-pong GEMM kernel (dev tool, GPU box; needs `make timeline`):

    python tools/pp_timeline.py [tl_lib/libs3od_hip.so]

Each block of one s3od_linear_fwd launch records [start, main loop done, epilogue done] (s_memrealtime, 10 ns ticks)
and its CU (HW_ID / XCC_ID).  Printed per case: the launch span, the per-block main-loop and epilogue durations, how
the blocks fall into rounds, and the idle gap on a CU between one block's end and the next block's start."""
import ctypes
import os
import sys
from collections import defaultdict
from pathlib import Path

os.environ.setdefault("S3OD_AB", "1")
os.environ.setdefault("S3OD_GEMM_CFG", "5")      # every case on the ping-pong kernel (plain K=768 defaults to 128x128)
import torch  # noqa: E402

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from tools.lib_ab import Lib  # noqa: E402
from s3od_amd._lib import BF16, stream  # noqa: E402


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))]


def run(L, tl, name, M, N, K, act=0, resf=False):
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    b = torch.randn(N, device="cuda", generator=g)
    res = torch.randn(M, N, device="cuda", generator=g) if resf else None
    out = torch.empty(M, N, device="cuda", dtype=torch.float32 if resf else torch.bfloat16)
    pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    st = stream()
    f = lambda: L("s3od_linear_fwd", BF16, M, N, K, x, K, w, b if act or resf else None, None, None, act, res, N, None, 0,
                  int(resf), out, N, int(resf), pre if act == 5 else None, N, 0, 0, 0, st)
    f(); f()
    torch.cuda.synchronize()
    tl.zero_()
    f()
    torch.cuda.synchronize()
    t = tl.view(-1, 8).cpu()
    t = t[t[:, 0] != 0]
    t0, t1, t2, hw, s0, e0, s1 = (t[:, i].tolist() for i in range(7))
    base = min(t0)
    us = lambda v: (v - base) / 100.0
    main = [(b_ - a) / 100.0 for a, b_ in zip(t0, t1)]
    epi = [(c - b_) / 100.0 for b_, c in zip(t1, t2)]
    span = (max(t2) - base) / 100.0
    print(f"\n{name}: M{M} N{N} K{K}  {len(t0)} blocks, span {span:.1f} us", flush=True)
    print(f"   main loop  us: p10 {pct(main, .1):6.2f} med {pct(main, .5):6.2f} p90 {pct(main, .9):6.2f} max {max(main):6.2f}")
    print(f"   epilogue   us: p10 {pct(epi, .1):6.2f} med {pct(epi, .5):6.2f} p90 {pct(epi, .9):6.2f} max {max(epi):6.2f}")
    for nm, a_, b_ in (("stage h0", t1, s0), ("epi h0", s0, e0), ("stage h1", e0, s1), ("epi h1", s1, t2)):
        d = [(y - x) / 100.0 for x, y in zip(a_, b_)]
        print(f"     {nm:9s} us: p10 {pct(d, .1):6.2f} med {pct(d, .5):6.2f} p90 {pct(d, .9):6.2f}")
    cu = defaultdict(list)
    for a, b_, c, h in zip(t0, t1, t2, hw):
        xcc, hid = h >> 32, h & 0xffffffff
        key = (xcc & 0xf, (hid >> 13) & 0x7, (hid >> 12) & 1, (hid >> 8) & 0xf)
        cu[key].append((a, b_, c))
    gaps, nper = [], []
    for k, v in cu.items():
        v.sort()
        nper.append(len(v))
        gaps += [(v[i + 1][0] - v[i][2]) / 100.0 for i in range(len(v) - 1)]
    print(f"   CUs used {len(cu)}, blocks per CU min {min(nper)} max {max(nper)}")
    if gaps:
        print(f"   gap end->next start us: p10 {pct(gaps, .1):6.2f} med {pct(gaps, .5):6.2f} p90 {pct(gaps, .9):6.2f} max {max(gaps):6.2f}")
    # start-time histogram in 5 us bins (how lock-stepped the rounds are)
    hist = defaultdict(int)
    for a in t0:
        hist[int(us(a) // 5)] += 1
    print("   starts per 5 us bin:", " ".join(f"{k * 5}:{hist[k]}" for k in sorted(hist)))
    ends = defaultdict(int)
    for b_ in t1:
        ends[int(us(b_) // 5)] += 1
    print("   main-loop ends per 5 us bin:", " ".join(f"{k * 5}:{ends[k]}" for k in sorted(ends)))


if __name__ == "__main__":
    L = Lib(sys.argv[1] if len(sys.argv) > 1 else "tl_lib/libs3od_hip.so")
    tl = torch.zeros(8 * 16384, dtype=torch.int64, device="cuda")
    fn = L.lib.s3od_dbg_timeline
    fn.argtypes = [ctypes.c_void_p]
    assert fn(ctypes.c_void_p(tl.data_ptr())) == 0
    run(L, tl, "plain bf16", 65536, 3072, 768)
    os.environ["S3OD_PP_FLAGS"] = "2"
    run(L, tl, "plain bf16, bare store loop", 65536, 3072, 768)
    os.environ["S3OD_PP_FLAGS"] = "0"
    run(L, tl, "up GELU+gelu'", 65536, 3072, 768, act=5)
    run(L, tl, "down f32 res", 65536, 768, 3072, resf=True)
    run(L, tl, "plain bf16 K3072", 65536, 3072, 3072)
