"""Library A/B on the GPU box (dev tool): two or more builds of libs3od_hip.so loaded side by side in ONE process
(separate ctypes handles), their entry points called alternately on the same inputs, HIP-event medians per build and
the relative difference of every output against the first build.

    python tools/lib_ab.py attn old_lib/libs3od_hip.so s3od_amd/libs3od_hip.so

Workloads: attn (s3od_attn_fwd + s3od_attn_bwd_qkv at the training shape bs 16 N 4101 and the C5 shape bs 4 N 16389).
"""
import ctypes
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd import _lib  # noqa: E402
from s3od_amd._lib import BF16, NREP, stream  # noqa: E402
from tools.attn_ab import inputs  # noqa: E402


class Lib(_lib._Lib):
    def __init__(self, path):
        self.lib = ctypes.CDLL(str(Path(path).resolve()))
        self.decls = _lib.parse_header()
        self.fns, self.timers, self.phase, self.cost = {}, {}, None, None
        for name, (ret, types) in self.decls.items():
            fn = getattr(self.lib, name)
            fn.argtypes = [_lib._CT[t] for t in types]
            fn.restype = ctypes.c_char_p if ret.startswith("const char") else ctypes.c_int
            self.fns[name] = (fn, types)


def timed(fn, n=3):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def attn(libs, B, N, rounds, H=12):
    q, k, v, do, cs, sn, P = inputs(B, N, H)
    st = stream()
    res = []
    for L in libs:
        o = torch.empty(B, N, H * 64, device="cuda", dtype=torch.bfloat16)
        lse = torch.empty(B * H, N, device="cuda")
        delta = torch.empty(B * H, N, device="cuda")
        dqkv = torch.empty(B * N, 3 * H * 64, device="cuda", dtype=torch.bfloat16)
        dbq, dbv = torch.zeros(H * 64, device="cuda"), torch.zeros(H * 64, device="cuda")
        ws = torch.zeros(NREP * 2 * H * 64, device="cuda")
        fwd = (lambda L=L, o=o, lse=lse: L("s3od_attn_fwd", BF16, q, k, v, o, lse, B, H, N, st))
        bwd = (lambda L=L, o=o, lse=lse, delta=delta, dqkv=dqkv, dbq=dbq, dbv=dbv, ws=ws:
               L("s3od_attn_bwd_qkv", BF16, q, k, v, o, do, lse, delta, cs, sn, P, dqkv, dbq, dbv, ws, B, H, N, st))
        fwd(); bwd(); torch.cuda.synchronize()
        outs = [t.clone() for t in (o, lse, dqkv, dbq, dbv)]
        res.append({"fwd": fwd, "bwd": bwd, "outs": outs, "t": {"fwd": [], "bwd": []}})
    for _ in range(rounds):
        for r in res:
            for nm in ("fwd", "bwd"):
                r["t"][nm].append(timed(r[nm]))
    fl = 4.0 * B * H * N * N * 64
    for i, r in enumerate(res):
        tf, tb = sorted(r["t"]["fwd"]), sorted(r["t"]["bwd"])
        print(f"B{B} N{N} lib{i}: fwd med {tf[len(tf) // 2] * 1e3:8.1f} us min {tf[0] * 1e3:8.1f} ({fl / tf[0] / 1e9:6.1f} TF/s) | "
              f"bwd med {tb[len(tb) // 2] * 1e3:8.1f} us min {tb[0] * 1e3:8.1f} ({2 * fl / tb[0] / 1e9:6.1f} TF/s alg)", flush=True)
        if i:
            errs = [f"{nm} {float((a.float() - b.float()).norm() / b.float().norm()):.2e}"
                    for nm, a, b in zip(("o", "lse", "dqkv", "dbq", "dbv"), r["outs"], res[0]["outs"])]
            print(f"   vs lib0: " + "  ".join(errs), "| finite", bool(torch.isfinite(r["outs"][2].float()).all()), flush=True)


if __name__ == "__main__":
    what, paths = sys.argv[1], sys.argv[2:]
    libs = [Lib(p) for p in paths]
    rounds = int(os.environ.get("AB_ROUNDS", 5))
    if what == "attn":
        attn(libs, 16, 4101, rounds)
        if not os.environ.get("AB_SMALL"):
            attn(libs, 4, 16389, rounds)
