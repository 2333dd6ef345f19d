"""Library A/B on the GPU box (dev tool): two or more builds of libs3od_hip.so loaded side by side in ONE process
(separate ctypes handles), their entry points called alternately on the same inputs, HIP-event medians per build and
the relative difference of every output against the first build.

    python tools/lib_ab.py attn old_lib/libs3od_hip.so s3od_amd/libs3od_hip.so

A path may carry knobs, "path@S3OD_GEMM_CFG=6,S3OD_X=1": they are set in the environment around every call into that
build (S3OD_AB=1, set here, makes the library read them per call), so one build can be A/B'd against itself.

Workloads: attn (s3od_attn_fwd + s3od_attn_bwd_qkv at the training shape bs 16 N 4101 and the C5 shape bs 4 N 16389);
lin (the ViT linears of the bs-16 1024^2 step with their real epilogues, the 256-channel 3x3 conv; tools/lin_sweep.py shapes).
"""
import ctypes
import os
import sys
from pathlib import Path

os.environ.setdefault("S3OD_AB", "1")
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd import _lib  # noqa: E402
from s3od_amd._lib import BF16, NREP, stream  # noqa: E402
from tools.attn_ab import inputs  # noqa: E402


class Lib(_lib._Lib):
    def __init__(self, spec):
        path, _, knobs = spec.partition("@")
        self.env = dict(kv.split("=", 1) for kv in knobs.split(",") if kv)
        self.lib = ctypes.CDLL(str(Path(path).resolve()))
        self.decls = _lib.parse_header()
        self.fns, self.timers, self.phase, self.cost = {}, {}, None, None
        for name, (ret, types) in self.decls.items():
            fn = getattr(self.lib, name)
            fn.argtypes = [_lib._CT[t] for t in types]
            fn.restype = ctypes.c_char_p if ret.startswith("const char") else ctypes.c_int
            self.fns[name] = (fn, types)

    def __call__(self, *a):
        old = {k: os.environ.get(k) for k in self.env}
        os.environ.update(self.env)
        try:
            return super().__call__(*a)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v


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


def lin(libs, rounds):
    """Each case: a factory taking a library and returning (call, output tensor) on shared inputs."""
    M, D, F = 65616, 768, 3072
    g = torch.Generator(device="cuda").manual_seed(0)
    r = lambda *s, dt=torch.bfloat16: torch.randn(*s, device="cuda", generator=g).to(dt)
    st = stream()
    x768, x3072 = r(M, D), r(M, F)
    wq, bq = r(3 * D, D), r(3 * D, dt=torch.float32)
    wo, bo, so = r(D, D), r(D, dt=torch.float32), r(D, dt=torch.float32)
    wu, bu = r(F, D), r(F, dt=torch.float32)
    wd, bd, sd = r(D, F), r(D, dt=torch.float32), r(D, dt=torch.float32)
    res = r(M, D, dt=torch.float32)
    B, Nt, P = 16, 4101, 4096
    cs, sn = r(P, 64, dt=torch.float32), r(P, 64, dt=torch.float32)
    dy768, dy3072 = r(M, D), r(M, F)
    xc, wc, bc = r(16, 256, 256, 256), r(256, 3, 3, 256), r(256, dt=torch.float32)

    def c_qkv(L):
        q, k, v = (torch.empty(B * 12, Nt, 64, device="cuda", dtype=torch.bfloat16) for _ in range(3))
        return (lambda: L("s3od_qkv_rope_fwd", BF16, B, Nt, P, 12, x768, wq, bq, cs, sn, q, k, v, st)), q

    def c_fwd(w, b, N, K, x, act=0, resf=False, scale=None, pre=True):
        def mk(L):
            out = torch.empty(M, N, device="cuda", dtype=torch.float32 if resf else torch.bfloat16)
            pr = torch.empty(M, N, device="cuda", dtype=torch.bfloat16) if pre else None
            return (lambda: L("s3od_linear_fwd", BF16, M, N, K, x, K, w, b, scale, None, act, res if resf else None, N, None, 0,
                              int(resf), out, N, int(resf), pr, N, 0, 0, 0, st)), out
        return mk

    def c_dgrad(w, N, K, dy, act=0, aux=None):
        def mk(L):
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            return (lambda: L("s3od_linear_dgrad", BF16, M, N, K, dy, K, w, act, aux, N, out, N, 0, 0, 0, 0, None, st)), out
        return mk

    def c_wgrad(Nout, Kin, dy, x):
        """with the caller-owned split-K slab the engine passes (s3od_linear_wgrad_ws): slab partials + reduce"""
        def mk(L):
            dw = torch.zeros(Nout, Kin, device="cuda")
            nb = ctypes.c_long(0)
            L("s3od_linear_wgrad_ws", BF16, Nout, Kin, M, 0, ctypes.addressof(nb))
            slab = torch.empty(max(nb.value, 4) // 4, device="cuda")
            return (lambda: (dw.zero_(), L("s3od_linear_wgrad", BF16, Nout, Kin, M, dy, Nout, x, Kin, dw, 0, slab, nb.value,
                                           st))), dw
        return mk

    def c_conv(L):
        out = torch.empty(16, 256, 256, 256, device="cuda", dtype=torch.bfloat16)
        return (lambda: L("s3od_conv_fwd", BF16, 16, 256, 256, 256, 256, 256, 256, 3, 3, 1, 1, xc, 0, wc, bc, None, None, 0,
                          None, None, out, None, None, None, st)), out

    cases = [("qkv_rope fwd N2304 K768", 2.0 * M * 3 * D * D, c_qkv),
             ("o_proj fwd N768 K768 res f32", 2.0 * M * D * D, c_fwd(wo, bo, D, D, x768, resf=True, scale=so)),
             ("up fwd N3072 K768 GELU+gelu'", 2.0 * M * F * D, c_fwd(wu, bu, F, D, x768, act=5)),
             ("down fwd N768 K3072 res f32", 2.0 * M * D * F, c_fwd(wd, bd, D, F, x3072, resf=True, scale=sd)),
             ("up dgrad N768 K3072", 2.0 * M * D * F, c_dgrad(wu, D, F, dy3072)),
             ("qkv dgrad N768 K2304", 2.0 * M * D * 3 * D, c_dgrad(wq, D, 3 * D, r(M, 3 * D))),
             ("down dgrad N3072 K768 x gelu'", 2.0 * M * D * F, c_dgrad(wd, F, D, dy768, act=6, aux=r(M, F))),
             ("o_proj dgrad N768 K768", 2.0 * M * D * D, c_dgrad(wo, D, D, dy768)),
             ("DPT proj fwd N1024 K768 bias", 2.0 * M * 1024 * D, c_fwd(r(1024, D), r(1024, dt=torch.float32), 1024, D, x768, pre=False)),
             ("DPT proj fwd N512 K768 bias", 2.0 * M * 512 * D, c_fwd(r(512, D), r(512, dt=torch.float32), 512, D, x768, pre=False)),
             ("DPT proj fwd N256 K768 bias", 2.0 * M * 256 * D, c_fwd(r(256, D), r(256, dt=torch.float32), 256, D, x768, pre=False)),
             ("wgrad 3072x768", 2.0 * M * F * D, c_wgrad(F, D, dy3072, x768)),
             ("wgrad 768x3072", 2.0 * M * D * F, c_wgrad(D, F, dy768, x3072)),
             ("conv fwd 256->256 3x3 @256^2 bs16", 2.0 * 16 * 256 * 256 * 256 * 256 * 9, c_conv)]
    for name, fl, mk in cases:
        runs = [mk(L) for L in libs]
        ts = [[] for _ in libs]
        for _ in range(rounds):
            for i, (f, _) in enumerate(runs):
                ts[i].append(timed(f))
        line = f"{name:36s}"
        for i, t in enumerate(ts):
            t = sorted(t)
            line += f" | lib{i} {t[len(t) // 2] * 1e3:8.1f} us ({fl / t[len(t) // 2] / 1e9:6.1f} TF/s)"
        o0 = runs[0][1].float()
        errs = [float((rr[1].float() - o0).norm() / o0.norm()) for rr in runs[1:]]
        print(line, "| rel vs lib0", " ".join(f"{e:.1e}" for e in errs), flush=True)


if __name__ == "__main__":
    what, paths = sys.argv[1], sys.argv[2:]
    libs = [Lib(p) for p in paths]
    rounds = int(os.environ.get("AB_ROUNDS", 5))
    if what == "attn":
        attn(libs, 16, 4101, rounds)
        if not os.environ.get("AB_SMALL"):
            attn(libs, 4, 16389, rounds)
    elif what == "lin":
        lin(libs, rounds)
