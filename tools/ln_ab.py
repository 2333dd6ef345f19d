"""LayerNorm backward A/B between library builds on the GPU box (dev tool): s3od_layernorm_ls_bwd and
s3od_layernorm_bwd at the bs-16 1024^2 shape (M = 65616 tokens, D = 768, bf16), builds loaded side by side
(tools/lib_ab.py Lib), alternating calls, HIP-event medians, relative difference of dx / du against the first build.

    python tools/ln_ab.py old_lib/libs3od_hip.so s3od_amd/libs3od_hip.so
"""
import os
import sys
from pathlib import Path

os.environ.setdefault("S3OD_AB", "1")
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd._lib import BF16, NREP, stream  # noqa: E402
from tools.lib_ab import Lib  # noqa: E402


def main():
    libs = [Lib(p) for p in sys.argv[1:]]
    M, D = 65616, 768
    g = torch.Generator(device="cuda").manual_seed(0)
    r = lambda *s: torch.randn(*s, device="cuda", generator=g)
    x = r(M, D); mean = x.mean(1); rstd = 1.0 / (x.var(1, unbiased=False) + 1e-6).sqrt()
    dy = (r(M, D) * 0.1).bfloat16(); w = r(D); dres = r(M, D) * 0.1
    u = r(M, D).bfloat16(); lam = r(D) * 0.1
    st = stream()
    res = []
    for L in libs:
        dx = torch.empty(M, D, device="cuda"); du = torch.empty(M, D, device="cuda", dtype=torch.bfloat16)
        dw, db, dlam, dbias = (torch.zeros(D, device="cuda") for _ in range(4))
        ws = torch.zeros(NREP * 2 * D, device="cuda"); ws2 = torch.zeros(NREP * 2 * D, device="cuda")
        f1 = (lambda L=L, dx=dx, du=du, dw=dw, db=db, dlam=dlam, dbias=dbias, ws=ws, ws2=ws2:
              L("s3od_layernorm_ls_bwd", BF16, dy, x, mean, rstd, w, dres, dx, dw, db, ws, u, lam, du, dlam, dbias, ws2, M, D, st))
        f2 = lambda L=L, dx=dx, dw=dw, db=db, ws=ws: L("s3od_layernorm_bwd", BF16, dy, x, mean, rstd, w, dres, dx, dw, db, ws, M, D, st)
        res.append(dict(fns=(f1, f2), dx=dx, du=du, t=([], [])))
    for _ in range(7):
        for R in res:
            for i, f in enumerate(R["fns"]):
                f(); torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    f()
                e1.record(); torch.cuda.synchronize()
                R["t"][i].append(e0.elapsed_time(e1) / 5)
    outs = []
    for R in res:
        R["fns"][0](); torch.cuda.synchronize(); outs.append((R["dx"].clone(), R["du"].clone()))
    for k, R in enumerate(res):
        meds = [sorted(t)[len(t) // 2] * 1e3 for t in R["t"]]
        rel = [float((a.float() - b.float()).norm() / b.float().norm()) for a, b in zip(outs[k], outs[0])]
        print(f"lib{k}: layernorm_ls_bwd {meds[0]:7.1f} us  layernorm_bwd {meds[1]:7.1f} us  dx / du rel vs lib0 {rel[0]:.1e} / {rel[1]:.1e}", flush=True)


if __name__ == "__main__":
    main()
