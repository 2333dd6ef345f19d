"""Uninitialised-read hunt (dev tool): fill the caching allocator's free blocks with NaN, then run a bf16 (or f32,
DIAG_DT) train step at 256^2 bs 2 and report which outputs / parameter gradients are non-finite or differ from a run
on fresh (zero) memory."""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def poison():
    ts = [torch.full((n,), float("nan"), device="cuda") for n in [1 << 28] * 4 + [1 << 22] * 16 + [1 << 17] * 64 + [1 << 12] * 256]
    torch.cuda.synchronize()
    del ts


def step(tag):
    from s3od_amd.model import DPTSegmentation
    from s3od_amd.loss import LossModule, FOCAL_IOU
    torch.manual_seed(0)
    m = DPTSegmentation(compute_dtype=os.environ.get("DIAG_DT", "bf16")).cuda().train()
    m._rope_rescale = 1.0
    crit = LossModule(FOCAL_IOU, full_mask_lambda=0.1, decay_rate=0.2)
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(2, 3, 256, 256, device="cuda", generator=g)
    masks = (torch.rand(2, 256, 256, device="cuda", generator=g) > 0.5).float()
    out = m(x)
    fo = {k: v.detach().float().clone() for k, v in out.items()}
    loss, _ = crit(out, {"masks": masks}, 0)
    loss.backward()
    torch.cuda.synchronize()
    gr = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
    del m, out, loss
    torch.cuda.synchronize()
    return fo, gr


fo0, g0 = step("fresh")
torch.cuda.empty_cache()
poison()
fo1, g1 = step("poisoned")
for k in fo0:
    a, b = fo1[k], fo0[k]
    print(f"fwd {k}: nonfinite {int((~torch.isfinite(a)).sum())}  rel {float((a - b).norm() / b.norm()):.3e}", flush=True)
bad = [(n, int((~torch.isfinite(g1[n])).sum()), g1[n].numel()) for n in g0 if not torch.isfinite(g1[n]).all()]
print(f"grads with non-finite values: {len(bad)} of {len(g0)}", flush=True)
for n, c, t in bad[:40]:
    print(f"   {n}: {c} / {t}", flush=True)
diff = sorted(((float((g1[n] - g0[n]).norm() / max(float(g0[n].norm()), 1e-30)), n) for n in g0), reverse=True)[:10]
print("largest rel diffs:", ", ".join(f"{n} {e:.2e}" for e, n in diff), flush=True)
