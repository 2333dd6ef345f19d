"""Localise a side-stream vs single-stream gradient difference (dev tool): bf16 train step at 256^2 bs 2 under
several stream settings; prints the global rel difference of each vs the single-stream run and the 5 worst params."""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def grads(env):
    from s3od_amd.model import DPTSegmentation
    from s3od_amd.loss import LossModule, FOCAL_IOU
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        torch.manual_seed(0)
        m = DPTSegmentation(compute_dtype=os.environ.get("DIAG_DT", "bf16")).cuda().train()
        m._rope_rescale = 1.0
        crit = LossModule(FOCAL_IOU, full_mask_lambda=0.1, decay_rate=0.2)
        g = torch.Generator(device="cuda").manual_seed(5)
        x = torch.randn(2, 3, 256, 256, device="cuda", generator=g)
        masks = (torch.rand(2, 256, 256, device="cuda", generator=g) > 0.5).float()
        loss, _ = crit(m(x), {"masks": masks}, 0)
        loss.backward()
        torch.cuda.synchronize()
        return {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def cmp(a, b):
    d = t = 0.0
    per = []
    for n in b:
        dd = float((a[n] - b[n]).double().pow(2).sum())
        tt = float(b[n].double().pow(2).sum())
        d += dd; t += tt
        per.append(((dd / max(tt, 1e-30)) ** 0.5, n))
    per.sort(reverse=True)
    return (d / t) ** 0.5, per[:5]


base = grads({"S3OD_BWD_SIDE": "0"})
for name, env in [("single again", {"S3OD_BWD_SIDE": "0"}),
                  ("side (enc+dec)", {"S3OD_BWD_SIDE": "1", "S3OD_DEC_SIDE": "1"}),
                  ("side again", {"S3OD_BWD_SIDE": "1", "S3OD_DEC_SIDE": "1"}),
                  ("enc side only", {"S3OD_BWD_SIDE": "1", "S3OD_DEC_SIDE": "0"}),
                  ("side, no slabs", {"S3OD_BWD_SIDE": "1", "S3OD_WGRAD_SLAB": "0"}),
                  ("single, no slabs", {"S3OD_BWD_SIDE": "0", "S3OD_WGRAD_SLAB": "0"})]:
    tot, worst = cmp(grads(env), base)
    print(f"{name:18s} rel {tot:.3e}  worst: " + ", ".join(f"{n.replace('encoder.model.', '')} {e:.2e}" for e, n in worst), flush=True)
