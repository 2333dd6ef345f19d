"""Find the first C-ABI call whose outputs differ between a run on fresh memory and a run on reused (warm) caching-
allocator memory (dev tool): every call is followed by a synchronize and a float64 checksum of each tensor argument."""
import os
import sys
from pathlib import Path

import torch

os.environ["S3OD_BWD_SIDE"] = "0"
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from s3od_amd import _lib  # noqa: E402

LOG = []
_orig = _lib._Lib.__call__


def traced(self, name, *args):
    rc = _orig(self, name, *args)
    torch.cuda.synchronize()
    sums = []
    for a in args:
        if isinstance(a, torch.Tensor) and a.is_cuda and a.numel() and a.is_floating_point():
            t = a.detach().double()
            sums.append((float(t.abs().sum()), tuple(a.shape)))
    LOG.append((name, self.phase, sums))
    return rc


_lib._Lib.__call__ = traced


def step():
    from s3od_amd.model import DPTSegmentation
    from s3od_amd.loss import LossModule, FOCAL_IOU
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
    del m


runs = []
for r in range(4):
    LOG.clear()
    step()
    runs.append(list(LOG))
    print(f"run {r}: {len(LOG)} calls", flush=True)
ref = runs[0]
for r in range(1, 4):
    cur = runs[r]
    divs = []
    for i, (a, b) in enumerate(zip(ref, cur)):
        for j, ((sa, sha), (sb, shb)) in enumerate(zip(a[2], b[2])):
            if abs(sa - sb) > 1e-9 * max(abs(sa), 1e-30):
                divs.append((i, a[0], a[1], j, sha, f"{sa:.9e}", f"{sb:.9e}"))
    print(f"run {r} vs run 0: {len(divs)} divergent args; first 25:", flush=True)
    for d in divs[:25]:
        print("   ", d, flush=True)
