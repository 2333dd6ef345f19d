"""Where the training step's small PyTorch kernels come from (dev tool, GPU box): one step of configs[2] under
torch.profiler with Python stacks; prints, for every aten op that launches fill / copy kernels, its call count
per step and the innermost s3od_amd frames that issued it.

    python tools/fill_sources.py
"""
import collections
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    from bench import synthetic_batch
    from s3od_amd.model import DPTSegmentation
    from s3od_amd.loss import LossModule, FOCAL_IOU
    from s3od_amd.optim import FusedAdamW, reference_param_groups
    dev = torch.device("cuda", 0)
    m = DPTSegmentation(compute_dtype="bf16").to(dev).train()
    crit = LossModule(FOCAL_IOU, full_mask_lambda=0.1, decay_rate=0.2)
    opt = FusedAdamW(reference_param_groups(m, 1e-5), weight_decay=0.05)
    x, masks = synthetic_batch(16, 1024, 1000, dev)

    def step():
        out = m(x)
        loss, _ = crit(out, {"images": x, "masks": masks}, 0)
        loss.backward()
        opt.step()
        m.zero_grad(set_to_none=False)

    step(); step()
    torch.cuda.synchronize()
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    agg = collections.Counter()
    for ev in prof.events():
        if ev.name in ("aten::fill_", "aten::zero_", "aten::zeros", "aten::copy_", "aten::full", "aten::zeros_like",
                       "aten::add_", "aten::mul_", "aten::sum", "aten::to", "aten::cat", "aten::clone"):
            frames = [f for f in (ev.stack or []) if "s3od_amd" in f or "bench" in f or "tools" in f][:3]
            agg[(ev.name, str(ev.input_shapes)[:60], " <- ".join(frames))] += 1
    for (name, shp, where), n in agg.most_common(40):
        print(f"{n:4d}  {name:16s} {shp:60s} {where}")


if __name__ == "__main__":
    main()
